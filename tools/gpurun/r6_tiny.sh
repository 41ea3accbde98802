#!/bin/bash
# round 6: the one-launch path for tiny keyed batches (k_ed_tiny): parity (tiny tests, the types
# layer, Ed25519 and service suites, the C1 config test), C1 latency with and without it, and a
# kernel trace of C1's Certificate::verify
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tiny
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_types.py tests/test_gpu_ed25519.py tests/test_gpu_service.py "tests/test_gpu_baseline_configs.py::test_c1_certificate_n4_and_batch_1024" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python3 tools/c1_times.py 1000 > $O/c1_tiny_$r.json 2> $O/c1_tiny_$r.err || exit $?
  timeout -k 10 200 python3 tools/c1_times.py 1000 4096 > $O/c1_msm_$r.json 2> $O/c1_msm_$r.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c1trace -o run --output-format csv -- python3 tools/c1_driver.py 300 > $O/c1trace.log 2>&1 || exit $?
echo ALLDONE
