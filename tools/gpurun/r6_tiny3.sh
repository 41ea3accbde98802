#!/bin/bash
# round 6: the tiny path comparing [8] R (on the rows of wave 0) with [8]([s]B - [k]A): parity,
# C1 latency, phase stamps of k_ed_tiny
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6tiny3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_types.py tests/test_gpu_service.py "tests/test_gpu_baseline_configs.py::test_c1_certificate_n4_and_batch_1024" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python3 tools/c1_times.py 1000 > $O/c1_tiny_$r.json 2> $O/c1_tiny_$r.err || exit $?
done
NWV_TINY_STAMPS=1 timeout -k 10 200 python3 tools/c1_driver.py 50 > $O/stamps.log 2> $O/stamps.txt || exit $?
echo ALLDONE
