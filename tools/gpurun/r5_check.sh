#!/bin/bash
# round 5: the MSM / Ed25519 GPU tests, the BLS ring test, the latency-side probe and tail stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py tests/test_gpu_baseline_configs.py "tests/test_gpu_bls.py::test_ring_wraps_under_concurrent_verifies_and_aggregates" "tests/test_gpu_bls.py::test_verify_many_sharded_over_devices" "tests/test_gpu_types_bls.py::test_bls_service_concurrent_submitters" tests/test_gpu_service.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tail_probe.py > $O/probe.json 2> $O/probe.err || exit $?
NWV_TAIL_STAMPS=1 timeout -k 10 300 python -u tools/tail_sweep.py 1024 65536 > $O/sweep.json 2> $O/stamps.txt || exit $?
echo ALLDONE
