#!/bin/bash
# tail bucket-piece join on quads in the quad path:
# GPU suite, the MSM suites under the lane-local tail path, kernel times, 1K latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/qj_pytest.log 2>&1 || exit $?
NWV_TAIL_QUAD_MAX_N=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py -x -q --timeout 200 --timeout-method thread > $O/qj_pytest_lane.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 64 1024 4096 > $O/qj_k.jsonl 2> $O/qj_k.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/qj_lat.json 2> $O/qj_lat.err || exit $?
echo ALLDONE
