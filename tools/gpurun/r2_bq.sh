#!/bin/bash
# quad-lane bucket sums for small batches: GPU suite, per-kernel times with and without, 1K latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2q_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 16384 > $O/r2q_kernels.jsonl 2> $O/r2q_kernels.err || exit $?
NWV_BUCKET_QUAD_MAX_N=0 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 16384 > $O/r2q_kernels_lane.jsonl 2> $O/r2q_kernels_lane.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2q_latgraph.json 2> $O/r2q_latgraph.err || exit $?
echo ALLDONE
