#!/bin/bash
# quad bucket sums owning whole buckets (no fixup pass): GPU suite, kernel times, 1K latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2w_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 > $O/r2w_kernels.jsonl 2> $O/r2w_kernels.err || exit $?
NWV_MSM_SEG=12 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 > $O/r2w_kernels12.jsonl 2> $O/r2w_kernels12.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2w_latgraph.json 2> $O/r2w_latgraph.err || exit $?
echo ALLDONE
