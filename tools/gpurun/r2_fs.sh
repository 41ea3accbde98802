#!/bin/bash
# quad-tree final sum in k_msm_tail: GPU suite, per-kernel times, stamps, 1K latency, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2f_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 65536 > $O/r2f_kernels.jsonl 2> $O/r2f_kernels.err || exit $?
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 > $O/r2f_stamps1k.jsonl 2> $O/r2f_stamps1k.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2f_latgraph.json 2> $O/r2f_latgraph.err || exit $?
timeout -k 10 400 python3 -u bench.py > $O/r2f_bench.json 2> $O/r2f_bench.err || exit $?
echo ALLDONE
