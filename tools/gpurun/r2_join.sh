#!/bin/bash
# bucket-piece join folded into k_msm_tail (no k_msm_fixup launch): GPU suite, kernel times,
# 1K latency, headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2j_pytest.log 2>&1 || exit $?
timeout -k 10 180 python3 -u tools/tail_sweep.py 64 1024 4096 65536 > $O/r2j_kernels.jsonl 2> $O/r2j_kernels.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2j_latgraph.json 2> $O/r2j_latgraph.err || exit $?
timeout -k 10 120 python3 -u tools/single_verify_lat.py > $O/r2j_single.json 2> $O/r2j_single.err || exit $?
timeout -k 10 400 python3 -u bench.py > $O/r2j_bench.json 2> $O/r2j_bench.err || exit $?
echo ALLDONE
