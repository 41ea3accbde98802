#!/bin/bash
# k_msm_prep row mode (decompression chain on 16-lane rows for small batches): GPU suite,
# kernel times with and without it, 1K latency, single-signature / certificate latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2r_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 4 64 256 1024 2048 4096 > $O/r2r_kernels.jsonl 2> $O/r2r_kernels.err || exit $?
NWV_PREP_ROW_MAX=0 timeout -k 10 120 python3 -u tools/tail_sweep.py 4 64 256 1024 2048 4096 > $O/r2r_kernels_lane.jsonl 2> $O/r2r_kernels_lane.err || exit $?
NWV_PREP_ROW_MAX=100000 timeout -k 10 120 python3 -u tools/tail_sweep.py 4096 8192 16384 > $O/r2r_kernels_rowbig.jsonl 2> $O/r2r_kernels_rowbig.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2r_latgraph.json 2> $O/r2r_latgraph.err || exit $?
timeout -k 10 120 python3 -u tools/single_verify_lat.py > $O/r2r_single.json 2> $O/r2r_single.err || exit $?
echo ALLDONE
