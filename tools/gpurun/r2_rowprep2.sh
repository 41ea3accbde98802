#!/bin/bash
# split prep (hash / decompression as separate kernels), row mode on and off: which role is the
# small-batch latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
NWV_SWEEP_FLAGS=4 timeout -k 10 120 python3 -u tools/tail_sweep.py 64 64 1024 4096 > $O/r2r2_split_row.jsonl 2> $O/r2r2_split_row.err || exit $?
NWV_SWEEP_FLAGS=4 NWV_PREP_ROW_MAX=0 timeout -k 10 120 python3 -u tools/tail_sweep.py 64 64 1024 4096 > $O/r2r2_split_lane.jsonl 2> $O/r2r2_split_lane.err || exit $?
echo ALLDONE
