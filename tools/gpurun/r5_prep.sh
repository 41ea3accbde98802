#!/bin/bash
# round 5: the decompression alone (split prep) at several sizes, row form vs lane-local
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5prep
mkdir -p $O
NWV_SWEEP_FLAGS=4 timeout -k 10 120 python -u tools/tail_sweep.py 16 64 256 1024 2048 > $O/rows.json 2> $O/rows.err || exit $?
NWV_SWEEP_FLAGS=516 timeout -k 10 120 python -u tools/tail_sweep.py 16 64 256 1024 2048 > $O/lanes.json 2> $O/lanes.err || exit $?
echo ALLDONE
