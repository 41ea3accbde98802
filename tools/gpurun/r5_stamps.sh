#!/bin/bash
# round 5: phase stamps of k_msm_tail (NWV_TAIL_STAMPS) at 1,024 and 65,536 signatures
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5stamps
mkdir -p $O
NWV_TAIL_STAMPS=1 timeout -k 10 300 python -u tools/tail_sweep.py 1024 65536 > $O/sweep.json 2> $O/stamps.txt || exit $?
echo ALLDONE
