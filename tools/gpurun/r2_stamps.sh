#!/bin/bash
# tail phase stamps (NWV_TAIL_STAMPS) at 65,536 and 1,024, default tail shape and 1-bucket lanes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
for n in 65536 1024; do
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 tools/profile_driver.py --n $n --reps 4 --mode 1 > $O/st_$n.out 2> $O/st_$n.err || exit $?
NWV_MSM_TAIL_M4=1000000000 NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 tools/profile_driver.py --n $n --reps 4 --mode 1 > $O/st1_$n.out 2> $O/st1_$n.err || exit $?
done
echo ALLDONE
