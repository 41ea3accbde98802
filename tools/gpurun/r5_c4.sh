#!/bin/bash
# round 5: C4 (65,536 x 512 B, 1 % adversarial, exact bad set) host-to-host time, its host-side
# timeline (NWV_HOST_TRACE) and its kernel trace, at the current sources; tag = $1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-c4}
O=gpurun_out/r5$T
mkdir -p $O
NWV_HOST_TRACE=1 timeout -k 10 300 python -u tools/c4_times.py > $O/c4.json 2> $O/c4_trace.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c4 -- python3 -u tools/c4_times.py > $O/c4_prof.json 2> $O/c4_prof.err || exit $?
echo ALLDONE
