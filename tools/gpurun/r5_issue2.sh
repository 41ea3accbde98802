#!/bin/bash
# round 5 experiment: the 20-step region with and without the per-replay seed copy
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5issue2
mkdir -p $O
export GPU_MAX_HW_QUEUES=16
for i in 1 2; do
timeout -k 10 200 python -u tools/run_timing.py 20 5 > $O/seed$i.json 2>> $O/err || exit $?
NWV_EXP_NOSEED=1 timeout -k 10 200 python -u tools/run_timing.py 20 5 > $O/noseed$i.json 2>> $O/err || exit $?
done
NWV_EXP_NOSEED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o b -- python3 tools/run_timing.py 20 5 > $O/noseed_prof.json 2>> $O/err || exit $?
echo ALLDONE
