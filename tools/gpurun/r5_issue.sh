#!/bin/bash
# round 5: host-side duration of each graph-replay call in the 20-step timed region
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5issue
mkdir -p $O
timeout -k 10 200 python -u tools/run_timing.py 20 5 > $O/t20.json 2> $O/t20.err || exit $?
timeout -k 10 200 python -u tools/run_timing.py 20 5 > $O/t20b.json 2>> $O/t20.err || exit $?
echo ALLDONE
