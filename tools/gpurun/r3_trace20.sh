#!/bin/bash
# kernel trace of the headline at the driver's step count (--steps 20 --warmup 5) and at 96 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r3b_tr20 -o t -- python3 bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 > $O/r3b_tr20.json 2> $O/r3b_tr20.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r3b_tr96 -o t -- python3 bench.py --steps 96 --warmup 24 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 > $O/r3b_tr96.json 2> $O/r3b_tr96.err || exit $?
echo ALLDONE
