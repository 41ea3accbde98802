#!/bin/bash
# round 3: the headline at the driver's step count (20 / 5) with the in-flight batches' preps
# chained in a ring (nwv_staged_follow, bench --chain D), D = 0 repeated for the box's noise
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for d in 0 1 2 3 4 6 0; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --chain $d --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 >> $O/r3c_s20.jsonl 2>> $O/r3c_s20.err || exit $?
done
for d in 0 1 2; do
  timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --chain $d --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 >> $O/r3c_s192.jsonl 2>> $O/r3c_s192.err || exit $?
done
echo ALLDONE
