#!/bin/bash
# round 3: the headline at the driver's step count (20 / 5) against the start offset between the
# in-flight batches' first timed steps (nwv_staged_delay), with 0 repeated for the box's noise
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for d in 0 10 20 30 45 60 90 0; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --stagger-us $d --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 >> $O/r3s_s20.jsonl 2>> $O/r3s_s20.err || exit $?
done
for d in 0 30; do
  timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --stagger-us $d --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 >> $O/r3s_s192.jsonl 2>> $O/r3s_s192.err || exit $?
done
echo ALLDONE
