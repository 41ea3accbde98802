#!/bin/bash
# A/B: this tree against _prev/ (the previous commit's build) on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
A="--no-configs --no-cpu-baseline --latency-reps 100 --h2h-seconds 0 --single-steps 20"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/ab_cur$r.json 2> $O/ab_cur$r.err || exit $?
  (cd _prev && timeout -k 10 200 python3 bench.py $A) > $O/ab_prev$r.json 2> $O/ab_prev$r.err || exit $?
done
echo ALLDONE
