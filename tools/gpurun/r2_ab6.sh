#!/bin/bash
# throughput A/B: this build (default tail shape; M = 1 everywhere) against _prev/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
A="--no-configs --no-cpu-baseline --latency-reps 20 --h2h-seconds 0"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/ab6_cur$r.json 2> /dev/null || exit $?
  NWV_MSM_TAIL_M4=1000000000 timeout -k 10 200 python3 bench.py $A > $O/ab6_m1$r.json 2> /dev/null || exit $?
  (cd _prev && timeout -k 10 200 python3 bench.py $A) > $O/ab6_prev$r.json 2> /dev/null || exit $?
done
echo ALLDONE
