#!/bin/bash
# round 5 experiment, second pass: the 20-step headline three times per chain depth, k interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5chain2
mkdir -p $O
for r in 1 2 3; do
  for k in 0 3 4 6 8; do
    NWV_STAGE_CHAIN=$k timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/k${k}_s20_$r.json 2>> $O/err || exit $?
  done
done
echo ALLDONE
