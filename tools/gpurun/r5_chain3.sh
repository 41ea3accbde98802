#!/bin/bash
# round 5 experiment, third pass: chain depth x batches in flight on the 20-step headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5chain3
mkdir -p $O
for r in 1 2; do
  for cfg in "0 12" "3 12" "3 8" "3 16" "2 12" "4 16"; do
    set -- $cfg
    NWV_STAGE_CHAIN=$1 timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline --inflight $2 > $O/k$1_f$2_$r.json 2>> $O/err || exit $?
  done
done
echo ALLDONE
