#!/bin/bash
# round 4: the driver's 20-step headline (bench.py --steps 20 --warmup 5) at several batch-in-flight
# depths: the data behind bench.py's --inflight default for short timed regions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
for k in 4 6 8 12 16; do
  for rep in 1 2; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --headline-only --inflight $k > $O/k${k}_r${rep}.json 2> $O/k${k}_r${rep}.err || exit $?
  done
done
echo ALLDONE
