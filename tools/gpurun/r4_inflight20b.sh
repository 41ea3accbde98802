#!/bin/bash
# round 4: the 20-step headline at 16-24 batches in flight and 4-16 hardware queues (second half of the sweep in profiles/round4_inflight20_sweep.jsonl)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i2
mkdir -p $O
for k in 20 24; do
  for q in 16 24; do
    NWV_BENCH_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --headline-only --inflight $k > $O/k${k}_q${q}.json 2> $O/k${k}_q${q}.err || exit $?
  done
done
echo ALLDONE
