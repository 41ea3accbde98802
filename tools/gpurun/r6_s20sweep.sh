#!/bin/bash
# round 6: the driver's 20-step headline at 8-16 batches in flight and prep-chain depths 2 / 3
# (NWV_STAGE_CHAIN), two rounds, alternating; headline only
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s20
mkdir -p $O
for r in 1 2; do
  for i in 8 10 12 16; do
    for c in 2 3; do
      NWV_STAGE_CHAIN=$c timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --headline-only --inflight $i --steady-steps 0 --single-steps 1 > $O/s20_i${i}_c${c}_$r.json 2>> $O/err.log || exit $?
      echo "i=$i c=$c r=$r $(python3 -c "import json; print(json.loads(open('$O/s20_i${i}_c${c}_$r.json').read().strip().splitlines()[-1])['value'])")" >> $O/summary.txt
    done
  done
done
echo ALLDONE
