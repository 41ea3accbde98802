#!/bin/bash
# round 6: the MSM tail's waves at raised issue priority (s_setprio 3, build -DNWV_TAIL_PRIO=3 as
# lib/libnwv_exp.so) against the kept build: the driver's 20-step headline, alternating, 4 rounds
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6prio
mkdir -p $O
for r in 1 2 3 4; do
  for v in base prio; do
    if [ $v = prio ]; then L=libnwv_exp.so; else L=libnwv.so; fi
    NWV_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --headline-only --steady-steps 64 --single-steps 20 > $O/${v}_$r.json 2>> $O/err.log || exit $?
    echo "$v r=$r $(python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d.get('steady_state',{}).get('sigs_per_s'), d.get('single_stream',{}).get('ms_per_step'))")" >> $O/summary.txt
  done
done
echo ALLDONE
