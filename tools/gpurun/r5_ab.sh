#!/bin/bash
# round 5: same-box A/B of two in-tree builds (NWV_LIB=libnwv_old.so vs libnwv.so), alternating:
# 20- and 192-step headline, C1 / 1K per-call latency, C4, tail sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5ab
mkdir -p $O
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export NWV_LIB=libnwv_old.so; else export NWV_LIB=libnwv.so; fi
    timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/${v}_s20_$r.json 2>> $O/err || exit $?
    timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 5 --no-cpu-baseline > $O/${v}_s192_$r.json 2>> $O/err || exit $?
    timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/${v}_c1_$r.json 2>> $O/err || exit $?
    timeout -k 10 300 python -u tools/c4_times.py > $O/${v}_c4_$r.json 2>> $O/err || exit $?
    timeout -k 10 120 python -u tools/tail_sweep.py 1024 65536 > $O/${v}_sweep_$r.json 2>> $O/err || exit $?
  done
done
echo ALLDONE
