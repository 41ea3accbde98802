#!/bin/bash
# round 5 experiment: host-device copies as blit kernels on the compute queues (HSA_ENABLE_SDMA=0)
# against the SDMA engines (default): per-call latency (C1, 1K x 512 B), C4, and the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5sdma
mkdir -p $O
for mode in sdma blit; do
  if [ $mode = blit ]; then export HSA_ENABLE_SDMA=0; else unset HSA_ENABLE_SDMA; fi
  timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/${mode}_c1.json 2>> $O/err || exit $?
  timeout -k 10 120 python -u tools/lat1k.py 512 1000 > $O/${mode}_512.json 2>> $O/err || exit $?
  timeout -k 10 300 python -u tools/c4_times.py > $O/${mode}_c4.json 2>> $O/err || exit $?
  timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/${mode}_s20.json 2>> $O/err || exit $?
done
unset HSA_ENABLE_SDMA
timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/sdma2_c1.json 2>> $O/err || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/blit2_c1.json 2>> $O/err || exit $?
echo ALLDONE
