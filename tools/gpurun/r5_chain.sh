#!/bin/bash
# round 5 experiment: staged runs with their k_msm_prep launches chained across batches
# (NWV_STAGE_CHAIN = k: run r's prep waits for run r - k's), 20- and 192-step headline per k
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5chain
mkdir -p $O
for k in 0 1 2 4; do
  NWV_STAGE_CHAIN=$k timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/k${k}_s20a.json 2>> $O/err || exit $?
  NWV_STAGE_CHAIN=$k timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 5 --no-cpu-baseline > $O/k${k}_s192.json 2>> $O/err || exit $?
  NWV_STAGE_CHAIN=$k timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/k${k}_s20b.json 2>> $O/err || exit $?
done
echo ALLDONE
