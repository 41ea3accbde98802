#!/bin/bash
# round 5 experiment: staged batches replayed through their HIP graph (default) vs direct launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5nograph
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/def_$i.json 2>> $O/err || exit $?
  NWV_STAGE_NOGRAPH=1 timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/nog_$i.json 2>> $O/err || exit $?
done
echo ALLDONE
