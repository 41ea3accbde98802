#!/bin/bash
# round 5 experiment: the staged batches' prep on a low-priority stream and the sorts, buckets and
# tail on a high-priority one (NWV_STAGE_PRIO) against the graph-replay default, 20 and 192 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5prio
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread -k "staged or stage" > $O/pytest_default.log 2>&1 || exit $?
NWV_STAGE_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread -k "staged or stage" > $O/pytest_prio.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/def_s20_$i.json 2>> $O/err || exit $?
  NWV_STAGE_PRIO=1 timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/prio_s20_$i.json 2>> $O/err || exit $?
done
timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 48 --no-cpu-baseline > $O/def_s192.json 2>> $O/err || exit $?
NWV_STAGE_PRIO=1 timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 48 --no-cpu-baseline > $O/prio_s192.json 2>> $O/err || exit $?
echo ALLDONE
