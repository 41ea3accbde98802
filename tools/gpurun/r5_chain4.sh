#!/bin/bash
# round 5: prep chaining as the staged default (depth 3): MSM / concurrency / baseline-config GPU
# tests, then the 20-step headline (x3) and 192 steps at the default and unchained
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5chain4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_concurrency.py tests/test_gpu_baseline_configs.py tests/test_gpu_ed25519.py > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/def_s20_$r.json 2>> $O/err || exit $?
  NWV_STAGE_CHAIN=0 timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/off_s20_$r.json 2>> $O/err || exit $?
done
timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 5 --no-cpu-baseline > $O/def_s192.json 2>> $O/err || exit $?
NWV_STAGE_CHAIN=0 timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 5 --no-cpu-baseline > $O/off_s192.json 2>> $O/err || exit $?
echo ALLDONE
