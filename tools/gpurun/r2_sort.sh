#!/bin/bash
# per-window sort (window-local entry ranges, one-launch small sort): MSM parity tests, bench,
# kernel stats of one 2M-signature batch MSM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py > $O/r2o_pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r2o_bench.json 2> $O/r2o_bench.err || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r2o_2m -o k --output-format csv -- python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 3 --mode 1 > $O/r2o_2m.log 2>&1 || exit $?
echo ALLDONE
