#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py > $O/r2p_pytest.log 2>&1 || exit $?
for d in .; do
(cd $d && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ab7$d -o k --output-format csv -- python3 tools/profile_driver.py --n 65536 --reps 10 --mode 1) > $O/ab7.log 2>&1 || exit $?
done
timeout -k 10 200 python3 bench.py --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r2p_bench.json 2> $O/r2p_bench.err || exit $?
echo ALLDONE
