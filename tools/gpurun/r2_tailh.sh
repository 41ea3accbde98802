#!/bin/bash
# hybrid tail (4 buckets per lane below the top three windows): MSM parity, kernel trace, VALU
# PMC of the tail, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py > $O/r2h_pytest.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r2h_k -o k --output-format csv -- python3 tools/profile_driver.py --n 65536 --reps 10 --mode 1 > $O/r2h_k.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 -d $O/r2h_p -o p --output-format csv -- python3 tools/profile_driver.py --n 65536 --reps 3 --mode 1 > $O/r2h_p.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r2h_bench.json 2> $O/r2h_bench.err || exit $?
echo ALLDONE
