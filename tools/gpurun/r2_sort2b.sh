#!/bin/bash
# two-level sort with <= 128 coarse bins: 2M kernel times and WRITE/FETCH passes, MSM parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_firehose.py -x -q --timeout 200 --timeout-method thread > $O/r2t_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 3 --mode 1 > $O/r2t_2m.json 2> $O/r2t_2m.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r2t_w -o p --output-format csv -- python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1 > $O/r2t_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/r2t_f -o p --output-format csv -- python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1 > $O/r2t_f.log 2>&1 || exit $?
python3 tools/pmc_summary.py --n 2097152 --note "two-level sort (<= 128 coarse bins) at 2M: FETCH_SIZE / WRITE_SIZE passes" --out $O/r2t_pmc_2m.json $O/r2t_w $O/r2t_f || exit $?
echo ALLDONE
