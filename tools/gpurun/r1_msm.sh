set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/pytest_msm.log 2>&1
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -u tools/profile_driver.py --n 65536 --reps 5 --mode 1 > $O/msm_65536.json 2>&1
timeout -k 10 120 python -u tools/profile_driver.py --n 1048576 --reps 3 --mode 1 > $O/msm_1m.json 2>&1
echo ALLDONE
