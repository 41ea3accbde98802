set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_firehose.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_msm.log 2>&1
for s in 8 16 32; do NWV_MSM_SEG=$s timeout -k 10 120 python -u tools/profile_driver.py --n 65536 --reps 5 --mode 1 > $O/msm_65536_s$s.json 2>&1; done
timeout -k 10 120 python -u tools/profile_driver.py --n 2097152 --msg-len 32 --reps 3 --mode 1 > $O/msm_2m.json 2>&1
timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 1,2,3 > $O/sweep_65536.jsonl 2>&1
echo ALLDONE
