set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -u tools/profile_driver.py --n 65536 --reps 5 --mode 1 > $O/msm_65536.json 2>&1
timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 1,2,3 > $O/sweep_65536.jsonl 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --latency-reps 100 > $O/bench_a.json 2> $O/bench_a.err
NWV_MSM_MIN_N=1000 timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --latency-reps 100 > $O/bench_b.json 2> $O/bench_b.err
echo ALLDONE
