set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 60 ./tools/ubench_valu > $O/ubench.json
timeout -k 10 400 python -u bench.py --cpu-seconds 10 > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python -u bench.py --mode 0 --inflight 1 --no-cpu-baseline --latency-reps 50 > $O/bench_mode0.json 2> $O/bench_mode0.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/profile_driver.py --n 65536 --reps 5 --mode 1 > $O/prof.log 2>&1
echo ALLDONE
