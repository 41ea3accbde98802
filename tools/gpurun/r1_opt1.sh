set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-reps 30 > $O/bench_opt1.json 2> $O/bench_opt1.err
timeout -k 10 300 python -u bench.py --keys 100 --no-cpu-baseline --latency-reps 30 > $O/bench_opt1_k100.json 2> $O/bench_opt1_k100.err
echo ALLDONE
