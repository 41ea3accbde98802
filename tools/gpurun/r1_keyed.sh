set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --latency-reps 100 > $O/bench_d.json 2> $O/bench_d.err
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --latency-reps 20 --keys 100 > $O/bench_k.json 2> $O/bench_k.err
echo ALLDONE
