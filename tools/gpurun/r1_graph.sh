set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 1,2,3,4 > $O/sweep_65536.jsonl 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --latency-reps 50 > $O/bench_d.json 2> $O/bench_d.err
echo ALLDONE
