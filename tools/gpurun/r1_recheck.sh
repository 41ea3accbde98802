set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 5 --latency-reps 50 > $O/bench_if1.json 2> $O/bench_if1.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-reps 50 --inflight 2 > $O/bench_if2.json 2> $O/bench_if2.err
timeout -k 10 300 python -u bench.py --steps 21 --warmup 3 --no-cpu-baseline --latency-reps 50 --inflight 3 > $O/bench_if3.json 2> $O/bench_if3.err
for n in 262144 1048576; do timeout -k 10 200 python -u tools/profile_driver.py --n $n --reps 4 > $O/size_$n.json 2>&1; done
echo ALLDONE
