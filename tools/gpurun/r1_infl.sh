set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
for k in 8 12 16 20; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-configs --latency-reps 10 --inflight $k --steps 192 --warmup 48 > $O/infl_$k.json 2> $O/infl_$k.err
done
for q in 24 32; do
  NWV_BENCH_HW_QUEUES=$q timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-configs --latency-reps 10 --inflight 16 --steps 192 --warmup 48 > $O/hwq_$q.json 2> $O/hwq_$q.err
done
echo ALLDONE
