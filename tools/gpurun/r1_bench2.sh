set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u bench.py --cpu-seconds 10 > $O/bench_full.json 2> $O/bench_full.err
timeout -k 10 300 python -u bench.py --keys 100 --no-cpu-baseline --latency-reps 30 > $O/bench_keys100.json 2> $O/bench_keys100.err
echo ALLDONE
