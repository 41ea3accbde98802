set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u bench.py --cpu-seconds 5 --latency-reps 300 > $O/bench_cfg.json 2> $O/bench_cfg.err
echo ALLDONE
