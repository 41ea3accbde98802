set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/latency_sweep.py > $O/latency_sweep.jsonl 2> $O/latency_sweep.err
timeout -k 10 400 python -u tools/firehose_bench.py --n 16777216 --reps 2 > $O/fh_16m.json 2> $O/fh_16m.err
echo ALLDONE
