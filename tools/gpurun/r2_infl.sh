#!/bin/bash
# in-flight batches x hardware queues re-sweep at HEAD (bench.py --no-configs, headline only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r2i_sweep.jsonl
for Q in 16 24; do
  for K in 8 12 16 20; do
    NWV_BENCH_HW_QUEUES=$Q timeout -k 10 200 python3 -u bench.py --inflight $K --no-configs --no-cpu-baseline --latency-reps 20 --h2h-seconds 0 --steps 240 --warmup 48 > $O/r2i_tmp.json 2> $O/r2i_tmp.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/r2i_tmp.json').read().strip().splitlines()[-1]); print(json.dumps({'queues': $Q, 'inflight': $K, 'sigs_per_s': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $O/r2i_sweep.jsonl || exit $?
  done
done
echo ALLDONE
