#!/bin/bash
# join with the next piece prefetched: tail phase stamps (slot 7 = join done) at 1K and 65K,
# headline without configs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 65536 > $O/jp_k.jsonl 2> $O/jp_k.err || exit $?
timeout -k 10 300 python3 -u bench.py --latency-reps 50 --h2h-seconds 0 --no-configs --no-cpu-baseline --steps 384 > $O/jp_bench.json 2> $O/jp_bench.err || exit $?
echo ALLDONE
