#!/bin/bash
# tail wave priorities by window (NWV_TAIL_PRIO): kernel times at 1K / 65K and the headline, off / on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 65536 > $O/pr0_k.jsonl 2> $O/pr0_k.err || exit $?
NWV_TAIL_PRIO=1 NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 65536 > $O/pr1_k.jsonl 2> $O/pr1_k.err || exit $?
timeout -k 10 300 python3 -u bench.py --latency-reps 50 --h2h-seconds 0 --no-configs --no-cpu-baseline --steps 384 > $O/pr0_bench.json 2> $O/pr0_bench.err || exit $?
NWV_TAIL_PRIO=1 timeout -k 10 300 python3 -u bench.py --latency-reps 50 --h2h-seconds 0 --no-configs --no-cpu-baseline --steps 384 > $O/pr1_bench.json 2> $O/pr1_bench.err || exit $?
echo ALLDONE
