#!/bin/bash
# tail phases at 65,536 (lane-local vs quad butterflies) and the headline with quad butterflies
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 65536 > $O/t65_lane.jsonl 2> $O/t65_lane.err || exit $?
NWV_TAIL_QUAD_MAX_N=65536 NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 65536 > $O/t65_quad.jsonl 2> $O/t65_quad.err || exit $?
timeout -k 10 300 python3 -u bench.py --latency-reps 50 --h2h-seconds 0 --no-configs --no-cpu-baseline --steps 384 > $O/t65_bench_lane.json 2> $O/t65_bench_lane.err || exit $?
NWV_TAIL_QUAD_MAX_N=65536 timeout -k 10 300 python3 -u bench.py --latency-reps 50 --h2h-seconds 0 --no-configs --no-cpu-baseline --steps 384 > $O/t65_bench_quad.json 2> $O/t65_bench_quad.err || exit $?
echo ALLDONE
