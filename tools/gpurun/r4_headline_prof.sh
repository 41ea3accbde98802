#!/bin/bash
# round 4: rocprofv3 kernel trace of the 65,536 headline alone, one batch in flight, so the
# per-kernel averages are the single-stream event times the bench line's kernel_ms reports
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --headline-only --inflight 1 --steady-steps 0 --single-steps 8 > $O/prof_bench.json 2> $O/prof.log || exit $?
echo ALLDONE
