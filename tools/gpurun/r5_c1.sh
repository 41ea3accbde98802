#!/bin/bash
# round 5: C1 per-call latency (Certificate::verify n = 4, verify_batch 1,024 x 32 B) with its
# host-side timeline and kernel trace; tag = $1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-c1}
O=gpurun_out/r5$T
mkdir -p $O
NWV_HOST_TRACE=1 timeout -k 10 300 python -u tools/c1_times.py 300 > $O/c1.json 2> $O/c1_trace.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c1 -- python3 -u tools/c1_times.py 100 > $O/c1_prof.json 2> $O/c1_prof.err || exit $?
echo ALLDONE
