#!/bin/bash
# round 5: C1 calls under rocprofv3 with kernel and memory-copy traces (where the H2D copy of a
# small call sits relative to its first kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5c1copy
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o c1 -- python3 -u tools/c1_times.py 100 > $O/c1.json 2> $O/c1.err || exit $?
echo ALLDONE
