#!/bin/bash
# round 6: kernel + copy trace of the BLS single verify and the aggregate of 67 verified votes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6agg
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/bls_single_trace.py 100 > $O/single_trace.json 2> $O/err.log || exit $?
echo ALLDONE
