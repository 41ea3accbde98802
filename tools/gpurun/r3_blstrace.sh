#!/bin/bash
# round 3: kernel trace of the BLS 100-certificate round alone (no throughput leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r3t_blstrace -o b --output-format csv -- python3 tools/bls_bench.py 0 > $O/r3t_bls.json 2> $O/r3t_bls.err || exit $?
echo ALLDONE
