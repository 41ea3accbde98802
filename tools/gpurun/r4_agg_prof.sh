#!/bin/bash
# round 4: AggregateAuthenticator::aggregate of 67 verified votes (the verified-signature ring and
# the g1_sum32 tree) -- host p50, then its kernels under a rocprofv3 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_agg
mkdir -p $O
timeout -k 10 120 python3 tools/bls_agg_probe.py 67 400 > $O/probe.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bls_agg_probe.py 67 200 > $O/trace.log 2>&1 || exit $?
cat $O/probe.log
echo ALLDONE
