#!/bin/bash
# round 5: the BLS leg alone (round and 16,384-item calls timed on prepared arrays)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5blsleg
mkdir -p $O
timeout -k 10 500 python -u tools/bls_bench.py 16384 > $O/bls_leg.json 2> $O/bls_leg.err || exit $?
echo ALLDONE
