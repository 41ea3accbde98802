#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3u_smoke.log 2>&1 || exit $?
timeout -k 10 300 ./tools/ubench_bls > $O/r3u_ubench_bls.jsonl 2> $O/r3u_ubench_bls.err || exit $?
echo ALLDONE
