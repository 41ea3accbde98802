#!/bin/bash
# round 4: the whole GPU suite (BLS key cache register-only, 100-key committee parity, the BLS
# types layer's 100-node round and Core drain), then the BLS bench leg alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/r4a_pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bls_bench.py 16384 > $O/r4a_bls.json 2> $O/r4a_bls.err || exit $?
echo ALLDONE
