#!/bin/bash
# single-signature verify through a one-signature keyed MSM; GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2p_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/single_verify_lat.py > $O/r2p_single.json 2> $O/r2p_single.err || exit $?
timeout -k 10 400 python -u bench.py > $O/r2p_bench.json 2> $O/r2p_bench.err || exit $?
echo ALLDONE
