#!/bin/bash
# first GPU run of the BLS12-381 engine: its parity tests, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py -x -v --timeout 300 --timeout-method thread > $O/r3c_bls.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r3c_pytest.log 2>&1 || exit $?
echo ALLDONE
