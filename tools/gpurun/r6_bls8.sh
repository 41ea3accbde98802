#!/bin/bash
# round 6: multi-step Miller programs for computed key lines (an aggregate's key sum: mlc2_* /
# mlc3_*, BLS_WAVE_GROUPS_C_STR): BLS parity, then the BLS leg (its certificate round runs them)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/bls_leg.json 2> $O/bls_leg.err || exit $?
echo ALLDONE
