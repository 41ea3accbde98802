#!/bin/bash
# round 6: the single-verify pairing kernel on the flat script too (k_blsw_pair_sub), BLS parity,
# then the whole BLS leg (single verify, aggregate, 16,384-item throughput, DAG round, service)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/bls_leg.json 2> $O/bls_leg.err || exit $?
echo ALLDONE
