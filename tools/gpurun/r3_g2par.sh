#!/bin/bash
# round 3: the Miller loop's G2 doubling as four rounds of Fp products over the group's lanes
# (g_ml_dbl) -- BLS GPU parity, the BLS leg, the tower microbenchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bls.py -v --timeout 200 --timeout-method thread > $O/r3g_bls_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bls_bench.py 16384 > $O/r3g_bls.json 2> $O/r3g_bls.err || exit $?
timeout -k 10 300 ./tools/ubench_bls > $O/r3g_ubench_bls.jsonl 2> $O/r3g_ubench_bls.err || exit $?
echo ALLDONE
