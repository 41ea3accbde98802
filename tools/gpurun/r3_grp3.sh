#!/bin/bash
# round 3: templated group Miller loop -- BLS parity and leg; the BASELINE-size parity tests with
# forged keyed entries (C2) and the whole-shard oracle comparison (C3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py -v --timeout 300 --timeout-method thread > $O/r3q_bls_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bls_bench.py 16384 > $O/r3q_bls16k.json 2> $O/r3q_bls16k.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_configs.py -v --timeout 400 --timeout-method thread > $O/r3q_baseline.log 2>&1 || exit $?
echo ALLDONE
