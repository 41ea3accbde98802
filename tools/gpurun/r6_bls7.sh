#!/bin/bash
# round 6: the packed pairing kernel's Miller loop by lane-capped programs (mlp_*: stages of at most
# 21 lanes, three items a pass): BLS parity, the 16,384-item shape three times, the BLS leg
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 3 > $O/pair_$r.log 2>&1 || exit $?
done
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/bls_leg.json 2> $O/bls_leg.err || exit $?
echo ALLDONE
