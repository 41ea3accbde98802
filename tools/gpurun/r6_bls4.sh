#!/bin/bash
# round 6: registers that are never live together share slots (NSLOTS_PC 171 -> 116): BLS parity,
# the 16,384-item shape at pack 2 / 3 / 4, the whole BLS leg at the best pack
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for pk in 2 3 4; do
  NWV_BLS_PACK=$pk timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 3 > $O/pack_$pk.log 2>&1 || exit $?
  echo "pack $pk: $(tail -1 $O/pack_$pk.log)" >> $O/summary.txt
done
NWV_BLS_PACK=3 timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/leg_pack3.json 2> $O/leg_pack3.err || exit $?
echo ALLDONE
