#!/bin/bash
# round 5: BLS pairing checks packed several items per wave -- parity (every pack size) and the
# 16,384-item throughput shape at pack 1..4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5pack
mkdir -p $O
timeout -k 10 600 python -u -m pytest "tests/test_gpu_bls.py::test_verify_many_packed_waves" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for pk in 1 2 3 4; do
  NWV_BLS_PACK=$pk timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 2 > $O/pack_$pk.log 2>&1 || exit $?
  echo "pack $pk: $(tail -1 $O/pack_$pk.log)" >> $O/summary.txt
done
echo ALLDONE
