#!/bin/bash
# round 5: the BLS slot layout with the pairing check's slots first (packed banks of NSLOTS_PC):
# every BLS GPU test, the pack sweep at 16,384 items; then the C4 early form (r5_c4b.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5pcl
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_bls.log 2>&1 || exit $?
for pk in 2 3 4; do
  NWV_BLS_PACK=$pk timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 2 > $O/pack_$pk.log 2>&1 || exit $?
  echo "pack $pk: $(tail -1 $O/pack_$pk.log)" >> $O/summary.txt
done
bash tools/gpurun/r5_c4b.sh c4b || exit $?
echo ALLDONE
