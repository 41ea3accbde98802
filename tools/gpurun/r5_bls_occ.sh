#!/bin/bash
# round 5: does the BLS pairing kernel slow down with fewer resident waves (LDS padded per wave)?
# 15 KB per wave today (10 waves / CU); +5 KB -> 8, +10.5 KB -> 6, +21 KB -> 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5occ
mkdir -p $O
for pad in 0 5120 10752 21504 0; do
  NWV_BLS_LDS_PAD=$pad timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 2 > $O/pad_$pad.log 2>&1 || exit $?
  echo "pad $pad: $(tail -1 $O/pad_$pad.log)" >> $O/summary.txt
done
echo ALLDONE
