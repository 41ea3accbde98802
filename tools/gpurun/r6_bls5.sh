#!/bin/bash
# round 6: hash to G1 on lane pairs (k_bls_h2c_2) against the 8-lane group form; BLS parity; the leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for g in 0 1; do
  NWV_BLS_H2C_GROUP=$g timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 3 > $O/h2c_group$g.log 2>&1 || exit $?
  echo "h2c group $g: $(tail -1 $O/h2c_group$g.log)" >> $O/summary.txt
done
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/leg.json 2> $O/leg.err || exit $?
echo ALLDONE
