#!/bin/bash
# round 6: flat-loop lane divisions by a magic table; the single-verify pairing on the flat loop
# (NWV_BLS_SUB_FLAT=1) against the call-based kernel; pack 2 / 3 on the throughput shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
NWV_BLS_SUB_FLAT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_subflat.log 2>&1 || exit $?
for pk in 2 3; do
  NWV_BLS_PACK=$pk timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 3 > $O/pack_$pk.log 2>&1 || exit $?
  echo "pack $pk: $(tail -1 $O/pack_$pk.log)" >> $O/summary.txt
done
for f in 0 1; do
  NWV_BLS_SUB_FLAT=$f timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/leg_subflat$f.json 2> $O/leg_subflat$f.err || exit $?
done
echo ALLDONE
