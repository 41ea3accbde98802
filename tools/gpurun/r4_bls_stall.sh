#!/bin/bash
# round 4: where the BLS pairing kernel's wave cycles go (16,384 single-key items): parked
# (s_waitcnt / barrier), issue-stalled (all, and on LDS), issuing, and the LDS array's busy and
# bank-conflict cycles -- one rocprofv3 --pmc pass of 8 SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_bls_stall
mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/pmc -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc.log 2>&1 || exit $?
python3 tools/pmc_summary.py --bls --n 16384 --note "BLS pairing kernel stall breakdown (one pass of 8 SQ counters), tools/bls_pmc_driver.py 16384 1" --out $O/bls_stall_n16384.json $O/pmc || exit $?
echo ALLDONE
