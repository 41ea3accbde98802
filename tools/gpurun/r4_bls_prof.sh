#!/bin/bash
# round 4: the BLS12-381 throughput shape (16,384 single-key items) under rocprofv3 -- a kernel
# trace with stats, then PMC passes (instruction mix; HBM bytes), each its own run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_bls_prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bls_pmc_driver.py 16384 2 > $O/trace.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM -d $O/pmc1 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc2 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc3 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc3.log 2>&1 || exit $?
python3 tools/pmc_summary.py --bls --n 16384 --note "BLS12-381 wave engine: 16,384 single-key items (registered committee keys), tools/bls_pmc_driver.py" --out $O/bls_pmc_n16384.json $O/pmc1 $O/pmc2 $O/pmc3 || exit $?
echo ALLDONE
