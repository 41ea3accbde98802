#!/bin/bash
# round 6, after the last BLS12-381 source change (the per-call paths' timing events): the BLS GPU
# tests, the throughput shape's kernel trace and its PMC passes keyed by the new bls_source_hash
# (the Ed25519 evidence of r6_evidence.sh is unchanged: its kernel_source_hash still matches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ev
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_bls.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bls_trace -o run --output-format csv -- python3 tools/bls_pmc_driver.py 16384 2 > $O/bls_trace.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM -d $O/bls_pmc1 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/bls_pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/bls_pmc2 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/bls_pmc2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/bls_pmc3 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/bls_pmc3.log 2>&1 || exit $?
python3 tools/pmc_summary.py --bls --n 16384 --note "round 6 at HEAD: BLS12-381 flat-script pairing kernel, three items a wave, two waves per SIMD; 16,384 single-key items (registered committee keys), tools/bls_pmc_driver.py" --out $O/round6_bls_pmc_n16384.json $O/bls_pmc1 $O/bls_pmc2 $O/bls_pmc3 || exit $?
echo BLSDONE
