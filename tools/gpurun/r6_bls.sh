#!/bin/bash
# round 6: the flat-script pairing kernel (no interpreter calls, shared P << k table): BLS parity,
# the 16,384-item shape at pack 2..4 for the default build and the 2-waves-per-SIMD build
# (libnwv_w2.so), a kernel trace and the PMC passes (instructions, scratch writes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
NWV_LIB=libnwv_w2.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_bls.py::test_verify_many_packed_waves" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_w2.log 2>&1 || exit $?
for lib in libnwv.so libnwv_w2.so libnwv_w2g4.so; do
  for pk in 2 3 4; do
    NWV_LIB=$lib NWV_BLS_PACK=$pk timeout -k 10 120 python3 tools/bls_pmc_driver.py 16384 3 > $O/pack_${lib}_$pk.log 2>&1 || exit $?
    echo "$lib pack $pk: $(tail -1 $O/pack_${lib}_$pk.log)" >> $O/summary.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bls_pmc_driver.py 16384 2 > $O/trace.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM -d $O/pmc1 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc2 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc3 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/pmc3.log 2>&1 || exit $?
python3 tools/pmc_summary.py --bls --n 16384 --note "round 6: flat-script pairing kernel, 16,384 single-key items (registered committee keys), tools/bls_pmc_driver.py" --out $O/round6_bls_pmc_n16384.json $O/pmc1 $O/pmc2 $O/pmc3 || exit $?
echo ALLDONE
