#!/bin/bash
# round 6 closing evidence at HEAD, every output under its own name (nothing overwrites another):
#   pytest -m gpu, smoke(); batch-MSM PMC passes (n = 65,536 and 2,097,152; copied into profiles/
#   on the box so the bench's roofline reads them); the BLS throughput shape's trace + PMC passes;
#   the default bench; the driver's 20-step bench; the headline alone under rocprofv3 with ONE
#   batch in flight (its averages are single-stream kernel times: compare kernel_ms) and, under a
#   different name, with 12 in flight (averages stretched by the overlap).
# Part 2 (r6_evidence2.sh, a separate call: the PMC summaries copied into profiles/ first) runs the
# benches; afterwards (container) tools/gpurun/r6_collect.sh copies the summaries to profiles/round6_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ev
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for n in 65536 2097152; do
  reps=5; [ $n -gt 65536 ] && reps=2
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_n$n/p1 -o pmc --output-format csv -- python3 tools/profile_driver.py --mode 1 --n $n --reps $reps > $O/pmc_n$n.p1.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_n$n/p2 -o pmc --output-format csv -- python3 tools/profile_driver.py --mode 1 --n $n --reps $reps > $O/pmc_n$n.p2.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_n$n/p3 -o pmc --output-format csv -- python3 tools/profile_driver.py --mode 1 --n $n --reps $reps > $O/pmc_n$n.p3.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --n $n --note "round 6 at HEAD: rocprofv3 --pmc, 3 separate passes, tools/profile_driver.py --mode 1 (batch MSM), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2)" --out $O/round6_msm_pmc_n$n.json $O/pmc_n$n/p1 $O/pmc_n$n/p2 $O/pmc_n$n/p3 || exit $?
  cp $O/round6_msm_pmc_n$n.json profiles/ || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bls_trace -o run --output-format csv -- python3 tools/bls_pmc_driver.py 16384 2 > $O/bls_trace.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM -d $O/bls_pmc1 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/bls_pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/bls_pmc2 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/bls_pmc2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/bls_pmc3 -o pmc --output-format csv -- python3 tools/bls_pmc_driver.py 16384 1 > $O/bls_pmc3.log 2>&1 || exit $?
python3 tools/pmc_summary.py --bls --n 16384 --note "round 6 at HEAD: BLS12-381 flat-script pairing kernel, three items a wave, two waves per SIMD; 16,384 single-key items (registered committee keys), tools/bls_pmc_driver.py" --out $O/round6_bls_pmc_n16384.json $O/bls_pmc1 $O/bls_pmc2 $O/bls_pmc3 || exit $?
cp $O/round6_bls_pmc_n16384.json profiles/ || exit $?
echo PART1DONE
