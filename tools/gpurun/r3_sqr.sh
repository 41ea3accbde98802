#!/bin/bash
# round 3: BLS group squaring in four Fp2 products (coef_sqr) -- BLS GPU parity, the BLS leg, the
# tower microbenchmark; the C4 leg with the MSM's early reject; and the PMC passes of the batch MSM
# at HEAD (the MSM kernels changed: kernel_source_hash)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bls.py -v --timeout 200 --timeout-method thread > $O/r3q_bls_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bls_bench.py 16384 > $O/r3q_bls.json 2> $O/r3q_bls.err || exit $?
timeout -k 10 300 ./tools/ubench_bls > $O/r3q_ubench_bls.jsonl 2> $O/r3q_ubench_bls.err || exit $?
for N in 65536 2097152; do
  if [ $N = 65536 ]; then D="python3 tools/profile_driver.py --n 65536 --reps 3 --mode 1"; else D="python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/r3qp1_$N -o p --output-format csv -- $D > $O/r3qp1_$N.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/r3qp2_$N -o p --output-format csv -- $D > $O/r3qp2_$N.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r3qp3_$N -o p --output-format csv -- $D > $O/r3qp3_$N.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --n $N --note "round 3 at HEAD (MSM kernels skip their work after a prep-flagged failure): rocprofv3 --pmc, 3 separate passes, tools/profile_driver.py --mode 1 (batch MSM), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2)" --out $O/round3_msm_pmc_n$N.json $O/r3qp1_$N $O/r3qp2_$N $O/r3qp3_$N || exit $?
done
echo ALLDONE
