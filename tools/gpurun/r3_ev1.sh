#!/bin/bash
# round 3: drain-coalescer parity, headline at the driver's step count vs a long run, the default
# bench (all config legs), rocprofv3 kernel stats, and the PMC passes at HEAD (65,536 and 2M)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bls.py -v --timeout 200 --timeout-method thread > $O/r3e_bls_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -v --timeout 120 --timeout-method thread > $O/r3e_svc.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --latency-reps 100 --h2h-seconds 0 > $O/r3e_b20_1.json 2> $O/r3e_b20_1.err || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --latency-reps 100 --h2h-seconds 0 > $O/r3e_b20_2.json 2> $O/r3e_b20_2.err || exit $?
timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --no-configs --no-cpu-baseline --latency-reps 100 --h2h-seconds 0 > $O/r3e_b192.json 2> $O/r3e_b192.err || exit $?
timeout -k 10 500 python -u bench.py > $O/r3e_bench.json 2> $O/r3e_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3e_prof -o b --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r3e_prof_bench.json 2> $O/r3e_prof.log || exit $?
for N in 65536 2097152; do
  if [ $N = 65536 ]; then D="python3 tools/profile_driver.py --n 65536 --reps 3 --mode 1"; else D="python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/r3ep1_$N -o p --output-format csv -- $D > $O/r3ep1_$N.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/r3ep2_$N -o p --output-format csv -- $D > $O/r3ep2_$N.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r3ep3_$N -o p --output-format csv -- $D > $O/r3ep3_$N.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --n $N --note "round 3 at HEAD: rocprofv3 --pmc, 3 separate passes, tools/profile_driver.py --mode 1 (batch MSM), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2)" --out $O/round3_msm_pmc_n$N.json $O/r3ep1_$N $O/r3ep2_$N $O/r3ep3_$N || exit $?
done
timeout -k 10 600 python -u tools/bls_bench.py 16384 > $O/r3e_bls.json 2> $O/r3e_bls.err || exit $?
echo ALLDONE
