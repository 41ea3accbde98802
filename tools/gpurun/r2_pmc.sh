#!/bin/bash
# round 2 (HEAD): rocprofv3 kernel-trace stats of bench.py, and PMC passes (one counter group per
# run, as MI355X_MICROARCH.md prescribes) of the batch MSM at n = 65,536 and 2M
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r2c_bstat -o b --output-format csv -- python3 bench.py --steps 48 --warmup 12 --no-configs --no-cpu-baseline --latency-reps 50 --h2h-seconds 0 > $O/r2c_bstat.json 2> $O/r2c_bstat.log || exit $?
for N in 65536 2097152; do
  if [ $N = 65536 ]; then D="python3 tools/profile_driver.py --n 65536 --reps 3 --mode 1"; else D="python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/r2cp1_$N -o p --output-format csv -- $D > $O/r2cp1_$N.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/r2cp2_$N -o p --output-format csv -- $D > $O/r2cp2_$N.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r2cp3_$N -o p --output-format csv -- $D > $O/r2cp3_$N.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --n $N --note "round 2 at HEAD (per-window counting sort, fused tail, basepoint term in k_msm_prep): rocprofv3 --pmc, 3 separate passes, tools/profile_driver.py --mode 1 (batch MSM), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2)" --out $O/round2b_msm_pmc_n$N.json $O/r2cp1_$N $O/r2cp2_$N $O/r2cp3_$N || exit $?
done
echo ALLDONE
