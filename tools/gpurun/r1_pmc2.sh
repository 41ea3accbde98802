set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -s KILL 60 ./tools/ubench_valu > $O/ubench2.json
D="python tools/profile_driver.py --n 65536 --reps 2 --mode 1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pm1 -o p --output-format csv -- $D > $O/pm1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pm2 -o p --output-format csv -- $D > $O/pm2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pm3 -o p --output-format csv -- $D > $O/pm3.log 2>&1
python tools/pmc_summary.py --n 65536 --note "rocprofv3 --pmc, separate passes, tools/profile_driver.py --mode 1 (batch MSM, timed kernel-by-kernel runs), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2); SQ_INSTS_VALU_INT64 = v_mad_u64_u32 and the other 64-bit integer forms" --out $O/msm_pmc_n65536.json $O/pm1 $O/pm2 $O/pm3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python tools/profile_driver.py --n 65536 --reps 5 --mode 1 > $O/prof3.log 2>&1
echo ALLDONE
