set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 60 ./tools/ubench_valu > $O/ubench.json
timeout -k 10 400 python -u bench.py --cpu-seconds 10 > $O/bench_full.json 2> $O/bench_full.err
timeout -k 10 300 python -u bench.py --keys 100 --no-cpu-baseline --no-configs --latency-reps 30 > $O/bench_keys100.json 2> $O/bench_keys100.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python tools/profile_driver.py --n 65536 --reps 5 --mode 1 > $O/prof2.log 2>&1
D="python tools/profile_driver.py --n 65536 --reps 2 --mode 1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mr1 -o p --output-format csv -- $D > $O/mr1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/mr2 -o p --output-format csv -- $D > $O/mr2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/mr3 -o p --output-format csv -- $D > $O/mr3.log 2>&1
python tools/pmc_summary.py --n 65536 --note "rocprofv3 --pmc, separate passes, tools/profile_driver.py --mode 1 (batch MSM, timed kernel-by-kernel runs), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2); SQ_INSTS_VALU_INT64 = v_mad_u64_u32 and the other 64-bit integer forms" --out $O/msm_pmc_n65536.json $O/mr1 $O/mr2 $O/mr3
timeout -k 10 300 python -u tools/firehose_bench.py --n 2097152 --reps 3 > $O/fh_2m.json 2> $O/fh_2m.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o bench --output-format csv -- python bench.py --no-cpu-baseline --no-configs --latency-reps 10 > $O/prof_bench.log 2>&1
echo ALLDONE
