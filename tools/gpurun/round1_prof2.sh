set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 180 --timeout-method thread -m gpu > $O/pytest_gpu2.log 2>&1
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python tools/profile_driver.py --n 65536 --reps 5 > $O/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc1 -o p --output-format csv -- python tools/profile_driver.py --n 65536 --reps 2 > $O/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc2 -o p --output-format csv -- python tools/profile_driver.py --n 65536 --reps 2 > $O/pmc2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc3 -o p --output-format csv -- python tools/profile_driver.py --n 65536 --reps 2 > $O/pmc3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d $O/pmc4 -o p --output-format csv -- python tools/profile_driver.py --n 65536 --reps 2 > $O/pmc4.log 2>&1
for n in 262144 1048576; do timeout -k 10 200 python -u tools/profile_driver.py --n $n --reps 4 > $O/size_$n.json 2>&1; done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-reps 50 > $O/bench_if1.json 2> $O/bench_if1.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-reps 50 --inflight 2 > $O/bench_if2.json 2> $O/bench_if2.err
timeout -k 10 300 python -u bench.py --steps 21 --warmup 3 --no-cpu-baseline --latency-reps 50 --inflight 3 > $O/bench_if3.json 2> $O/bench_if3.err
echo ALLDONE
