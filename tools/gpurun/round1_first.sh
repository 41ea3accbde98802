set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 60 ./tools/ubench_valu > gpurun_out/ubench.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 8 > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --latency-reps 20 > gpurun_out/prof_bench.log 2>&1
echo ALLDONE
