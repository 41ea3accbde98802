set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_row.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/lat3 -o lat --output-format csv -- python tools/latency_sweep.py > $O/lat3.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-reps 200 > $O/bench_row.json 2> $O/bench_row.err
echo ALLDONE
