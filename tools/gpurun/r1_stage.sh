set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_stage.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/lat4 -o lat --output-format csv -- python tools/latency_sweep.py > $O/lat4.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-reps 1000 > $O/bench_stage.json 2> $O/bench_stage.err
echo ALLDONE
