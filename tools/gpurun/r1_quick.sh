set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_quick.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-reps 200 > $O/bench_quick.json 2> $O/bench_quick.err
echo ALLDONE
