set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_msm.py tests/test_gpu_types.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_cfg2.log 2>&1
timeout -k 10 400 python -u bench.py --cpu-seconds 3 --latency-reps 300 > $O/bench_cfg.json 2> $O/bench_cfg.err
echo ALLDONE
