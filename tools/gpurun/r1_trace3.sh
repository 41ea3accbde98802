set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_msm.log 2>&1
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr5 -o tr --output-format csv -- python tools/inflight_sweep.py --n 65536 --modes 1 --inflight 12 --steps 96 > $O/tr5.log 2>&1
timeout -k 10 300 python -u bench.py --keys 100 --no-cpu-baseline --latency-reps 30 > $O/bench_k100.json 2> $O/bench_k100.err
echo ALLDONE
