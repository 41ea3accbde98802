#!/bin/bash
# full GPU suite + default bench (driver shape) + the --gpus 2 spawn rehearsal on one device
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_full_pytest.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2_full_bench.json 2> gpurun_out/r2_full_bench.err || exit $?
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/r2_full_bench_g2.json 2> gpurun_out/r2_full_bench_g2.err
