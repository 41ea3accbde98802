#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_tail3_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/tail_sweep.py 1024 8192 65536 2097152 > gpurun_out/r2_tail3_sweep.jsonl 2> gpurun_out/r2_tail3_sweep.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --h2h-seconds 0 --latency-reps 300 > gpurun_out/r2_tail3_bench20.json 2> gpurun_out/r2_tail3_bench.err
