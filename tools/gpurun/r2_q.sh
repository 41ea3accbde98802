#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_q_pytest.log 2>&1 || exit $?
NWV_TAIL_STAMPS=1 timeout -k 10 120 python -u tools/tail_sweep.py 1024 65536 2097152 > gpurun_out/r2_q_sweep.jsonl 2> gpurun_out/r2_q_sweep.err || exit $?
timeout -k 10 200 python -u tools/run_cost.py > gpurun_out/r2_runcost2.json 2>gpurun_out/r2_runcost2.err || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --h2h-seconds 0 --latency-reps 200 > gpurun_out/r2_q_bench.json 2> gpurun_out/r2_q_bench.err
