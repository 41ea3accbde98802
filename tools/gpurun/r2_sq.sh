#!/bin/bash
# 9-step row squaring in the tail's doubling chain: MSM parity tests, per-kernel times, stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_sq_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/tail_sweep.py 1024 4096 65536 > gpurun_out/r2_sq_kernels.jsonl 2> gpurun_out/r2_sq_kernels.err || exit $?
NWV_TAIL_STAMPS=1 timeout -k 10 120 python -u tools/tail_sweep.py 1024 > gpurun_out/r2_sq_stamps1k.jsonl 2> gpurun_out/r2_sq_stamps1k.err || exit $?
