#!/bin/bash
# basepoint term folded into k_msm_prep (no k_msm_bscalar): GPU suite, per-kernel times, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/tail_sweep.py 1024 4096 65536 > gpurun_out/r2b_kernels.jsonl 2> gpurun_out/r2b_kernels.err || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r2b_bench.json 2> gpurun_out/r2b_bench.err || exit $?
