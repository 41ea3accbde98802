#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_ed25519.py tests/test_gpu_types.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_tail2_pytest.log 2>&1 || exit $?
: > gpurun_out/r2_tail2_sweep.jsonl
for S in auto 32 64; do
  if [ "$S" = auto ]; then unset NWV_MSM_TAIL_S; else export NWV_MSM_TAIL_S=$S; fi
  timeout -k 10 120 python -u tools/tail_sweep.py 1024 8192 65536 2097152 >> gpurun_out/r2_tail2_sweep.jsonl 2>> gpurun_out/r2_tail2_sweep.err || exit $?
done
unset NWV_MSM_TAIL_S
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --h2h-seconds 0 --latency-reps 300 > gpurun_out/r2_tail2_bench20.json 2> gpurun_out/r2_tail2_bench.err
