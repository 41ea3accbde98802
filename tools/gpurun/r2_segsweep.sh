#!/bin/bash
# small-batch tuning: entries per bucket lane (NWV_MSM_SEG) at 1K / 4K / 64K, and the fused
# tail's phase stamps at 1K
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r2_segsweep.jsonl
for G in auto 2 3 4 6 8 12; do
  if [ "$G" = auto ]; then unset NWV_MSM_SEG; else export NWV_MSM_SEG=$G; fi
  echo "{\"seg\": \"$G\"}" >> gpurun_out/r2_segsweep.jsonl
  timeout -k 10 120 python -u tools/tail_sweep.py 1024 4096 >> gpurun_out/r2_segsweep.jsonl 2>> gpurun_out/r2_segsweep.err || exit $?
done
unset NWV_MSM_SEG
NWV_TAIL_STAMPS=1 timeout -k 10 120 python -u tools/tail_sweep.py 1024 > gpurun_out/r2_stamps1k.jsonl 2> gpurun_out/r2_stamps1k.err || exit $?
