#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r2_tailsweep.jsonl
for S in auto 1 2 4 8 16 32 64; do
  if [ "$S" = auto ]; then unset NWV_MSM_TAIL_S; else export NWV_MSM_TAIL_S=$S; fi
  timeout -k 10 120 python -u tools/tail_sweep.py 1024 8192 65536 >> gpurun_out/r2_tailsweep.jsonl 2>> gpurun_out/r2_tailsweep.err || exit $?
done
