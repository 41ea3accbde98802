#!/bin/bash
# entries per bucket lane with quad bucket sums at 1K / 4K
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r2s2_sweep.jsonl
for G in auto 3 4 5 6 10 12; do
  if [ "$G" = auto ]; then unset NWV_MSM_SEG; else export NWV_MSM_SEG=$G; fi
  echo "{\"seg\": \"$G\"}" >> $O/r2s2_sweep.jsonl
  timeout -k 10 120 python -u tools/tail_sweep.py 1024 4096 >> $O/r2s2_sweep.jsonl 2>> $O/r2s2_sweep.err || exit $?
done
echo ALLDONE
