#!/bin/bash
# window-width cap (NWV_MSM_CMAX) against small-batch latency: kernel times at 1K / 4K / 16K and the
# coalesced C5 round
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
for c in 15 11 10 9 8; do
  NWV_MSM_CMAX=$c timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 16384 > $O/cm_k$c.jsonl 2> $O/cm_k$c.err || exit $?
  NWV_MSM_CMAX=$c timeout -k 10 120 python3 -u tools/c5_mixed_prof.py > $O/cm_c5_$c.json 2> $O/cm_c5_$c.err || exit $?
done
echo ALLDONE
