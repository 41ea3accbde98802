#!/bin/bash
# quad bucket-sum threshold (NWV_BUCKET_QUAD_MAX_N) for mid-size batches: kernel times at 8K / 16K
# and the coalesced C5 round (6,999 signatures)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
for t in 4096 8192 16384 32768; do
  NWV_BUCKET_QUAD_MAX_N=$t timeout -k 10 120 python3 -u tools/tail_sweep.py 8192 16384 32768 > $O/bqt_k$t.jsonl 2> $O/bqt_k$t.err || exit $?
  NWV_BUCKET_QUAD_MAX_N=$t timeout -k 10 120 python3 -u tools/c5_mixed_prof.py > $O/bqt_c5_$t.json 2> $O/bqt_c5_$t.err || exit $?
done
echo ALLDONE
