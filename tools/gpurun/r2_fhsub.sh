#!/bin/bash
# firehose sub-shard size sweep at the 8-GPU per-rank share (2M) and the 2-GPU share (8M)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u tools/firehose_sub_sweep.py 2097152 > $O/r2h_fhsub_2m.jsonl 2> $O/r2h_fhsub_2m.err || exit $?
timeout -k 10 300 python3 -u tools/firehose_sub_sweep.py 8388608 > $O/r2h_fhsub_8m.jsonl 2> $O/r2h_fhsub_8m.err || exit $?
echo ALLDONE
