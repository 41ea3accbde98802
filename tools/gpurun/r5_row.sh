#!/bin/bash
# round 5: row-doubling forms on one wave (tools/ubench_row.hip): shift DPP, LDS exchange, row rotations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5row
mkdir -p $O
for i in 1 2 3; do timeout -k 10 60 ./tools/ubench_row >> $O/ubench_row.jsonl || exit $?; done
timeout -k 10 60 ./tools/ubench_prep >> $O/ubench_prep.jsonl || exit $?
echo ALLDONE
