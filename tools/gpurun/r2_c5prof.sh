#!/bin/bash
# device timeline of one coalesced C5 round (nwv_verify_mixed_many), rocprofv3 kernel trace (csv)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 120 python3 -u tools/c5_mixed_prof.py > $O/c5p_plain.json 2> $O/c5p_plain.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/c5p" -o run -- python3 "$GRAFT_REPO_ROOT/tools/c5_mixed_prof.py" > "$GRAFT_REPO_ROOT/$O/c5p.log" 2>&1 || exit $?
echo ALLDONE
