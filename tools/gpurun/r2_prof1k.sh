#!/bin/bash
# per-kernel device durations at 1,024 and 64 signatures (rocprofv3 kernel trace, csv)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/p1k" -o run -- python3 "$GRAFT_REPO_ROOT/tools/tail_sweep.py" 1024 64 > "$GRAFT_REPO_ROOT/$O/p1k.log" 2>&1 || exit $?
echo ALLDONE
