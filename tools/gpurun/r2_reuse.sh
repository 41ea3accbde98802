#!/bin/bash
# per-signature fallback tables from the MSM's point records: GPU suite, per-kernel fallback
# times, the C4 config
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2u_pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_times.py > $O/r2u_c4.json 2> $O/r2u_c4.err || exit $?
echo ALLDONE
