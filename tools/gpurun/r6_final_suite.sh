#!/bin/bash
# round 6 closing check at HEAD: the whole GPU suite and smoke() (after the last BLS change)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fin
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo ALLDONE
