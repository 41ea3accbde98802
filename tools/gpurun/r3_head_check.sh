#!/bin/bash
# round 3, last commit: the whole GPU suite and smoke() at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/r3h_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3h_smoke.log 2>&1 || exit $?
echo ALLDONE
