#!/bin/bash
# round 6 closing run at HEAD: the whole GPU suite and smoke(), then the default bench, the
# driver's 20-step bench and the headline traces (r6_evidence2.sh's steps), every output under
# its own name; the PMC summaries were committed beforehand (r6_evidence.sh, r6_evidence_bls.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ev
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/gpurun/r6_evidence2.sh || exit $?
echo CLOSINGDONE
