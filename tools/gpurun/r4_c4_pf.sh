#!/bin/bash
# round 4: C4 with k_ed_straus vs k_ed_straus_pf (A / R table entries loaded one window ahead),
# two processes (the kernel is chosen once per process), then the per-signature GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
NWV_STRAUS_PF=0 timeout -k 10 300 python -u tools/c4_times.py > $O/r4_c4_pf0.json 2> $O/r4_c4_pf0.err || exit $?
NWV_STRAUS_PF=1 timeout -k 10 300 python -u tools/c4_times.py > $O/r4_c4_pf1.json 2> $O/r4_c4_pf1.err || exit $?
NWV_STRAUS_PF=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py -x -q --timeout 300 --timeout-method thread > $O/r4_c4_pf1_pytest.log 2>&1 || exit $?
echo ALLDONE
