#!/bin/bash
# lane-interleaved per-signature tables: GPU suite, per-kernel times of the per-signature pipeline, C4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2i_pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/ed_times.py 65536 512 > $O/r2i_ed.json 2> $O/r2i_ed.err || exit $?
timeout -k 10 200 python3 -u tools/c4_times.py > $O/r2i_c4.json 2> $O/r2i_c4.err || exit $?
echo ALLDONE
