#!/bin/bash
# round 5: C4 with msm_launch's early form (decompressions + fallback tables under the messages'
# PCIe transfer, gated Straus) against the one-stream order; GPU parity of both; tag = $1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-c4b}
O=gpurun_out/r5$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_baseline_configs.py -x -v --timeout 300 --timeout-method thread -k "early_prep or c4 or c2" > $O/pytest.log 2>&1 || exit $?
NWV_HOST_TRACE=1 timeout -k 10 300 python -u tools/c4_times.py > $O/c4.json 2> $O/c4_trace.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- python3 -u tools/c4_times.py > $O/c4_prof.json 2> $O/c4_prof.err || exit $?
echo ALLDONE
