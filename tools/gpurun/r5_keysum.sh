#!/bin/bash
# round 5: keyed-batch parity after the parallel key sums, then C1 latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5keysum
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_configs.py tests/test_gpu_types.py tests/test_gpu_msm.py tests/test_gpu_ed25519.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/c1_times.py 500 > $O/c1.json 2> $O/c1.err || exit $?
echo ALLDONE
