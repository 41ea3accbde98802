#!/bin/bash
# round 5: the batch verdict polled from pinned host memory (default) vs copied back after the
# stream's completion (NWV_NO_HOST_POLL); Ed25519 / MSM / baseline GPU tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5poll
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/poll_$i.json 2>> $O/err || exit $?
  NWV_POLL_SYNC=1 timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/pollsync_$i.json 2>> $O/err || exit $?
done
echo ALLDONE
