#!/bin/bash
# round 5: zero-copy staging of small one-shot calls (default) vs the staging copy (NWV_NO_ZERO_COPY)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py tests/test_gpu_concurrency.py tests/test_gpu_service.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/zc_c1_$i.json 2>> $O/err || exit $?
  timeout -k 10 120 python -u tools/lat1k.py 512 1000 > $O/zc_512_$i.json 2>> $O/err || exit $?
  NWV_NO_ZERO_COPY=1 timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/copy_c1_$i.json 2>> $O/err || exit $?
  NWV_NO_ZERO_COPY=1 timeout -k 10 120 python -u tools/lat1k.py 512 1000 > $O/copy_512_$i.json 2>> $O/err || exit $?
done
echo ALLDONE
