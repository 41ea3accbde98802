#!/bin/bash
# round 5: keyed small batches with the key sums fused into k_msm_prep's hash workgroup: MSM and
# types-layer GPU tests, then C1 per-call latency A/B against the previous build (NWV_LIB)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5fkeysum
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_types.py tests/test_gpu_baseline_configs.py > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
  NWV_LIB=libnwv_old.so timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/old_c1_$r.json 2>> $O/err || exit $?
  timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/new_c1_$r.json 2>> $O/err || exit $?
done
echo ALLDONE
