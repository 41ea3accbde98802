#!/bin/bash
# parity of the MSM's alternate code paths: the MSM / baseline-config / per-signature GPU suites under
# each tuning switch (lane-local vs quad bucket sums and tail butterflies, the two-level sort at
# every multi-chunk size, smaller tail chunks, fixed bucket-lane sizes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
T="tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_ed25519.py tests/test_gpu_types.py"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u -m pytest $T -x -q --timeout 200 --timeout-method thread > $O/paths_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/paths_$tag.log; exit 1; }
  echo "$tag: $(tail -1 $O/paths_$tag.log)"
}
run lane_bucket_tail NWV_BUCKET_QUAD_MAX_N=0 NWV_TAIL_QUAD_MAX_N=0
run quad_everywhere NWV_BUCKET_QUAD_MAX_N=100000000 NWV_TAIL_QUAD_MAX_N=100000000
run sort2_everywhere NWV_MSM_SORT2_MIN_PTS=1
run tail_s64_seg3 NWV_MSM_TAIL_S=64 NWV_MSM_SEG=3
run seg64 NWV_MSM_SEG=64
echo ALLDONE
