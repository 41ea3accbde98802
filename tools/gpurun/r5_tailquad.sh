#!/bin/bash
# round 5 experiment: k_msm_tail at 65,536 with its chunk butterflies on lane quads
# (NWV_TAIL_QUAD_MAX_N) and with more, smaller chunks per window (NWV_MSM_TAIL_S); kernel times
# and phase stamps (NWV_TAIL_STAMPS) per setting
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5tailquad
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" NWV_TAIL_STAMPS=1 timeout -k 10 120 python -u tools/tail_sweep.py 65536 > $O/$tag.json 2> $O/$tag.stamps || exit $?
}
run base
run quad NWV_TAIL_QUAD_MAX_N=1000000
run s32 NWV_MSM_TAIL_S=32
run quad_s32 NWV_TAIL_QUAD_MAX_N=1000000 NWV_MSM_TAIL_S=32
run base2
run quad2 NWV_TAIL_QUAD_MAX_N=1000000
echo ALLDONE
