#!/bin/bash
# round 5: the MSM tail (rotation-form row multiplies, compacted chunk butterflies, top + rest final
# sum): the MSM / Ed25519 GPU tests, then the latency-side probe (C1 legs, per-kernel times)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5tail
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py tests/test_gpu_baseline_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tail_probe.py > $O/probe.json 2> $O/probe.err || exit $?
echo ALLDONE
