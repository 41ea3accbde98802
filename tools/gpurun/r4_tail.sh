#!/bin/bash
# round 4: the MSM tail's row multiplies with two carry passes instead of three -- the GPU MSM
# tests, then the 1K latency + device breakdown and C1 (bench.py at the driver's step count)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
echo ALLDONE
