#!/bin/bash
# round 4: staging copies on a persistent helper pool -- the Ed25519 GPU tests, C4 (both Straus
# forms), then the default bench at the driver's step count
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ed25519.py tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/c4_times.py > $O/c4.json 2> $O/c4.err || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
echo ALLDONE
