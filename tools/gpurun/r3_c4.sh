#!/bin/bash
# round 3: MSM kernels skip their work once k_msm_prep has flagged a decode failure / s >= l, and
# k_ed_straus gathers the basepoint tables from LDS: Ed25519 GPU parity tests, per-kernel times of
# the per-signature pipeline, and the C4 call time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_types.py > $O/r3k_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ed_times.py 65536 512 > $O/r3k_ed_times.json 2> $O/r3k_ed_times.err || exit $?
timeout -k 10 200 python -u tools/c4_times.py > $O/r3k_c4.json 2> $O/r3k_c4.err || exit $?
echo ALLDONE
