#!/bin/bash
# round 4: the wave engine (bls_wave.h) -- BLS GPU tests (wave default, batch and per-item paths),
# the BLS types layer, the BLS bench leg, then the leg's throughput shape under rocprofv3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -v --timeout 300 --timeout-method thread > $O/r4w_pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bls_bench.py 16384 > $O/r4w_bls.json 2> $O/r4w_bls.err || exit $?
bash tools/gpurun/r4_bls_prof.sh || exit $?
echo ALLDONE
