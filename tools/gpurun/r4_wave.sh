#!/bin/bash
# round 4: the wave engine (bls_wave.h) -- interpreter microbenchmark, BLS GPU tests (wave default,
# batch and per-item paths), the BLS types layer, then the BLS bench leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 200 ./tools/ubench_wave > $O/r4w_ubw.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -v --timeout 300 --timeout-method thread > $O/r4w_pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bls_bench.py 16384 > $O/r4w_bls.json 2> $O/r4w_bls.err || exit $?
echo ALLDONE
