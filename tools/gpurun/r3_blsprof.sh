#!/bin/bash
# round 3: where the BLS12-381 time goes: the tower microbenchmark (single lane and 8-lane groups)
# and a rocprofv3 kernel trace of the BLS leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py -v --timeout 300 --timeout-method thread > $O/r3p_bls_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bls_bench.py 16384 > $O/r3p_bls16k.json 2> $O/r3p_bls16k.err || exit $?
timeout -k 10 300 ./tools/ubench_bls > $O/r3p_ubench_bls.jsonl 2> $O/r3p_ubench_bls.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r3p_blsprof -o b --output-format csv -- python3 tools/bls_bench.py 1024 > $O/r3p_bls.json 2> $O/r3p_bls.err || exit $?
echo ALLDONE
