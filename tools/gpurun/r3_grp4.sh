#!/bin/bash
# round 3: BLS with the uniform Miller-loop grid -- parity, the leg, kernel trace of the round
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py -v --timeout 300 --timeout-method thread > $O/r3v_bls_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bls_bench.py 16384 > $O/r3v_bls16k.json 2> $O/r3v_bls16k.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r3v_blstrace -o b --output-format csv -- python3 tools/bls_bench.py 0 > $O/r3v_bls.json 2> $O/r3v_bls.err || exit $?
echo ALLDONE
