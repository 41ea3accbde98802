#!/bin/bash
# round 6: the Miller loop with a key's line table by two-step programs (ml2_*_fixed, 332 stages
# against 408) in the one-item pairing kernels: BLS parity, then the whole BLS leg
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6bls6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/bls_leg.json 2> $O/bls_leg.err || exit $?
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/bls_leg2.json 2>> $O/bls_leg.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/strace -o run -- python3 tools/bls_single_trace.py 100 > $O/single_trace.json 2> $O/single_trace.err || exit $?
echo ALLDONE
