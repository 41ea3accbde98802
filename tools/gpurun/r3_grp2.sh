#!/bin/bash
# round 3: BLS12-381 with the device key cache, group key sums and three streams: GPU parity and
# the BLS leg; the headline with the post-timed steady-state loop
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py -v --timeout 300 --timeout-method thread > $O/r3h_bls_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bls_bench.py 16384 > $O/r3h_bls.json 2> $O/r3h_bls.err || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 > $O/r3h_s20.json 2> $O/r3h_s20.err || exit $?
echo ALLDONE
