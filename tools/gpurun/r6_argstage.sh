#!/bin/bash
# round 6: small host-to-device staging through kernel arguments (stage_args.h) against the async
# copy (NWV_NO_ARG_STAGE=1), same box: the Ed25519 and BLS GPU suites first, then C1 and the BLS
# single verify / aggregate, alternating, and a kernel + copy trace of C1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6arg
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_types.py tests/test_gpu_ed25519.py tests/test_gpu_bls.py tests/test_gpu_types_bls.py tests/test_gpu_blake2b.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
  for a in 0 1; do
    NWV_NO_ARG_STAGE=$a timeout -k 10 300 python3 tools/c1_times.py 1000 > $O/c1_noarg${a}_$r.json 2>> $O/err.log || exit $?
    NWV_NO_ARG_STAGE=$a timeout -k 10 300 python3 tools/bls_single_trace.py 200 > $O/bls1_noarg${a}_$r.json 2>> $O/err.log || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c1trace -o run -- python3 tools/c1_times.py 200 > $O/c1_trace.json 2>> $O/err.log || exit $?
echo ALLDONE
