#!/bin/bash
# round 6: BLS per-call paths without the per-stage timing events (they are recorded only on a
# NWV_FLAG_BLS_STAGE_TIMES context now; the stream-ordering events no longer take timestamps):
# BLS parity, then the single verify / aggregate and the whole BLS leg (stage times from a timing
# context)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6blst
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python3 tools/bls_single_trace.py 300 > $O/single_$r.json 2>> $O/err.log || exit $?
done
timeout -k 10 600 python3 tools/bls_bench.py 16384 > $O/bls_leg.json 2>> $O/err.log || exit $?
echo ALLDONE
