#!/bin/bash
# round 4: the wave-parallel Fp inversion (fp_inv_wave) and the aggregate's sum tree -- the
# microbenchmark's inversion / final exponentiation / pairing cases, the BLS GPU tests, then the
# aggregate probe (67 verified votes) under a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_inv
mkdir -p $O
for c in fp_inv_vt_lane0 fp_inv_wave final_exp pairing_check g1_sum32 g1_dbl_u; do
  timeout -k 10 60 ./tools/ubench_wave $c >> $O/ubench.jsonl || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py tests/test_gpu_types_bls.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/bls_agg_probe.py 67 400 > $O/probe.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/bls_agg_probe.py 67 200 > $O/trace.log 2>&1 || exit $?
cat $O/ubench.jsonl $O/probe.log
echo ALLDONE
