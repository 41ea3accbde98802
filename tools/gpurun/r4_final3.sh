#!/bin/bash
# round 4 evidence at HEAD (16-point sum programs: the pairing kernel back at 307 slots): the inversion and sum
# microbenchmarks, the whole GPU suite, smoke(), the BLS PMC passes (copied into profiles/ so the
# bench's roofline finds a summary of these sources), the aggregate probe under a kernel trace,
# the default bench (all legs), the headline at the driver's step count and its kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4f3
mkdir -p $O
for c in fp_inv_vt_lane0 fp_inv_wave final_exp pairing_check g1_sum16 g1_dbl_u; do
  timeout -k 10 60 ./tools/ubench_wave $c >> $O/ubench.jsonl || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/gpurun/r4_bls_prof.sh || exit $?
cp gpurun_out/r4_bls_prof/bls_pmc_n16384.json profiles/round4_bls_pmc_n16384.json || exit $?
timeout -k 10 120 python3 tools/bls_agg_probe.py 67 400 > $O/agg_probe.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/agg -o run --output-format csv -- python3 tools/bls_agg_probe.py 67 200 > $O/agg_trace.log 2>&1 || exit $?
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline > $O/bench_s20.json 2> $O/bench_s20.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --headline-only --steady-steps 0 --single-steps 8 > $O/prof_bench.json 2> $O/prof.log || exit $?
echo ALLDONE
