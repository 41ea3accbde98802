#!/bin/bash
# round 3 closing evidence at HEAD (after the MSM early reject and the BLS product rounds): the whole GPU suite, smoke(), the default bench (all legs), the
# headline at the driver's step count, a rocprofv3 kernel trace of the headline, a one-device
# --gpus 2 rehearsal, and the BLS leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/r3y_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3y_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/r3y_bench.json 2> $O/r3y_bench.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline > $O/r3y_bench_s20.json 2> $O/r3y_bench_s20.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r3y_prof -o b --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r3y_prof_bench.json 2> $O/r3y_prof.log || exit $?
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/r3y_bench_g2.json 2> $O/r3y_bench_g2.err || exit $?
timeout -k 10 400 python -u tools/bls_bench.py 16384 > $O/r3y_bls.json 2> $O/r3y_bls.err || exit $?
echo ALLDONE
