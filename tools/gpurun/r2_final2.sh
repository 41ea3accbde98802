#!/bin/bash
# round 2 HEAD: GPU suite, default bench, rocprofv3 kernel stats of the bench (csv), smoke(), and the
# --gpus 2 spawn rehearsal on one device
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/r2y_pytest.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r2y_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/r2y_bench.json 2> $O/r2y_bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r2y_prof -o b --output-format csv -- python3 bench.py --steps 96 --warmup 24 --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r2y_prof_bench.json 2> $O/r2y_prof.log || exit $?
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 > $O/r2y_bench_g2.json 2> $O/r2y_bench_g2.err || exit $?
echo ALLDONE
