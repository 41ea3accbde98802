#!/bin/bash
# round 4 evidence at HEAD: the whole GPU suite, smoke(), the default bench (all legs), the
# headline at the driver's step count, a rocprofv3 kernel trace of the headline alone, and a
# one-device --gpus 2 rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline > $O/bench_s20.json 2> $O/bench_s20.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --headline-only --steady-steps 0 --single-steps 8 > $O/prof_bench.json 2> $O/prof.log || exit $?
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_g2.json 2> $O/bench_g2.err || exit $?
echo ALLDONE
