#!/bin/bash
# round 2 (re-entry): GPU test suite + default bench + rocprof kernel stats of the bench at HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2h_pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r2h_bench.json 2> gpurun_out/r2h_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2h_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 48 --warmup 12 > $GRAFT_REPO_ROOT/gpurun_out/r2h_prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r2h_prof.err
