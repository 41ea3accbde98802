#!/bin/bash
# the MSM prep leaves k_i and the s < l flag for the fallback (no k_ed_hash after a rejected batch):
# GPU suite, C4 with / without reuse, headline without configs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2hr_pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/c4_times.py > $O/r2hr_c4.json 2> $O/r2hr_c4.err || exit $?
timeout -k 10 300 python3 -u bench.py --latency-reps 50 --h2h-seconds 0 --no-configs --no-cpu-baseline --steps 384 > $O/r2hr_bench.json 2> $O/r2hr_bench.err || exit $?
echo ALLDONE
