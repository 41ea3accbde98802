#!/bin/bash
# throughput A/B: this build against _prev/ (MSM parity tests first)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py > $O/ab6_pytest.log 2>&1 || exit $?
A="--no-configs --no-cpu-baseline --latency-reps 20 --h2h-seconds 0"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $A > $O/ab6_cur$r.json 2> /dev/null || exit $?
  (cd _prev && timeout -k 10 200 python3 bench.py $A) > $O/ab6_prev$r.json 2> /dev/null || exit $?
done
echo ALLDONE
