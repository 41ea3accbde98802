#!/bin/bash
# round 3 start: GPU suite at HEAD, then the headline at the driver's step count vs a long run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r3a_pytest.log 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --latency-reps 100 --h2h-seconds 0 > $O/r3a_b20_$i.json 2> $O/r3a_b20_$i.err || exit $?
timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --no-configs --no-cpu-baseline --latency-reps 100 --h2h-seconds 0 > $O/r3a_b192_$i.json 2> $O/r3a_b192_$i.err || exit $?
done
echo ALLDONE
