#!/bin/bash
# round 6: kernel trace of the driver's 20-step headline (12 setup runs, 5 warmup, 20 timed, then
# 64 steady steps): where the timed region's time goes against the steady state
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6s20trace
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --headline-only --steady-steps 64 --single-steps 1 > $O/plain.json 2> $O/plain.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --headline-only --steady-steps 64 --single-steps 1 > $O/traced.json 2> $O/traced.err || exit $?
echo ALLDONE
