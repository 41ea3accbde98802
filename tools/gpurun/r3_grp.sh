#!/bin/bash
# round 3: BLS12-381 on 8-lane groups (bls_group.h): GPU parity, the BLS leg; then resident-batch
# stream priorities at the driver's step count (NWV_STAGE_PRIORITY=1) against the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bls.py -v --timeout 300 --timeout-method thread > $O/r3g_bls_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bls_bench.py 16384 > $O/r3g_bls.json 2> $O/r3g_bls.err || exit $?
for p in 1 0 1; do
NWV_STAGE_PRIORITY=$p timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 >> $O/r3g_prio_s20.jsonl 2>> $O/r3g_prio.err || exit $?
done
NWV_STAGE_PRIORITY=1 timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 >> $O/r3g_prio_s192.jsonl 2>> $O/r3g_prio.err || exit $?
echo ALLDONE
