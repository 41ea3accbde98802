#!/bin/bash
# round 3: the headline at the driver's step count (20 / 5) against in-flight batches and hardware
# queues (every stream gets whole waves of steps), a 192-step reference, and the C5 drain leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
for cfg in 16:10 16:12 16:16 20:20 24:20 24:24; do
  Q=${cfg%%:*}; K=${cfg##*:}
  NWV_BENCH_HW_QUEUES=$Q timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --inflight $K --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 > $O/r3i_q${Q}_k${K}_s20.json 2> $O/r3i_q${Q}_k${K}_s20.err || exit $?
done
NWV_BENCH_HW_QUEUES=24 timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --inflight 20 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 > $O/r3i_q24_k20_s192.json 2> $O/r3i_q24_k20_s192.err || exit $?
NWV_BENCH_HW_QUEUES=16 timeout -k 10 200 python -u bench.py --steps 192 --warmup 48 --inflight 16 --no-configs --no-cpu-baseline --latency-reps 10 --h2h-seconds 0 --single-steps 2 > $O/r3i_q16_k16_s192.json 2> $O/r3i_q16_k16_s192.err || exit $?
timeout -k 10 300 python -u tools/c5_leg.py 20 > $O/r3i_c5.json 2> $O/r3i_c5.err || exit $?
timeout -k 10 300 ./tools/ubench_bls > $O/r3i_ubench_bls.jsonl 2> $O/r3i_ubench_bls.err || exit $?
echo ALLDONE
