#!/bin/bash
# scatter XCD grouping: MSM parity tests, WRITE_SIZE of the sort kernels at 65,536 and 2M, kernel
# times; headline throughput of this build against the round-1 build (_r1/, same box); radix
# microbenchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py > $O/r2s_pytest.log 2>&1 || exit $?
for N in 65536 2097152; do
  if [ $N = 65536 ]; then D="python3 tools/profile_driver.py --n 65536 --reps 3 --mode 1"; else D="python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1"; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r2s3_$N -o p --output-format csv -- $D > $O/r2s3_$N.log 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-configs --no-cpu-baseline --latency-reps 200 --h2h-seconds 0 > $O/r2s_bench_cur$r.json 2> $O/r2s_bench_cur$r.err || exit $?
  (cd _r1 && timeout -k 10 200 python3 bench.py --no-configs --no-cpu-baseline --latency-reps 200) > $O/r2s_bench_r1_$r.json 2> $O/r2s_bench_r1_$r.err || exit $?
done
timeout -k 10 180 tools/ubench_field > $O/r2_ubench_field.jsonl 2> $O/r2_ubench_field.err || exit $?
echo ALLDONE
