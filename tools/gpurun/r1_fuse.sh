set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_msm.log 2>&1
for F in 0 1; do
  NWV_MSM_FUSE=$F timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-reps 30 > $O/bench_fuse$F.json 2> $O/bench_fuse$F.err
done
NWV_MSM_FUSE=1 timeout -k 10 300 python -u bench.py --keys 100 --no-cpu-baseline --latency-reps 30 > $O/bench_fuse1_k100.json 2> $O/bench_fuse1_k100.err
NWV_MSM_FUSE=1 timeout -k 10 300 python -u tools/firehose_bench.py --n 2097152 --reps 3 > $O/fh_fuse1.json 2> $O/fh_fuse1.err
echo ALLDONE
