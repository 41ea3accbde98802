set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
for s in 8 10 12 15 20; do
  NWV_MSM_SEG=$s timeout -k 10 120 python -u bench.py --no-cpu-baseline --latency-reps 20 > $O/seg_$s.json 2> $O/seg_$s.err
done
echo ALLDONE
