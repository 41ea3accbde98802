set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/firehose_bench.py --n 2097152 --reps 3 > $O/fh_2m.json 2> $O/fh_2m.err
NWV_MSM_SEG=32 timeout -k 10 300 python -u tools/firehose_bench.py --n 2097152 --reps 3 > $O/fh_2m_s32.json 2> $O/fh_2m_s32.err
echo ALLDONE
