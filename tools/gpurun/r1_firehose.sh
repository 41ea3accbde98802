set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_firehose.py -x -v --timeout 280 --timeout-method thread -m gpu > $O/pytest_fh.log 2>&1
timeout -k 10 300 python -u tools/firehose_bench.py --n 2097152 --reps 3 > $O/fh_2m.json 2> $O/fh_2m.err
timeout -k 10 400 python -u tools/firehose_bench.py --n 16777216 --reps 2 > $O/fh_16m.json 2> $O/fh_16m.err
echo ALLDONE
