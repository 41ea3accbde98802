set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_blake2b.py tests/test_gpu_types.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_b2.log 2>&1
timeout -k 10 300 python -u tools/b2_timing.py > $O/b2_timing.json 2> $O/b2_timing.err
echo ALLDONE
