set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_concurrency.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/pytest_conc.log 2>&1
echo ALLDONE
