set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u tools/latency_sweep.py > $O/latency_sweep.jsonl 2>&1
echo ALLDONE
