set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo ALLDONE
