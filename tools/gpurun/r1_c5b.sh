set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
NWV_HOST_TRACE=1 timeout -k 10 120 python -u tools/c5_round_trace.py --reps 8 > $O/c5_host.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c5t -o c5 --output-format csv -- python tools/c5_round_trace.py > $O/c5t.log 2>&1
D=$(dirname $(find $O/c5t -name 'c5_kernel_trace.csv' | head -1))
python tools/c5_round_trace.py --timeline $D > $O/c5_timeline.txt
echo ALLDONE
