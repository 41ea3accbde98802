set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c5t -o c5 --output-format csv -- python tools/c5_round_trace.py > $O/c5t.log 2>&1
D=$(dirname $(find $O/c5t -name 'c5_kernel_trace.csv' | head -1))
python tools/c5_round_trace.py --timeline $D > $O/c5_timeline.txt
echo ALLDONE
