set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/c4t -o c4 --output-format csv -- python tools/c4_trace.py > $O/c4t.log 2>&1
D=$(dirname $(find $O/c4t -name 'c4_kernel_trace.csv' | head -1))
python tools/c4_trace.py --timeline $D > $O/c4_timeline.txt
echo ALLDONE
