set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
NWV_HOST_TRACE=1 timeout -k 10 200 python -u tools/c4_trace.py > $O/c4_host.log 2>&1
echo ALLDONE
