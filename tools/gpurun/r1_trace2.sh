set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr4 -o tr --output-format csv -- python tools/inflight_sweep.py --n 65536 --modes 1 --inflight 3 --steps 30 > $O/tr4.log 2>&1
echo ALLDONE
