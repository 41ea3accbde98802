set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 > $O/sweep_65536.jsonl 2>&1
timeout -k 10 200 python -u tools/inflight_sweep.py --n 16384 --inflight 1,4,8 > $O/sweep_16384.jsonl 2>&1
timeout -k 10 200 python -u tools/inflight_sweep.py --n 262144 --inflight 1,2 --steps 8 > $O/sweep_262144.jsonl 2>&1
echo ALLDONE
