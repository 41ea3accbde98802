set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 2,3,4,6,8 --steps 48 > $O/hwq4.jsonl 2> $O/hwq4.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 2,3,4,6,8 --steps 48 > $O/hwq8.jsonl 2> $O/hwq8.err
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 3,4,6,8,12 --steps 48 > $O/hwq16.jsonl 2> $O/hwq16.err
echo ALLDONE
