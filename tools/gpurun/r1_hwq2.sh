set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
for Q in 16 24 32; do
GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python -u tools/inflight_sweep.py --n 65536 --modes 1 --inflight 8,12,16,24,32 --steps 96 > $O/hwqb$Q.jsonl 2> $O/hwqb$Q.err
done
echo ALLDONE
