set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 96 --warmup 24 --cpu-seconds 2 --latency-reps 50 > $O/bench_dist2.json 2> $O/bench_dist2.err
echo ALLDONE
