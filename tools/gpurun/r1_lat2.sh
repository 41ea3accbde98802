set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/lat2 -o lat --output-format csv -- python tools/latency_sweep.py > $O/lat2.log 2>&1
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 48 --warmup 12 --no-cpu-baseline --latency-reps 10 > $O/bench_dist2.json 2> $O/bench_dist2.err
echo ALLDONE
