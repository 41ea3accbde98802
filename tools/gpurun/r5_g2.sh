#!/bin/bash
# round 5: the multi-rank bench path rehearsed on one device (two ranks share device 0, so the
# value is not a scaling figure): the driver's torch.distributed.run launch shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5g2
mkdir -p $O
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > $O/g2.json 2> $O/g2.err || exit $?
echo ALLDONE
