#!/bin/bash
# the --gpus 2 spawn path rehearsed on one device (firehose line with its roofline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
NWV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 > $O/r2g_bench_g2.json 2> $O/r2g_bench_g2.err || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 200 --timeout-method thread -k "many_keys or keyed" > $O/r2g_pytest.log 2>&1 || exit $?
echo ALLDONE
