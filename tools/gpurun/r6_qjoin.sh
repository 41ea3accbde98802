#!/bin/bash
# round 6: tail bucket joins on lane quads (chunks of <= 128 buckets) -- MSM parity, then a same-box
# A/B against the lane-local joins (libnwv_tailB.so): headline single-stream kernel times, 1K latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6qjoin
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py tests/test_gpu_baseline_configs.py tests/test_gpu_tail_timeout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2 3; do
  for lib in libnwv.so libnwv_tailB.so; do
    NWV_LIB=$lib timeout -k 10 200 python3 bench.py --headline-only --inflight 1 --steps 20 --warmup 5 --steady-steps 0 --single-steps 40 > $O/${lib}_$r.json 2> $O/${lib}_$r.err || exit $?
  done
done
for lib in libnwv.so libnwv_tailB.so; do
  NWV_LIB=$lib timeout -k 10 200 python3 tools/c1_times.py 1000 > $O/c1_${lib}.json 2> $O/c1_${lib}.err || exit $?
  NWV_LIB=$lib NWV_TAIL_STAMPS=1 timeout -k 10 200 python3 tools/tail_sweep.py 1024 65536 > $O/stamps_${lib}.json 2> $O/stamps_${lib}.txt || exit $?
done
echo ALLDONE
