#!/bin/bash
# round 6: same-box A/B of the MSM tail: HEAD (spin bound as a kernel argument) vs a build with the
# constant bound (libnwv_tailA.so); single-stream kernel times from the headline alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6tailab
mkdir -p $O
for r in 1 2 3; do
  for lib in libnwv.so libnwv_tailA.so; do
    NWV_LIB=$lib timeout -k 10 200 python3 bench.py --headline-only --inflight 1 --steps 20 --warmup 5 --steady-steps 0 --single-steps 40 > $O/${lib}_$r.json 2> $O/${lib}_$r.err || exit $?
  done
done
echo ALLDONE
