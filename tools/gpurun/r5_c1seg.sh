#!/bin/bash
# round 5: C1 latency against the bucket lanes' segment length (NWV_MSM_SEG) and the BLAKE2b quad
# form for few messages; GPU BLAKE2b parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5c1seg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_blake2b.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_b2.log 2>&1 || exit $?
for s in 0 1 2 4; do
  if [ $s = 0 ]; then unset NWV_MSM_SEG; else export NWV_MSM_SEG=$s; fi
  timeout -k 10 120 python -u tools/c1_times.py 300 > $O/c1_seg$s.json 2> $O/c1_seg$s.err || exit $?
  echo "seg $s: $(cat $O/c1_seg$s.json)" >> $O/summary.txt
done
echo ALLDONE
