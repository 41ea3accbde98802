#!/bin/bash
# round 5: C1 under a kernel trace with the fused key sums (k_msm_keysum should be absent from the
# certificate calls), then C1 latency A/B again
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5fkeysum2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c1 -- python3 -u tools/c1_times.py 100 > $O/c1_prof.json 2> $O/c1_prof.err || exit $?
for r in 1 2 3; do
  NWV_LIB=libnwv_old.so timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/old_c1_$r.json 2>> $O/err || exit $?
  timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/new_c1_$r.json 2>> $O/err || exit $?
done
echo ALLDONE
