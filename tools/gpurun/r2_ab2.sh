#!/bin/bash
# A/B kernel stats at 65,536 (rocprofv3 kernel trace): this tree, and the variant trees given as args
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
for d in . "$@"; do
  tag=$(basename $(cd $d && pwd))
  (cd $d && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ab2_$tag -o k --output-format csv -- python3 tools/profile_driver.py --n 65536 --reps 10 --mode 1) > $O/ab2_$tag.log 2>&1 || exit $?
done
echo ALLDONE
