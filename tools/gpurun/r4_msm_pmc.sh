#!/bin/bash
# round 4: rocprofv3 --pmc passes of the batch MSM at HEAD (the Ed25519 sources changed this round:
# two carry passes per row multiply, the prefetching Straus kernel), n = 65,536 (the headline) and
# 2,097,152 (a firehose shard): instruction mix, then FETCH_SIZE, then WRITE_SIZE, each its own run;
# then the default bench line, whose roofline reads the new summaries
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_msm_pmc
mkdir -p $O
for n in 65536 2097152; do
  reps=5; [ $n -gt 65536 ] && reps=2
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/n$n/p1 -o pmc --output-format csv -- python3 tools/profile_driver.py --mode 1 --n $n --reps $reps > $O/n$n.p1.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/n$n/p2 -o pmc --output-format csv -- python3 tools/profile_driver.py --mode 1 --n $n --reps $reps > $O/n$n.p2.log 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/n$n/p3 -o pmc --output-format csv -- python3 tools/profile_driver.py --mode 1 --n $n --reps $reps > $O/n$n.p3.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --n $n --note "round 4 at HEAD: rocprofv3 --pmc, 3 separate passes, tools/profile_driver.py --mode 1 (batch MSM), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2)" --out $O/round4_msm_pmc_n$n.json $O/n$n/p1 $O/n$n/p2 $O/n$n/p3 || exit $?
  cp $O/round4_msm_pmc_n$n.json profiles/ || exit $?
done
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo ALLDONE
