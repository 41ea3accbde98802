#!/bin/bash
# round 4: instruction counts of single wave-interpreter stages (ubench_wave), one PMC pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ubw_pmc
mkdir -p $O
timeout -k 10 120 ./tools/ubench_wave > $O/all.jsonl 2>&1 || exit $?
for c in stage_copy_noload stage_cyc_products_noload stage_cyc_combos_noload; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM -d $O/$c -o pmc --output-format csv -- ./tools/ubench_wave $c > $O/$c.log 2>&1 || exit $?
done
echo ALLDONE
