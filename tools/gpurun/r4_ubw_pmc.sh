#!/bin/bash
# round 4: instruction counts of the wave interpreter (ubench_wave cases), one PMC pass per case
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ubw_pmc2
mkdir -p $O
for c in pairing_check cyc_sqr_F copy_F_to_M; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INSTS_SMEM -d $O/$c -o pmc --output-format csv -- ./tools/ubench_wave $c > $O/$c.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAVE_CYCLES -d $O/${c}_b -o pmc --output-format csv -- ./tools/ubench_wave $c > $O/${c}_b.log 2>&1 || exit $?
done
echo ALLDONE
