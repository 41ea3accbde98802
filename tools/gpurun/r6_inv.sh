#!/bin/bash
# round 6: the Fp inversion with each divstep matrix row packed in one 64-bit word (bls381.h
# inv_divsteps) against the previous form (tools/ubench_wave_old, built from the previous header),
# alternating on one box: tools/ubench_wave's fp_inv_wave and fp_inv_vt_lane0 cases (no gain: reverted;
# ubench_wave_old was a one-off build of the previous header, not kept)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6inv
mkdir -p $O
for r in 1 2 3; do
  for b in ubench_wave_old ubench_wave; do
    for c in fp_inv_wave fp_inv_vt_lane0; do
      timeout -k 10 120 ./tools/$b $c >> $O/${b}.jsonl 2>> $O/err.log || exit $?
    done
  done
done
echo ALLDONE
