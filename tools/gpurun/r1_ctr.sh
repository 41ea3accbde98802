set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 60 rocprofv3 --list-avail > $O/ctr_list.txt 2>&1 || true
grep -i "VALU\|INSTS" $O/ctr_list.txt | head -80 > $O/ctr_valu.txt || true
D="python tools/profile_driver.py --n 65536 --reps 2 --mode 1 --split"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sp1 -o p --output-format csv -- $D > $O/sp1.log 2>&1
python tools/pmc_summary.py --n 65536 --note "split prep (k_msm_scalars / k_msm_points), SQ_INSTS_VALU" --out $O/split_pmc.json $O/sp1
echo ALLDONE
