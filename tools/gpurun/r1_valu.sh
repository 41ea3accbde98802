set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C -d $O/va1 -o p --output-format csv -- python tools/profile_driver.py --n 65536 --reps 2 --mode 1 > $O/va1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc $C -d $O/va2 -o p --output-format csv -- python tools/profile_driver.py --n 65536 --reps 2 --mode 1 --split > $O/va2.log 2>&1
timeout -s KILL 60 ./tools/ubench_valu > $O/ubench_v.json
timeout -s KILL 90 rocprofv3 --pmc $C -d $O/va3 -o p --output-format csv -- ./tools/ubench_valu > $O/va3.log 2>&1
python tools/pmc_summary.py --n 65536 --note "VALU mix, fused prep" --out $O/valu_fused.json $O/va1
python tools/pmc_summary.py --n 65536 --note "VALU mix, split prep" --out $O/valu_split.json $O/va2
python tools/pmc_summary.py --n 0 --note "VALU mix, ubench" --out $O/valu_ubench.json $O/va3
echo ALLDONE
