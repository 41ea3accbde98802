set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
D="python tools/profile_driver.py --n 65536 --reps 2 --mode 1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mp1 -o p --output-format csv -- $D > $O/mp1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/mp2 -o p --output-format csv -- $D > $O/mp2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/mp3 -o p --output-format csv -- $D > $O/mp3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d $O/mp4 -o p --output-format csv -- $D > $O/mp4.log 2>&1
python tools/pmc_summary.py --n 65536 --note "rocprofv3 --pmc, 4 separate passes, tools/profile_driver.py --mode 1 (batch MSM), per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported (gfx950 FETCH_SIZE counts wide streaming reads at 1/2)" --out $O/msm_pmc_n65536.json $O/mp1 $O/mp2 $O/mp3 $O/mp4
D="python tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/mq1 -o p --output-format csv -- $D > $O/mq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/mq2 -o p --output-format csv -- $D > $O/mq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/mq3 -o p --output-format csv -- $D > $O/mq3.log 2>&1
python tools/pmc_summary.py --n 2097152 --note "as n65536, firehose per-GPU shard (2M sigs, 32 B messages)" --out $O/msm_pmc_n2m.json $O/mq1 $O/mq2 $O/mq3
echo ALLDONE
