#!/bin/bash
# two-level counting sort at large n: MSM parity tests (forced sort2 + the 2M shard), 2M kernel
# times, WRITE_SIZE pass at 2M
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py tests/test_gpu_firehose.py tests/test_gpu_types.py tests/test_gpu_ed25519.py -x -v --timeout 200 --timeout-method thread > $O/r2s_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 16384 65536 > $O/r2s_kernels.jsonl 2> $O/r2s_kernels.err || exit $?
NWV_TAIL_QUAD_MAX_N=0 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 16384 > $O/r2s_kernels_noquad.jsonl 2> $O/r2s_kernels_noquad.err || exit $?
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 > $O/r2s_stamps1k.jsonl 2> $O/r2s_stamps1k.err || exit $?
timeout -k 10 120 python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 3 --mode 1 > $O/r2s_2m.json 2> $O/r2s_2m.err || exit $?
NWV_MSM_SORT2_MIN_PTS=1000000000 timeout -k 10 120 python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 3 --mode 1 > $O/r2s_2m_one_level.json 2> $O/r2s_2m_one_level.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r2s_w -o p --output-format csv -- python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1 > $O/r2s_w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/r2s_f -o p --output-format csv -- python3 tools/profile_driver.py --n 2097152 --msg-len 32 --reps 1 --mode 1 > $O/r2s_f.log 2>&1 || exit $?
python3 tools/pmc_summary.py --n 2097152 --note "two-level sort at 2M: FETCH_SIZE / WRITE_SIZE passes" --out $O/r2s_pmc_2m.json $O/r2s_w $O/r2s_f || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2s_latgraph.json 2> $O/r2s_latgraph.err || exit $?
echo ALLDONE
