set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_ed25519.py tests/test_gpu_firehose.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_wgw.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs --latency-reps 200 > $O/wgw_512.json 2> $O/wgw_512.err
NWV_MSM_WG_WINDOW=256 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-configs --latency-reps 200 > $O/wgw_256.json 2> $O/wgw_256.err
timeout -k 10 300 python -u tools/firehose_bench.py --n 2097152 --reps 3 > $O/fh_2m.json 2> $O/fh_2m.err
echo ALLDONE
