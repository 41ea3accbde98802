set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/lat6 -o lat --output-format csv -- python tools/latency_sweep.py > $O/lat6.log 2>&1
for occ in 30 150 330; do python tools/trace_timeline.py $O/lat6 $occ > $O/lat6_tl_$occ.txt; done
timeout -k 10 300 python -u bench.py --cpu-seconds 10 > $O/bench_r6.json 2> $O/bench_r6.err
echo ALLDONE
