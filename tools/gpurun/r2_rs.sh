#!/bin/bash
# arrival-ordered running sum in k_msm_tail: quick sanity first (short limit), then the GPU suite,
# per-kernel times, stamps, 1K latency, firehose sub-shard sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 90 python3 -u tools/tail_sweep.py 1024 65536 > $O/r2r_quick.jsonl 2> $O/r2r_quick.err || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/r2r_pytest.log 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 4096 65536 > $O/r2r_kernels.jsonl 2> $O/r2r_kernels.err || exit $?
NWV_TAIL_STAMPS=1 timeout -k 10 120 python3 -u tools/tail_sweep.py 1024 > $O/r2r_stamps1k.jsonl 2> $O/r2r_stamps1k.err || exit $?
timeout -k 10 120 python3 -u tools/lat_graph.py 1024 > $O/r2r_latgraph.json 2> $O/r2r_latgraph.err || exit $?
timeout -k 10 300 python3 -u tools/firehose_sub_sweep.py 2097152 > $O/r2r_fhsub_2m.jsonl 2> $O/r2r_fhsub_2m.err || exit $?
echo ALLDONE
