#!/bin/bash
# round 6 closing evidence at HEAD, part 2 (after r6_evidence.sh), every output under its own name (nothing overwrites another):
#   pytest -m gpu, smoke(); batch-MSM PMC passes (n = 65,536 and 2,097,152; copied into profiles/
#   on the box so the bench's roofline reads them); the BLS throughput shape's trace + PMC passes;
#   the default bench; the driver's 20-step bench; the headline alone under rocprofv3 with ONE
#   batch in flight (its averages are single-stream kernel times: compare kernel_ms) and, under a
#   different name, with 12 in flight (averages stretched by the overlap).
# Afterwards (container): tools/gpurun/r6_collect.sh copies the summaries to profiles/round6_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ev
mkdir -p $O
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof1 -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --headline-only --inflight 1 --steady-steps 0 --single-steps 8 > $O/headline_inflight1_bench_line.json 2> $O/prof1.log || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof12 -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --headline-only --inflight 12 --steady-steps 0 --single-steps 8 > $O/headline_inflight12_bench_line.json 2> $O/prof12.log || exit $?
echo ALLDONE
