#!/bin/bash
# round 5: narrow top windows (wide windows at the bottom of each range) with the top windows'
# chunk butterflies on quads (NWV_TAIL_QUAD_TOP_C, 0 = off): tail stamps at 65,536, C4, C1,
# the 20- and 192-step headline, and the MSM GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5narrowtop
mkdir -p $O
NWV_TAIL_STAMPS=1 timeout -k 10 120 python -u tools/tail_sweep.py 1024 65536 > $O/top.json 2> $O/top.stamps || exit $?
NWV_TAIL_QUAD_TOP_C=0 NWV_TAIL_STAMPS=1 timeout -k 10 120 python -u tools/tail_sweep.py 1024 65536 > $O/noquad.json 2> $O/noquad.stamps || exit $?
timeout -k 10 120 python -u tools/tail_sweep.py 1024 4096 65536 > $O/sweep.json 2> $O/sweep.err || exit $?
timeout -k 10 300 python -u tools/c4_times.py > $O/c4.json 2>> $O/err || exit $?
timeout -k 10 120 python -u tools/c1_times.py 1000 > $O/c1.json 2>> $O/err || exit $?
timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/s20.json 2>> $O/err || exit $?
timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 5 --no-cpu-baseline > $O/s192.json 2>> $O/err || exit $?
NWV_TAIL_QUAD_TOP_C=0 timeout -k 10 200 python -u bench.py --headline-only --steps 192 --warmup 5 --no-cpu-baseline > $O/s192_noquad.json 2>> $O/err || exit $?
timeout -k 10 200 python -u bench.py --headline-only --steps 20 --warmup 5 --no-cpu-baseline > $O/s20b.json 2>> $O/err || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_msm.py tests/test_gpu_baseline_configs.py > $O/pytest.log 2>&1 || exit $?
echo ALLDONE
