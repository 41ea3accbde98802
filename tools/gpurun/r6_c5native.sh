#!/bin/bash
# round 6: the C5 service leg driven from native threads (tools/svcbench.cpp): the Core drain with and
# without the idle gap and the in-library service with 1 and 8 submitter threads (with and without
# the burst flush), beside the one coalesced call; then the bench's whole service leg, and the
# service / drain GPU tests
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c5n
mkdir -p $O
timeout -k 10 300 python3 tools/c5_native.py 20 > $O/c5_native.json 2> $O/c5_native.err || exit $?
timeout -k 10 300 python3 tools/c5_native.py 20 > $O/c5_native2.json 2>> $O/c5_native.err || exit $?
timeout -k 10 300 python3 tools/c5_native.py --python > $O/c5_python_leg.json 2>> $O/c5_native.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_types_bls.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
echo ALLDONE
