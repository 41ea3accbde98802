#!/bin/bash
# round 6: the new multi-device / tail-timeout tests first, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_tail_timeout.py "tests/test_gpu_baseline_configs.py::test_early_prep_equals_one_stream_order" -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/new.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
echo ALLDONE
