"""GPU firehose (configs[2] plumbing at test size, one rank): shard verification through the
batch MSM and the host verdict merge find exactly the corrupted indices."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_firehose_single_rank_exact_bad_set():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "firehose_bench.py"), "--n", "200000",
                        "--reps", "1", "--bad", "37"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert '"bad_found_exact": true' in r.stdout
