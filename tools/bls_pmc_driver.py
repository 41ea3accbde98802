"""A short BLS12-381 workload for rocprofv3 passes: the committee registered, then `n` single-key
items (the BLS leg's throughput shape) verified `reps` times in one call each.  Not part of the
product."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
from narwhal_amd.bls import Bls  # noqa: E402
import config_legs as CL  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
b = Bls(narwhal_amd.Engine(device=0))
rnd = np.random.default_rng(77)
sks, pks = CL._bls_committee(b, 100, rnd)
b.register_keys(pks)
msgs = [rnd.bytes(32) for _ in range(n)]
kidx = (np.arange(n) % 100).tolist()
sigs = b.sign([sks[k] for k in kidx], msgs)
for _ in range(reps):
    st = b.verify_many(pks, sigs, [[k] for k in kidx], msgs)
    assert not st.any()
print("ok", n, reps, b.last_kernel_ms(), flush=True)
