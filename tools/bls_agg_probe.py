"""AggregateAuthenticator::aggregate under rocprofv3: a 100-key committee, `q` votes verified in one
call (they enter the verified-signature ring), then `reps` aggregates of them, host-timed; argv[3]
= "cold" aggregates never-verified votes instead.  Not part of the product."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
from narwhal_amd.bls import Bls  # noqa: E402
import config_legs as CL  # noqa: E402

q = int(sys.argv[1]) if len(sys.argv) > 1 else 67
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cold = len(sys.argv) > 3 and sys.argv[3] == "cold"
b = Bls(narwhal_amd.Engine(device=0))
rnd = np.random.default_rng(5)
sks, pks = CL._bls_committee(b, 100, rnd)
b.register_keys(pks)
m = rnd.bytes(32)
vs = b.sign(sks[:q], [m] * q)
if not cold:
    assert not b.verify_many(pks, vs, [[k] for k in range(q)], [m] * q).any()
ts = []
for i in range(reps + 3):
    t0 = time.perf_counter()
    rc, agg, _ = b.aggregate(vs)
    if i >= 3:
        ts.append(time.perf_counter() - t0)
    assert rc == 0
print("aggregate", q, "cold" if cold else "warm", "p50_ms", 1e3 * float(np.median(ts)), flush=True)
