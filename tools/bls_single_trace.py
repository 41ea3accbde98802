"""One BLS12-381 Verifier::verify (registered key) repeated, then the aggregate of 67 verified votes,
for a kernel + copy trace of the calls (rocprofv3 --kernel-trace --memory-copy-trace): prints the
host-to-host p50s."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
import config_legs as CL  # noqa: E402
from narwhal_amd.bls import Bls  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
e = narwhal_amd.Engine(device=0)
b = Bls(e)
rnd = np.random.default_rng(77)
sks, pks = CL._bls_committee(b, 67, rnd)
b.register_keys(pks)
m = rnd.bytes(32)
s1 = b.sign([sks[0]], [m])[0]
ts = []
for i in range(reps + 3):
    t0 = time.perf_counter()
    assert b.verify(pks[0], m, s1) == 0
    if i >= 3:
        ts.append(time.perf_counter() - t0)
out = {"reps": reps, "p50_ms": float(np.median(ts)) * 1e3, "kernel_ms": b.last_kernel_ms()}
# AggregateAuthenticator::aggregate of 67 votes verified first (the signature ring)
vs = b.sign(sks, [m] * len(sks))
assert not b.verify_many(pks, vs, [[k] for k in range(len(sks))], [m] * len(sks)).any()
ta = []
for i in range(reps + 3):
    t0 = time.perf_counter()
    rc, agg, _ = b.aggregate(vs)
    assert rc == 0
    if i >= 3:
        ta.append(time.perf_counter() - t0)
assert b.aggregate_verify(agg, pks, m) == 0
out["aggregate67_p50_ms"] = float(np.median(ta)) * 1e3
print(json.dumps(out))
