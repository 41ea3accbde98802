"""configs[0]'s Certificate::verify (4-node committee, one call) repeated, for rocprofv3 kernel
traces of the small-call path.  Not part of the product."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
import config_legs as CL  # noqa: E402
from narwhal_amd import types as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
eng = narwhal_amd.Engine(device=0)
seeds, keys, com = CL.committee_fixture(eng, 4, b"nwv-bench-c1")
headers, votes, certs = CL.dag_round(eng, seeds, keys, com)
cert = certs[-1]
keep = T._Keep()
cc = com._c(keep)
carr = (T._Certificate * 1)(cert._c(keep))
res = (ctypes.c_int32 * 1)()
lib = T.lib()
for r in range(reps):
    rc = lib.nwv_certificate_verify_many(eng._h, ctypes.byref(cc), 1, carr, res)
    assert rc == 0 and res[0] == 0
print("ok", reps)
