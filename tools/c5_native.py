"""C5 service leg from native threads only (tools/svcbench.cpp via config_legs.leg_c5_service_native),
plus the one coalesced call for reference; prints one JSON line.  Usage: python tools/c5_native.py [rounds]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
from narwhal_amd import types as T  # noqa: E402
import config_legs as L  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
    eng = narwhal_amd.Engine(device=0)
    seeds, keys, com = L.committee_fixture(eng, 100, b"nwv-bench-c5")
    headers, votes, certs = L.dag_round(eng, seeds, keys, com)
    vsample = votes[:99]
    keep = T._Keep()
    cc = com._c(keep)
    carr = (T._Certificate * len(certs))(*[c._c(keep) for c in certs])
    harr = (T._Header * len(headers))(*[h._c(keep) for h in headers])
    varr = (T._Vote * len(vsample))(*[v._c(keep) for v in vsample])
    nsig = sum(1 + len(c.aggregated_signature) for c in certs) + len(headers) + len(vsample)
    hres = (ctypes.c_int32 * len(headers))()
    vres = (ctypes.c_int32 * len(vsample))()
    cres = (ctypes.c_int32 * len(certs))()
    lib = T.lib()
    tm = []
    for r in range(rounds + 2):
        t = time.perf_counter()
        assert lib.nwv_verify_mixed_many(eng._h, ctypes.byref(cc), len(headers), harr, hres, len(vsample), varr,
                                         vres, len(certs), carr, cres) == 0
        if r >= 2:
            tm.append(time.perf_counter() - t)
    if "--python" in sys.argv:  # the bench's whole service leg (Python CoreDrain, async submission, native)
        out = {"coalesced_ms_per_round": float(np.median(tm)) * 1e3,
               "service": L.leg_c5_service(eng, com, cc, harr, varr, carr, nsig)}
    else:
        out = {"coalesced_ms_per_round": float(np.median(tm)) * 1e3,
               "native": L.leg_c5_service_native(eng, cc, harr, varr, carr, nsig, rounds)}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
