#!/usr/bin/env python3
"""One C5 round (100-node DAG: 100 certificates, 100 headers, 99 votes) through ONE
nwv_verify_mixed_many call, repeated: host -> host latency per call (run it under rocprofv3
--kernel-trace for the device timeline of a call)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import narwhal_amd
    import config_legs as CL
    from narwhal_amd import types as T
    eng = narwhal_amd.Engine(device=0)
    seeds, keys, com = CL.committee_fixture(eng, 100, b"nwv-bench-c5")
    batches = [CL.worker_batch(a) for a in range(100)]
    pd = eng.blake2b256_many(batches)
    headers, votes, certs = CL.dag_round(eng, seeds, keys, com, payload_digests=pd)
    vsample = votes[:99]
    keep = T._Keep()
    cc = com._c(keep)
    carr = (T._Certificate * len(certs))(*[c._c(keep) for c in certs])
    harr = (T._Header * len(headers))(*[h._c(keep) for h in headers])
    varr = (T._Vote * len(vsample))(*[v._c(keep) for v in vsample])
    hres = (ctypes.c_int32 * len(headers))()
    vres = (ctypes.c_int32 * len(vsample))()
    cres = (ctypes.c_int32 * len(certs))()
    lib = T.lib()
    ts = []
    for r in range(60):
        t = time.perf_counter()
        rm = lib.nwv_verify_mixed_many(eng._h, ctypes.byref(cc), len(headers), harr, hres, len(vsample), varr, vres,
                                       len(certs), carr, cres)
        ts.append(time.perf_counter() - t)
        assert rm == 0 and not any(hres) and not any(vres) and not any(cres)
    ts = np.array(ts[10:]) * 1e3
    print(json.dumps({"p50_ms": float(np.median(ts)), "p99_ms": float(np.percentile(ts, 99))}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
