#!/usr/bin/env python3
"""p50 / p99 host-to-host latency of nwv_ed25519_verify_batch on 1,024 signatures (distinct keys)
with messages of argv[1] bytes (32: configs[0]; 512: the headline's), argv[2] reps.  One JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import narwhal_amd
    from narwhal_amd import _lib
    mlen = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    eng = narwhal_amd.Engine(device=0)
    rng = np.random.default_rng(5)
    n = 1024
    seeds = [rng.bytes(32) for _ in range(n)]
    msgs = [rng.bytes(mlen) for _ in range(n)]
    pk, sg = eng.sign_many(seeds, msgs)
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    apk, asg, arena, offs, lens = _lib.soa(items)
    allv = _lib._i32(0)
    lat = []
    for r in range(reps + 10):
        t = time.perf_counter()
        _lib._check(eng.lib.nwv_ed25519_verify_batch(eng._h, n, _lib._ptr(apk), _lib._ptr(asg), _lib._ptr(arena),
                                                     _lib._ptr(offs), _lib._ptr(lens), bytes([r % 256]) * 32,
                                                     ctypes.byref(allv), None))
        assert allv.value == 1
        if r >= 10:
            lat.append(time.perf_counter() - t)
    eng.close()
    print(json.dumps({"msg_len": mlen, "reps": reps, "p50_ms": float(np.median(lat)) * 1e3,
                      "p99_ms": float(np.percentile(lat, 99)) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
