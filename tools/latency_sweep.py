#!/usr/bin/env python3
"""Host-to-host latency of nwv_ed25519_verify_batch (H2D + kernels + D2H) per batch size, through
the batch MSM and through the per-signature pipeline: the data behind the MSM threshold."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import narwhal_amd  # noqa: E402
from narwhal_amd import _lib  # noqa: E402


def main():
    out = []
    n_max = 4096
    eng0 = narwhal_amd.Engine(device=0)
    pk, sg, msgs, offs, lens = bench.synth(eng0, n_max, 32, seed=3)
    eng0.close()
    for name, flag in (("msm", _lib.NWV_FLAG_MSM_ALWAYS), ("per_sig", _lib.NWV_FLAG_MSM_NEVER)):
        eng = narwhal_amd.Engine(device=0, flags=flag)
        for n in (1, 4, 16, 68, 256, 1024, 4096):
            bits = np.zeros(n // 64 + 2, dtype=np.uint64)
            allv = _lib._i32(0)
            lat = []
            for r in range(60):
                t = time.perf_counter()
                rc = eng.lib.nwv_ed25519_verify_batch(eng._h, n, pk.ctypes.data, sg.ctypes.data, msgs.ctypes.data,
                                                      offs.ctypes.data, lens.ctypes.data, b"\x07" * 32,
                                                      _lib.ctypes.byref(allv), bits.ctypes.data)
                if r >= 10:
                    lat.append((time.perf_counter() - t) * 1e3)
                assert rc == 0 and allv.value == 1
            out.append({"path": name, "n": n, "p50_ms": float(np.percentile(lat, 50)),
                        "p99_ms": float(np.percentile(lat, 99))})
            print(json.dumps(out[-1]), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
