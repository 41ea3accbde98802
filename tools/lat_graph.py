#!/usr/bin/env python3
"""1,024-signature latency three ways: the host-buffer call (nwv_ed25519_verify_batch: staging
copy + kernel-by-kernel launches + verdict copy), a resident batch replayed through its captured
HIP graph (+ verdict fetch), and the same resident batch launched kernel by kernel.  Separates
launch overhead from copies and device time."""
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


def pct(xs):
    return {"p50": float(np.percentile(xs, 50)), "p99": float(np.percentile(xs, 99))}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = 400
    eng = narwhal_amd.Engine(device=0)
    pk, sg, msgs, offs, lens = bench.synth(eng, n, 32, seed=5)
    bits = np.zeros(n // 64 + 2, dtype=np.uint64)
    allv = _lib._i32(0)
    host = []
    for r in range(reps + 20):
        t = time.perf_counter()
        rc = eng.lib.nwv_ed25519_verify_batch(eng._h, n, pk.ctypes.data, sg.ctypes.data, msgs.ctypes.data,
                                              offs.ctypes.data, lens.ctypes.data, None, _lib.ctypes.byref(allv),
                                              bits.ctypes.data)
        assert rc == 0 and allv.value == 1
        if r >= 20:
            host.append((time.perf_counter() - t) * 1e3)
    st = eng.stage(pk, sg, msgs, offs, lens)
    st.run(mode=1)
    st.fetch()
    graph, direct = [], []
    for r in range(reps + 20):
        t = time.perf_counter()
        st.run(mode=1)
        ok, _ = st.fetch()
        assert ok
        if r >= 20:
            graph.append((time.perf_counter() - t) * 1e3)
    for r in range(reps + 20):
        t = time.perf_counter()
        st.run(mode=1, timed=True)
        ok, _ = st.fetch()
        assert ok
        if r >= 20:
            direct.append((time.perf_counter() - t) * 1e3)
    kt = st.kernel_times(1, reset=True)
    st.free()
    eng.close()
    print(json.dumps({"n": n, "host_buffers_ms": pct(host), "resident_graph_ms": pct(graph),
                      "resident_direct_timed_ms": pct(direct), "device_ms": sum(kt.values()),
                      "kernel_ms": kt}))


if __name__ == "__main__":
    main()
