#!/usr/bin/env python3
"""Per-kernel device times of resident batches (single stream, HIP events) at a few sizes, for the
current NWV_* tuning environment.  Prints one JSON line per size."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import narwhal_amd
    sizes = [int(x) for x in (sys.argv[1:] or ["1024", "65536"])]
    eng = narwhal_amd.Engine(device=0, flags=int(os.environ.get("NWV_SWEEP_FLAGS", "0")))
    for n in sizes:
        rng = np.random.default_rng(n)
        mlen = 32 if n < 65536 else 512
        seeds = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
        msgs = rng.integers(0, 256, size=n * mlen + 64, dtype=np.uint8)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(mlen)
        lens = np.full(n, mlen, dtype=np.uint32)
        pk, sg = eng.sign_many_arrays(seeds, msgs, offs, lens)
        st = eng.stage(pk, sg, msgs, offs, lens)
        st.run(mode=1, timed=True)
        st.kernel_times(1, reset=True)
        for _ in range(10):
            st.run(mode=1, timed=True)
        kt = st.kernel_times(1, reset=True)
        ok = st.fetch()[0]
        print(json.dumps({"n": n, "tail_S": os.environ.get("NWV_MSM_TAIL_S", "auto"), "ok": ok,
                          "sum_ms": sum(kt.values()), "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
                          "shape": st.msm_stats()}), flush=True)
        st.free()
    eng.close()


if __name__ == "__main__":
    main()
