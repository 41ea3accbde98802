#!/usr/bin/env python3
"""Per-kernel device times of the per-signature pipeline (mode 0: k_ed_hash, k_ed_points,
k_ed_straus) next to the batch MSM (mode 1) on the same resident batch: the C4 fallback's cost."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import narwhal_amd
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    mlen = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    eng = narwhal_amd.Engine(device=0)
    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    msgs = rng.integers(0, 256, size=n * mlen + 64, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(mlen)
    lens = np.full(n, mlen, dtype=np.uint32)
    pk, sg = eng.sign_many_arrays(seeds, msgs, offs, lens)
    st = eng.stage(pk, sg, msgs, offs, lens)
    out = {"n": n, "msg_len": mlen}
    for mode in (0, 1):
        st.run(mode=mode, timed=True)
        st.kernel_times(mode, reset=True)
        for _ in range(10):
            st.run(mode=mode, timed=True)
        kt = st.kernel_times(mode, reset=True)
        ok, bits = st.fetch()
        out[f"mode{mode}"] = {"ok": bool(ok), "sum_ms": sum(kt.values()), "kernel_ms": {k: round(v, 4) for k, v in kt.items()}}
    print(json.dumps(out), flush=True)
    st.free()
    eng.close()


if __name__ == "__main__":
    main()
