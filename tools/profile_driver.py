#!/usr/bin/env python3
"""Minimal driver for rocprofv3 passes (kernel trace / PMC counters): stages one synthetic
batch of --n signatures and runs the verification pipeline --reps times.  No CPU baseline,
no latency loop, so every k_ed_* dispatch in the profile has the same size."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (synthetic data generator)
import narwhal_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--msg-len", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", type=int, default=0, help="0 per-signature pipeline, 1 batch MSM")
    ap.add_argument("--split", action="store_true",
                    help="hash and decompression as separate kernels (NWV_FLAG_MSM_SPLIT_PREP)")
    args = ap.parse_args()
    from narwhal_amd import _lib
    eng = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_SPLIT_PREP if args.split else 0)
    pk, sg, msgs, offs, lens = bench.synth(eng, args.n, args.msg_len, seed=7)
    st = eng.stage(pk, sg, msgs, offs, lens)
    for r in range(args.reps):
        st.run(mode=args.mode, seed=bytes([r + 1]) * 32, timed=True)
    allv, bits = st.fetch()
    ms = st.kernel_times(args.mode)
    st.free()
    eng.close()
    assert allv
    print(json.dumps({"n": args.n, "reps": args.reps, "mode": args.mode, "kernel_ms": ms,
                      "total_ms": sum(ms.values())}))


if __name__ == "__main__":
    main()
