#!/usr/bin/env python3
"""Throughput of K resident batches verified round-robin on K streams (mode 0 per-signature
pipeline / mode 1 batch MSM), per batch size: the data behind bench.py's --inflight default."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import narwhal_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--inflight", type=str, default="1,2,3,4")
    ap.add_argument("--modes", type=str, default="0,1")
    args = ap.parse_args()
    eng = narwhal_amd.Engine(device=0)
    pk, sg, msgs, offs, lens = bench.synth(eng, args.n, 512, seed=7)
    kmax = max(int(k) for k in args.inflight.split(","))
    stages = [eng.stage(pk, sg, msgs, offs, lens) for _ in range(kmax)]
    out = []
    for mode in [int(m) for m in args.modes.split(",")]:
        for K in [int(k) for k in args.inflight.split(",")]:
            for w in range(2 * K):
                stages[w % K].run(mode=mode, seed=bytes([w + 1]) * 32)
            for s in stages:
                s.sync()
            t0 = time.perf_counter()
            for i in range(args.steps):
                stages[i % K].run(mode=mode, seed=bytes([i + 1]) * 32)
            for s in stages:
                s.sync()
            dt = time.perf_counter() - t0
            ok = all(s.fetch()[0] for s in stages[:K])
            r = {"n": args.n, "mode": mode, "inflight": K, "ms_per_batch": dt / args.steps * 1e3,
                 "sigs_per_s": args.n * args.steps / dt, "ok": ok}
            print(json.dumps(r), flush=True)
            out.append(r)
    for s in stages:
        s.free()
    eng.close()


if __name__ == "__main__":
    main()
