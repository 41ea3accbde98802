#!/usr/bin/env python3
"""Host-side duration of every nwv_staged_run call in the bench's timed region (12 resident
65,536 x 512 B batches, W warmup steps, then K steps, step s on stage s % 12): does issuing a
graph replay block the host?  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")


def main():
    import narwhal_amd
    import bench
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = narwhal_amd.Engine(device=0)
    pk, sg, msgs, offs, lens = bench.synth(eng, 65536, 512, seed=1000)
    stages = [eng.stage(pk, sg, msgs, offs, lens) for _ in range(12)]
    for s_ in stages:
        s_.run(mode=1)
    for s_ in stages:
        s_.sync()
    for w in range(W):
        stages[w % 12].run(mode=1)
    for s_ in stages:
        s_.sync()
    calls = []
    t0 = time.perf_counter()
    for s in range(K):
        a = time.perf_counter()
        stages[s % 12].run(mode=1)
        calls.append(round((time.perf_counter() - a) * 1e6, 1))
    issued = time.perf_counter() - t0
    for s_ in stages:
        s_.sync()
    dt = time.perf_counter() - t0
    print(json.dumps({"steps": K, "region_ms": dt * 1e3, "issue_ms": issued * 1e3, "call_us": calls,
                      "sigs_per_s": K * 65536 / dt}), flush=True)


if __name__ == "__main__":
    main()
