#!/usr/bin/env python3
"""C5 round (100-node committee) through nwv_verify_mixed_many, repeated with 10 ms gaps so a
rocprofv3 --kernel-trace --memory-copy-trace run can be cut into rounds
(`--timeline DIR` prints the last round's kernel / copy timeline from such a run)."""
import argparse
import csv
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def timeline(d, prefix="c5"):
    ev = []
    for name in (f"{prefix}_kernel_trace.csv", f"{prefix}_memory_copy_trace.csv"):
        p = os.path.join(d, name)
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            label = r.get("Kernel_Name", "COPY " + r.get("Direction", ""))[:30]
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), label))
    ev.sort()
    groups, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[0] - cur[-1][1] > 5_000_000:
            groups.append(cur)
            cur = []
        cur.append(e)
    groups.append(cur)
    g = groups[-2] if len(groups) > 1 else groups[-1]
    t0 = g[0][0]
    for s, e, lab in g:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {lab}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--timeline", default=None)
    a = ap.parse_args()
    if a.timeline:
        timeline(a.timeline)
        return
    import narwhal_amd
    from narwhal_amd import types as T
    import config_legs as cl
    eng = narwhal_amd.Engine(device=0)
    seeds, keys, com = cl.committee_fixture(eng, 100, b"nwv-bench-c5")
    headers, votes, certs = cl.dag_round(eng, seeds, keys, com)
    votes = votes[:99]
    for r in range(a.reps):
        t0 = time.perf_counter()
        gh, gv, gc = T.verify_mixed(eng, com, headers, votes, certs)
        t1 = time.perf_counter()
        assert not any(gh) and not any(gv) and not any(gc)
        print(f"round {r}: {(t1 - t0) * 1e3:.3f} ms (incl. Python marshalling)", flush=True)
        time.sleep(0.01)
    eng.close()


if __name__ == "__main__":
    main()
