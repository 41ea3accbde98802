#!/usr/bin/env python3
"""Print one iteration's kernel / copy timeline from a rocprofv3 --kernel-trace
--memory-copy-trace CSV pair (latency analysis of tools/latency_sweep.py runs)."""
import csv
import sys


def main():
    d, occ = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(f"{d}/lat_kernel_trace.csv")))
    cps = list(csv.DictReader(open(f"{d}/lat_memory_copy_trace.csv")))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:28], r["Grid_Size_X"]) for r in rows]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"][12:], "") for r in cps]
    ev.sort()
    idx = [i for i, e in enumerate(ev) if e[2].startswith("k_msm_prep")]
    i0 = idx[occ]
    j = i0 - 1
    while j > 0 and not ev[j][2].startswith("k_msm_final"):
        j -= 1
    seg = ev[j + 1:]
    k = next(n for n, e in enumerate(seg) if e[2].startswith("k_msm_final")) + 3
    t0 = seg[0][0]
    for e in seg[:k]:
        print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f}  {e[2]:30s} {e[3]}")


if __name__ == "__main__":
    main()
