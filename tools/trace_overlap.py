#!/usr/bin/env python3
"""Kernel concurrency from a rocprofv3 --kernel-trace CSV: busy time (union of kernel intervals),
sum of kernel durations, and the average number of kernels in flight, over a window."""
import csv
import glob
import json
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
    msm = [x for x in iv if x[2].startswith(("k_msm", "k_scan"))]
    t0, t1 = msm[len(msm) // 3][0], msm[-1][1]  # skip warmup third
    sel = [x for x in msm if x[0] >= t0]
    total = sum(e - s for s, e, _ in sel)
    ev = sorted([(s, 1) for s, e, _ in sel] + [(e, -1) for s, e, _ in sel])
    busy, depth, last, hist = 0, 0, None, {}
    for t, d in ev:
        if last is not None and depth > 0:
            busy += t - last
            hist[depth] = hist.get(depth, 0) + (t - last)
        depth += d
        last = t
    print(json.dumps({"window_us": (t1 - t0) / 1e3, "busy_us": busy / 1e3, "sum_kernel_us": total / 1e3,
                      "avg_in_flight": total / max(busy, 1),
                      "time_at_depth_us": {k: v / 1e3 for k, v in sorted(hist.items())}}))


if __name__ == "__main__":
    main()
