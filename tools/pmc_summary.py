#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over the dispatches of one or more passes
(csv output dirs) -> JSON.  Usage: pmc_summary.py --n N --out FILE DIR [DIR ...]"""
import argparse
import collections
import csv
import glob
import json
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    ap.add_argument("--launch-list", default="", help="comma-separated kernels of the profiled pipeline")
    ap.add_argument("--bls", action="store_true", help="a BLS12-381 pass: record the BLS sources' hash")
    a = ap.parse_args()
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "").split("(")[0]
                    c = row.get("Counter_Name")
                    v = float(row.get("Counter_Value", 0) or 0)
                    did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                    sums[k][c] += v
                    cnt[k][c].add(did)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from narwhal_amd._lib import bls_source_hash, kernel_source_hash
    out = {"n": a.n, "note": a.note, "kernels": {}, "kernel_source_hash": kernel_source_hash(),
           "launch_list": a.launch_list.split(",") if a.launch_list else None}
    if a.bls:
        out["bls_source_hash"] = bls_source_hash()
    for k, cs in sums.items():
        out["kernels"][k] = {c: v / max(1, len(cnt[k][c])) for c, v in cs.items()}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
