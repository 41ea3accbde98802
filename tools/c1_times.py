#!/usr/bin/env python3
"""C1 (BASELINE configs[0]): Certificate::verify of a 4-node committee and verify_batch of 1,024
signatures over 32 B messages, host to host, as the bench's configs.C1 leg measures them (p50 /
p99 over `reps` calls).  For kernel traces of the per-call path (rocprofv3 --kernel-trace)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import narwhal_amd
    import config_legs as CL
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    flags = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0  # e.g. 4096 = NWV_FLAG_NO_TINY
    eng = narwhal_amd.Engine(device=0, flags=flags)
    r, _ = CL.leg_c1(eng, reps=reps)
    r["flags"] = flags
    r["diag_counters"] = eng.diag_counters()
    eng.close()
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
