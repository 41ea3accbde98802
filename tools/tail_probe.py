#!/usr/bin/env python3
"""Latency-side numbers of the batch MSM in one process: configs.C1 (Certificate::verify of the
4-node committee, verify_batch of 1,024 x 32 B, host -> host p50/p99, as the bench's C1 leg) and
the single-stream per-kernel device times at 1,024 and 65,536 signatures (tools/tail_sweep.py).
Prints one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import narwhal_amd
    import config_legs as CL
    eng = narwhal_amd.Engine(device=0)
    c1, _ = CL.leg_c1(eng, reps=int(os.environ.get("NWV_PROBE_REPS", "1000")))
    eng.close()
    out = {"C1": c1}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tail_sweep.py"), "1024", "65536"],
                       capture_output=True, text=True, timeout=300)
    out["kernels"] = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
