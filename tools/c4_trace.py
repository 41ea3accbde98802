#!/usr/bin/env python3
"""C4 (65,536 x 512 B, 1 % adversarial) through nwv_ed25519_verify_batch, a few calls with 10 ms
gaps, for a rocprofv3 --kernel-trace --memory-copy-trace run; `--timeline DIR` prints the last
call's kernel / copy timeline (tools/c5_round_trace.py does the cutting)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--timeline":
        import c5_round_trace
        c5_round_trace.timeline(sys.argv[2], prefix="c4")
        return
    import narwhal_amd
    import config_legs as cl
    eng = narwhal_amd.Engine(device=0)
    for _ in range(3):
        r, _ = cl.leg_c4(eng, reps=1)
        print(r, flush=True)
        time.sleep(0.01)
    eng.close()


if __name__ == "__main__":
    main()
