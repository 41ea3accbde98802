#!/usr/bin/env python3
"""C4 (65,536 x 512 B, 1 % adversarial) host-to-host call time with the per-signature fallback
building its tables from the MSM's point records (default: the early form, decompressions and
tables under the messages' transfer), on one stream (NWV_FLAG_NO_EARLY_PREP) and with a second
decompression (NWV_FLAG_NO_MSM_REUSE); every bad set must equal the injected one."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import narwhal_amd
    from narwhal_amd import _lib
    import config_legs as CL
    out = {}
    for name, flags in (("reuse", 0), ("one_stream", _lib.NWV_FLAG_NO_EARLY_PREP),
                        ("no_reuse", _lib.NWV_FLAG_NO_MSM_REUSE)):
        eng = narwhal_amd.Engine(device=0, flags=flags)
        r, _ = CL.leg_c4(eng, reps=9)
        out[name] = r
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
