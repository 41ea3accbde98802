#!/usr/bin/env python3
"""Latency of one Verifier::verify (nwv_ed25519_pubkey_verify) on a valid and on a forged
signature, host -> host: the single-signature path the reference's Header::verify / Vote::verify
call sites bind."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import narwhal_amd  # noqa: E402
from narwhal_amd import _lib  # noqa: E402


def main():
    out = {}
    for name, flags in (("msm_keyed", 0), ("per_signature", _lib.NWV_FLAG_MSM_NEVER)):
        eng = narwhal_amd.Engine(device=0, flags=flags)
        rnd = np.random.default_rng(1)
        seed, msg = rnd.bytes(32), rnd.bytes(32)
        pk, sg = eng.sign_many([seed], [msg])
        pk, sg = pk[:32].tobytes(), sg[:64].tobytes()
        bad = sg[:40] + bytes([sg[40] ^ 1]) + sg[41:]
        for label, s in (("valid", sg), ("forged", bad)):
            lat = []
            for r in range(220):
                t = time.perf_counter()
                rc = eng.lib.nwv_ed25519_pubkey_verify(eng._h, pk, msg, len(msg), s)
                if r >= 20:
                    lat.append((time.perf_counter() - t) * 1e3)
                assert rc == (0 if label == "valid" else _lib.NWV_ERR_SIGNATURE), rc
            out[f"{name}_{label}"] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99))}
        eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
