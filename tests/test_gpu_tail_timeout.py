"""k_msm_tail's bounded wait for a window that has not published its sum.  The final-sum wave polls
each window's ready flag at most NWV_TAIL_SPIN_LIMIT times; reaching the bound must never turn a
valid batch into a reported rejection.  The tail then stores "undetermined" (state word 2, host
word code 3) and the host runs the per-signature pass, so verify_batch -- the reference's
verify_batch / aggregate verify, types/src/primary.rs:531-534 -- still returns the oracle's verdict.
A child process with NWV_TAIL_SPIN_LIMIT=1 (read once per process) forces the bound on every
batch whose top window finishes after the basepoint term, i.e. all of them."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["NWV_T_HERE"]); sys.path.insert(0, os.path.dirname(os.environ["NWV_T_HERE"]))
import oracle_ffi as of
import narwhal_amd
e = narwhal_amd.Engine(device=0)
rng = np.random.default_rng(5)
out = {}
for n in (1, 4, 1024, 5000):
    seeds = [rng.bytes(32) for _ in range(n)]
    msgs = [rng.bytes(32) for _ in range(n)]
    pk, sg = e.sign_many(seeds, msgs)
    items = [(pk[32*i:32*i+32].tobytes(), sg[64*i:64*i+64].tobytes(), msgs[i]) for i in range(n)]
    ok_nobits, _ = e.verify_batch(items, want_bits=False)
    ok_bits, bits = e.verify_batch(items)
    bad = sorted({0, n // 2, n - 1})
    forged = list(items)
    for i in bad:
        p, s, m = forged[i]
        forged[i] = (p, s, bytes([m[0] ^ 1]) + m[1:])
    f_nobits, _ = e.verify_batch(forged, want_bits=False)
    f_bits, fb = e.verify_batch(forged)
    want = [of.verify(*it) for it in forged]
    out[str(n)] = {"valid_nobits": ok_nobits, "valid_bits": ok_bits and all(bits),
                   "forged_nobits": f_nobits, "forged_bits": f_bits, "forged_exact": fb == want}
# the key cache's one-signature keyed batch (nwv_ed25519_pubkey_verify, Verifier::verify)
from narwhal_amd import _lib
import ctypes
pk, sg = e.sign_many([b"\x11" * 32], [b"m"])
rc = e.lib.nwv_ed25519_pubkey_verify(e._h, pk.ctypes.data, b"m", 1, sg.ctypes.data)
rc2 = e.lib.nwv_ed25519_pubkey_verify(e._h, pk.ctypes.data, b"n", 1, sg.ctypes.data)
out["pubkey_verify"] = [rc, rc2]
e.close()
print(json.dumps(out))
"""


@pytest.mark.parametrize("limit", ["1"])
def test_undetermined_tail_falls_back_to_per_signature_pass(limit):
    env = dict(os.environ, NWV_TAIL_SPIN_LIMIT=limit, NWV_T_HERE=HERE)
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    for n, r in out.items():
        if n == "pubkey_verify":
            assert r == [0, 1], r  # NWV_OK, NWV_ERR_SIGNATURE
            continue
        assert r["valid_nobits"] and r["valid_bits"], (n, r)
        assert not r["forged_nobits"] and not r["forged_bits"] and r["forged_exact"], (n, r)
