"""The batch MSM (K5, narwhal_amd/csrc/msm.h) run sequentially on the host with the device
arithmetic (tests/hostemu): signed-digit recoding, the PRF coefficients, and the batch verdict
against the oracle (AND of ZIP-215 per-signature verdicts, SURVEY.md Appendix A "Batch verify")
on valid, invalid and adversarial batches.  The GPU kernels are checked by tests/test_gpu_msm.py."""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest

import oracle_ffi as of

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HE_PATH = os.path.join(ROOT, "tests", "_build", "libhostemu.so")
L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def he():
    if not os.path.exists(HE_PATH):
        import subprocess
        subprocess.run(["make", "-C", ROOT, "hostemu"], check=True)
    lib = ctypes.CDLL(HE_PATH)
    vp = ctypes.c_void_p
    lib.he_msm_batch.argtypes = [ctypes.c_size_t, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]
    lib.he_msm_recode.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, vp]
    lib.he_msm_layout.argtypes = [ctypes.c_int, vp]
    lib.he_msm_z.argtypes = [ctypes.c_char_p, ctypes.c_uint64, vp]
    return lib


def msm_batch(he, items, c, G, seed=b"\x11" * 32, counts=None):
    pk = np.frombuffer(b"".join(p for p, _, _ in items) + b"\0" * 16, dtype=np.uint8)
    sg = np.frombuffer(b"".join(s for _, s, _ in items) + b"\0" * 16, dtype=np.uint8)
    msgs = [m for _, _, m in items]
    lens = np.array([len(m) for m in msgs], dtype=np.uint32)
    offs = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
    sd = np.frombuffer(seed, dtype=np.uint8)
    cp = counts.ctypes.data if counts is not None else None
    r = he.he_msm_batch(len(items), pk.ctypes.data, sg.ctypes.data, arena.ctypes.data, offs.ctypes.data,
                        lens.ctypes.data, sd.ctypes.data, c, G, cp)
    assert r in (0, 1)
    return bool(r)


def honest(rnd, n, mlen=32):
    out = []
    for _ in range(n):
        seed = bytes(rnd.getrandbits(8) for _ in range(32))
        m = bytes(rnd.getrandbits(8) for _ in range(mlen))
        out.append((of.pubkey(seed), of.sign(seed, m), m))
    return out


@pytest.mark.parametrize("c", [6, 8, 10, 12, 13, 14, 15])
def test_window_layout_full_buckets(he, c):
    """Near-equal widths <= c; the z range ends exactly at 129 bits and the full range at 254,
    so every window's top digit range equals its bucket range (no skewed top window)."""
    out = (ctypes.c_int * 64)()
    nw = he.he_msm_layout(c, out)
    nwz, widths = out[1], [out[2 + w] for w in range(nw)]
    assert sum(widths[:nwz]) == 129 and sum(widths) == 254
    assert max(widths) <= c and max(widths) - min(widths) <= 1 + (c >= 14)


@pytest.mark.parametrize("c,bits", [(6, 253), (8, 253), (13, 253), (15, 253), (6, 128), (13, 128)])
def test_recoding_identity(he, c, bits):
    rnd = random.Random(c * 1000 + bits)
    d = (ctypes.c_int * 128)()
    lay = (ctypes.c_int * 64)()
    he.he_msm_layout(c, lay)
    widths = [lay[2 + w] for w in range(lay[0])]
    hi = L if bits == 253 else 2**128
    for s in [0, 1, hi - 1, 2**(bits - 1), (1 << (c - 1)), (1 << (c - 1)) - 1] + [rnd.randrange(hi) for _ in range(300)]:
        nw = he.he_msm_recode(s.to_bytes(32, "little"), c, bits, d)
        assert nw == (lay[1] if bits == 128 else lay[0])
        assert sum(d[2 * w + 1] << d[2 * w] for w in range(nw)) == s
        for w in range(nw):
            half = 1 << (widths[w] - 1)
            assert -half <= d[2 * w + 1] <= half, (s, w, d[2 * w + 1])
            if w + 1 < nw:
                assert d[2 * w + 1] < half
            else:
                assert d[2 * w + 1] >= 0


def test_z_prf(he):
    out = ctypes.create_string_buffer(32)
    seed = bytes(range(32))
    for i in (0, 1, 2**32 + 5, 123456789):
        he.he_msm_z(seed, i, out)
        want = hashlib.sha512(seed + i.to_bytes(8, "little") + b"nwv-z128").digest()[:16]
        assert out.raw == want + bytes(16)


@pytest.mark.parametrize("c,G", [(6, 1), (6, 8), (8, 128), (13, 256), (13, 64)])
def test_valid_batches_accept(he, c, G):
    rnd = random.Random(c + G)
    items = honest(rnd, 9, mlen=rnd.choice([0, 32, 100]))
    assert msm_batch(he, items, c, G)


def test_empty_batch_accepts(he):
    assert msm_batch(he, [], 8, 16)


def test_invalid_signature_rejects(he):
    rnd = random.Random(5)
    items = honest(rnd, 12)
    for kind in range(4):
        bad = list(items)
        pk, sg, m = bad[7]
        sg = bytearray(sg)
        if kind == 0:
            m = m[:-1] + bytes([m[-1] ^ 1])
        elif kind == 1:
            sg[40] ^= 4  # s
        elif kind == 2:
            sg[3] ^= 1  # R
        else:
            s = int.from_bytes(sg[32:], "little") + L  # s >= l
            sg[32:] = s.to_bytes(32, "little")
        bad[7] = (pk, bytes(sg), m)
        assert not any(False for _ in [])
        assert of.verify(*bad[7]) is False
        assert not msm_batch(he, bad, 8, 32)


def test_golden_and_zip215_batches_match_oracle(he):
    """Every golden vector (valid and adversarial categories) in small mixed batches: the MSM
    verdict equals the AND of the oracle's per-signature ZIP-215 verdicts."""
    rnd = random.Random(17)
    g = of.load_golden("ed25519_vectors.json")["vectors"]
    z = of.load_golden("zip215_small_order.json")["vectors"]
    vecs = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])) for v in g + z]
    base = honest(rnd, 5)
    for k, v in enumerate(vecs):
        items = base[:2] + [v] + base[2:]
        want = all(of.verify(*it) for it in items)
        assert msm_batch(he, items, 6 if k % 2 else 8, 16) == want, (k, v)


def test_all_small_order_batch_accepts(he):
    """ZIP-215's 196 small-order cases all verify individually, so their batch must too (the
    torsion parts cancel only through the cofactor)."""
    z = of.load_golden("zip215_small_order.json")["vectors"]
    items = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])) for v in z]
    assert msm_batch(he, items, 7, 64)


def test_point_kernel_op_count_matches_bench(he):
    """bench.py's roofline numerator for k_msm_points: field multiplies/squarings per signature."""
    import bench
    he.he_msm_point_counts.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    c = (ctypes.c_ulonglong * 2)()
    for seed in (b"\x01" * 32, b"\x77" * 32):
        he.he_msm_point_counts(of.pubkey(seed), of.sign(seed, b"m"), c)
        assert (c[0], c[1]) == bench.OPS_MSM_POINTS
