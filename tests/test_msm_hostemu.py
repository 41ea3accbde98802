"""The batch MSM (K5, narwhal_amd/csrc/msm.h) run sequentially on the host with the device
arithmetic (tests/hostemu): signed-digit recoding, the PRF coefficients, and the batch verdict
against the oracle (AND of ZIP-215 per-signature verdicts, SURVEY.md Appendix A "Batch verify")
on valid, invalid and adversarial batches.  The GPU kernels are checked by tests/test_gpu_msm.py."""
import ctypes
import hashlib
import os
import random
import struct

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
    lib.he_msm_batch_split.argtypes = [ctypes.c_size_t, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int]
    lib.he_comb_check.argtypes = [ctypes.c_char_p]
    lib.he_msm_recode.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, vp]
    lib.he_msm_layout.argtypes = [ctypes.c_int, vp]
    lib.he_msm_z.argtypes = [ctypes.c_char_p, ctypes.c_uint64, vp]
    return lib


def msm_batch(he, items, c, G, seed=b"\x11" * 32, counts=None, split=False):
    """split: the key-cache form (every scalar split at 2^128 over A / 2^128 A and B / 2^128 B,
    z-only window layout), as k_keycache_fill + k_msm_keysum run it"""
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
    if split:
        r = he.he_msm_batch_split(len(items), pk.ctypes.data, sg.ctypes.data, arena.ctypes.data,
                                  offs.ctypes.data, lens.ctypes.data, sd.ctypes.data, c, G)
        assert r in (0, 1)
        return bool(r)
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


@pytest.mark.parametrize("c", [6, 8, 10, 12, 13, 14, 15, -8, -12, -13])
def test_window_layout_full_buckets(he, c):
    """Near-equal widths <= c; the z range ends exactly at 129 bits and the full range at 254,
    so every window's top digit range equals its bucket range (no skewed top window).  c < 0:
    the narrow-top layout of width -c (large batches, msm.h msm_split): the same widths per
    range, non-increasing from each range's bottom window to its top."""
    out = (ctypes.c_int * 64)()
    nw = he.he_msm_layout(c, out)
    nwz, widths = out[1], [out[2 + w] for w in range(nw)]
    assert sum(widths[:nwz]) == 129 and sum(widths) == 254
    assert max(widths) <= abs(c) and max(widths) - min(widths) <= 1 + (abs(c) >= 14)
    if c < 0:
        even = (ctypes.c_int * 64)()
        assert he.he_msm_layout(-c, even) == nw and even[1] == nwz
        for lo, hi in ((0, nwz), (nwz, nw)):
            assert widths[lo:hi] == sorted(widths[lo:hi], reverse=True)
            assert sorted(widths[lo:hi]) == sorted(even[2 + w] for w in range(lo, hi))


@pytest.mark.parametrize("c,bits", [(6, 253), (8, 253), (13, 253), (15, 253), (6, 128), (13, 128), (-12, 253),
                                    (-13, 253), (-13, 128)])
def test_recoding_identity(he, c, bits):
    rnd = random.Random(abs(c) * 1000 + bits + (c < 0))
    d = (ctypes.c_int * 128)()
    lay = (ctypes.c_int * 64)()
    he.he_msm_layout(c, lay)
    widths = [lay[2 + w] for w in range(lay[0])]
    hi = L if bits == 253 else 2**128
    for s in [0, 1, hi - 1, 2**(bits - 1), (1 << (abs(c) - 1)), (1 << (abs(c) - 1)) - 1] + \
            [rnd.randrange(hi) for _ in range(300)]:
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


def _chacha20_block_py(key, counter, nonce):
    """RFC 8439 section 2.3, written out from the RFC text (test reference)"""
    def rotl(v, n):
        return ((v << n) | (v >> (32 - n))) & 0xFFFFFFFF

    def qr(x, a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = rotl(x[b] ^ x[c], 7)

    s = [0x61707865, 0x3320646e, 0x79622d32, 0x6b206574] + list(struct.unpack("<8I", key)) + [counter] + \
        list(struct.unpack("<3I", nonce))
    x = list(s)
    for _ in range(10):
        qr(x, 0, 4, 8, 12); qr(x, 1, 5, 9, 13); qr(x, 2, 6, 10, 14); qr(x, 3, 7, 11, 15)
        qr(x, 0, 5, 10, 15); qr(x, 1, 6, 11, 12); qr(x, 2, 7, 8, 13); qr(x, 3, 4, 9, 14)
    return struct.pack("<16I", *[(a + b) & 0xFFFFFFFF for a, b in zip(x, s)])


# RFC 8439 section 2.3.2 test vector (key 00..1f, counter 1, nonce 00:00:00:09:00:00:00:4a:00:00:00:00)
RFC8439_BLOCK = bytes.fromhex(
    "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
    "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def _openssl_chacha20(key, counter, nonce):
    """independent implementation: OpenSSL's EVP_chacha20 keystream (None if unavailable)"""
    try:
        lib = ctypes.CDLL("libcrypto.so.3")
    except OSError:
        return None
    lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    lib.EVP_chacha20.restype = ctypes.c_void_p
    lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.c_char_p]
    lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, ctypes.c_int]
    lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    ctx = lib.EVP_CIPHER_CTX_new()
    iv = struct.pack("<I", counter) + nonce
    assert lib.EVP_EncryptInit_ex(ctx, lib.EVP_chacha20(), None, key, iv) == 1
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_int(0)
    assert lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), bytes(64), 64) == 1
    lib.EVP_CIPHER_CTX_free(ctx)
    return out.raw


def test_chacha20_block(he):
    """the coefficient PRF's block function: RFC 8439 vector, the RFC's algorithm in Python, and
    OpenSSL's ChaCha20 keystream on random keys / counters / nonces"""
    he.he_chacha20_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_void_p]
    out = ctypes.create_string_buffer(64)
    key, nonce = bytes(range(32)), bytes.fromhex("000000090000004a00000000")
    assert _chacha20_block_py(key, 1, nonce) == RFC8439_BLOCK
    he.he_chacha20_block(key, 1, nonce, out)
    assert out.raw == RFC8439_BLOCK
    rnd = random.Random(8439)
    for _ in range(20):
        key, nonce, ctr = rnd.randbytes(32), rnd.randbytes(12), rnd.getrandbits(32)
        he.he_chacha20_block(key, ctr, nonce, out)
        assert out.raw == _chacha20_block_py(key, ctr, nonce)
        ossl = _openssl_chacha20(key, ctr, nonce)
        if ossl is not None:
            assert out.raw == ossl


def test_z_prf(he):
    """z_i = first 16 bytes of ChaCha20(key = seed, counter = low word of i, nonce = high word of
    i || "nwv-" || "z128"), low bit forced to 1 (z_i != 0)"""
    out = ctypes.create_string_buffer(32)
    seed = bytes(range(32))
    for i in (0, 1, 2**32 + 5, 123456789):
        he.he_msm_z(seed, i, out)
        want = bytearray(_chacha20_block_py(seed, i & 0xFFFFFFFF, struct.pack("<I", i >> 32) + b"nwv-z128")[:16])
        want[0] |= 1
        assert out.raw == bytes(want) + bytes(16)


@pytest.mark.parametrize("c,G", [(6, 1), (6, 8), (8, 128), (13, 256), (13, 64), (-12, 64), (-13, 256)])
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
        assert of.verify(*bad[7]) is False
        assert not msm_batch(he, bad, 8, 32)
        assert not msm_batch(he, bad, -9, 32)  # the narrow-top layout


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


@pytest.mark.parametrize("c,G", [(6, 8), (9, 64), (13, 256), (15, 64)])
def test_split_form_valid_batches_accept(he, c, G):
    rnd = random.Random(700 + c)
    assert msm_batch(he, honest(rnd, 11, mlen=40), c, G, split=True)


def test_split_form_invalid_and_zip215_match_oracle(he):
    """key-cache form: one forged signature rejects; every golden / ZIP-215 vector inside a
    batch gives the AND of the oracle's per-signature verdicts (small-order A included: its
    2^128 multiple is the identity, and K A = lo A + hi 2^128 A holds for every group element)"""
    rnd = random.Random(23)
    items = honest(rnd, 6)
    pk, sg, m = items[4]
    items_bad = list(items)
    items_bad[4] = (pk, sg[:40] + bytes([sg[40] ^ 2]) + sg[41:], m)
    assert not msm_batch(he, items_bad, 8, 16, split=True)
    g = of.load_golden("ed25519_vectors.json")["vectors"]
    z = of.load_golden("zip215_small_order.json")["vectors"]
    vecs = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])) for v in g + z[::7]]
    for k, v in enumerate(vecs):
        batch = items[:2] + [v] + items[2:4]
        want = all(of.verify(*it) for it in batch)
        assert msm_batch(he, batch, 7 if k % 2 else 10, 16, split=True) == want, (k, v)


def test_basepoint_comb_term(he):
    """[8 b]B from the fixed-base comb (64 signed radix-16 digits of 8 b mod l over the table
    i 16^j B) equals [8]([b]B), for b = 0, 1, l - 1, 2^252 and random scalars mod l"""
    rnd = random.Random(99)
    for b in [0, 1, 2, L - 1, 2**252, 2**128 - 1] + [rnd.randrange(L) for _ in range(12)]:
        assert he.he_comb_check(b.to_bytes(32, "little")) == 1, b


def test_point_kernel_op_count_matches_bench(he):
    """bench.py's roofline numerator for k_msm_points: field multiplies/squarings per signature."""
    import bench
    he.he_msm_point_counts.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    c = (ctypes.c_ulonglong * 2)()
    for seed in (b"\x01" * 32, b"\x77" * 32):
        he.he_msm_point_counts(of.pubkey(seed), of.sign(seed, b"m"), c)
        assert (c[0], c[1]) == bench.OPS_MSM_POINTS


def test_tiny_path_per_signature_check(he):
    """the one-launch path for tiny keyed batches (k_ed_tiny): [8](R - ([s]B - [k]A)) = 0 with both
    multiples summed from fixed-base combs (B's and the key's i 16^j A), run on the host, equals the
    oracle's ZIP-215 verdict on every golden vector (every Appendix-B category) and on the 196-case
    small-order table -- including undecodable keys (the identity's table) and s >= l"""
    he.he_tiny_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32]
    vecs = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]))
            for v in of.load_golden("ed25519_vectors.json")["vectors"]]
    vecs += [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]))
             for v in of.load_golden("zip215_small_order.json")["vectors"]]
    seen = set()
    for pk, sig, msg in vecs:
        got = he.he_tiny_verify(pk, sig, msg, len(msg))
        want = int(of.verify(pk, sig, msg))
        assert got == want, (pk.hex(), sig.hex())
        seen.add(want)
    assert seen == {0, 1} and len(vecs) > 300
