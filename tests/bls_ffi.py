"""ctypes wrapper around oracle/build/libbls_oracle.so -- TEST INFRASTRUCTURE ONLY (the BLS12-381
checker).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg load it."""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libbls_oracle.so")
DST_NUL = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"
ORB_OK, ORB_BAD_ENCODING, ORB_NOT_ON_CURVE, ORB_NOT_IN_GROUP, ORB_AGGR_MISMATCH, ORB_VERIFY_FAIL, ORB_PK_INFINITY = range(7)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(LIB_PATH)
        c, sz, vp = ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p
        for name, args, res in [
            ("orb_sha256", [c, sz, vp], None),
            ("orb_expand_message_xmd", [c, sz, c, sz, vp, sz], None),
            ("orb_hash_to_g1", [c, sz, c, sz, vp], None),
            ("orb_keygen", [c, vp], ctypes.c_int),
            ("orb_sign", [c, c, sz, c, sz, vp], ctypes.c_int),
            ("orb_g1_decompress", [c, vp, vp], ctypes.c_int),
            ("orb_g2_decompress", [c, vp, vp], ctypes.c_int),
            ("orb_g1_in_group", [c], ctypes.c_int),
            ("orb_g2_in_group", [c], ctypes.c_int),
            ("orb_pubkey_validate", [c], ctypes.c_int),
            ("orb_verify", [c, c, sz, c, c, sz], ctypes.c_int),
            ("orb_aggregate", [sz, c, vp], ctypes.c_int),
            ("orb_aggregate_pubkeys", [sz, c, vp], ctypes.c_int),
            ("orb_fast_aggregate_verify", [c, sz, c, c, sz, c, sz], ctypes.c_int),
            ("orb_fast_aggregate_verify_mt", [sz, vp, vp, vp, vp, vp, vp, vp, c, sz, vp, ctypes.c_int], None),
            ("orb_verify_items_keytab_mt", [sz, vp, sz, vp, vp, vp, vp, vp, vp, vp, c, sz, vp, ctypes.c_int], None),
            ("orb_pairing", [c, c, vp], None),
            ("orb_pairing_ref", [c, c, vp], None),
            ("orb_gt_pow", [c, c, sz, vp], None),
            ("orb_gt_mul", [c, c, vp], None),
            ("orb_g1_mul", [c, c, sz, vp], None),
            ("orb_g2_mul", [c, c, sz, vp], None),
            ("orb_g1_add", [c, c, vp], None),
            ("orb_g2_add", [c, c, vp], None),
            ("orb_g1_compress", [c, vp], None),
            ("orb_g2_compress", [c, vp], None),
            ("orb_g1_generator", [vp], None),
            ("orb_g2_generator", [vp], None),
            ("orb_hard_exponent", [vp], None),
        ]:
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _lib = L
    return _lib


def _buf(n):
    return ctypes.create_string_buffer(n)


def sha256(m):
    o = _buf(32)
    lib().orb_sha256(m, len(m), o)
    return o.raw


def expand_xmd(msg, dst, n):
    o = _buf(n)
    lib().orb_expand_message_xmd(msg, len(msg), dst, len(dst), o, n)
    return o.raw


def hash_to_g1(msg, dst=DST_NUL):
    o = _buf(96)
    lib().orb_hash_to_g1(msg, len(msg), dst, len(dst), o)
    return o.raw


def keygen(sk):
    o = _buf(96)
    rc = lib().orb_keygen(sk, o)
    return rc, o.raw


def sign(sk, msg, dst=DST_NUL):
    o = _buf(48)
    lib().orb_sign(sk, msg, len(msg), dst, len(dst), o)
    return o.raw


def g1_decompress(b):
    o, inf = _buf(96), ctypes.c_int(0)
    rc = lib().orb_g1_decompress(b, o, ctypes.byref(inf))
    return rc, (None if rc else (b"\0" * 96 if inf.value else o.raw))


def g2_decompress(b):
    o, inf = _buf(192), ctypes.c_int(0)
    rc = lib().orb_g2_decompress(b, o, ctypes.byref(inf))
    return rc, (None if rc else (b"\0" * 192 if inf.value else o.raw))


def verify(pk, msg, sig, dst=DST_NUL):
    return lib().orb_verify(pk, msg, len(msg), sig, dst, len(dst))


def aggregate(sigs):
    o = _buf(48)
    rc = lib().orb_aggregate(len(sigs), b"".join(sigs), o)
    return rc, o.raw


def aggregate_pubkeys(pks):
    o = _buf(96)
    rc = lib().orb_aggregate_pubkeys(len(pks), b"".join(pks), o)
    return rc, o.raw


def fast_aggregate_verify(sig, pks, msg, dst=DST_NUL):
    return lib().orb_fast_aggregate_verify(sig, len(pks), b"".join(pks), msg, len(msg), dst, len(dst))


def verify_items(keys, sigs, key_lists, msgs, threads=None, dst=DST_NUL):
    """orb_fast_aggregate_verify's status per item with the key table validated once:
    item i = (sigs[i], [keys[k] for k in key_lists[i]], msgs[i]) -> list of ORB_* codes"""
    import numpy as np
    n = len(sigs)
    kb = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
    sg = np.frombuffer(b"".join(sigs) or b"\0", dtype=np.uint8)
    cnt = np.array([len(k) for k in key_lists] or [0], dtype=np.uint32)
    off = np.zeros(max(n, 1), dtype=np.uint32)
    if n > 1:
        off[1:] = np.cumsum(cnt[:-1], dtype=np.uint32)
    idx = np.array([k for ks in key_lists for k in ks] or [0], dtype=np.uint32)
    arena = np.frombuffer(b"".join(msgs) + b"\0" * 8, dtype=np.uint8)
    lens = np.array([len(m) for m in msgs] or [0], dtype=np.uint32)
    moff = np.zeros(max(n, 1), dtype=np.uint64)
    if n > 1:
        moff[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    st = np.zeros(max(n, 1), dtype=np.int32)
    threads = threads or min(16, os.cpu_count() or 1)
    lib().orb_verify_items_keytab_mt(len(keys), kb.ctypes.data, n, sg.ctypes.data, off.ctypes.data, cnt.ctypes.data,
                                     idx.ctypes.data, arena.ctypes.data, moff.ctypes.data, lens.ctypes.data, dst,
                                     len(dst), st.ctypes.data, threads)
    return [int(x) for x in st[:n]]


def pairing(P, Q):
    o = _buf(576)
    lib().orb_pairing(P, Q, o)
    return o.raw


def pairing_ref(P, Q):
    o = _buf(576)
    lib().orb_pairing_ref(P, Q, o)
    return o.raw


def gt_pow(a, e):
    eb = e.to_bytes(max(1, (e.bit_length() + 7) // 8), "big")
    o = _buf(576)
    lib().orb_gt_pow(a, eb, len(eb), o)
    return o.raw


def gt_mul(a, b):
    o = _buf(576)
    lib().orb_gt_mul(a, b, o)
    return o.raw


def g1_mul(P, k):
    kb = k.to_bytes(max(1, (k.bit_length() + 7) // 8), "big")
    o = _buf(96)
    lib().orb_g1_mul(P, kb, len(kb), o)
    return o.raw


def g2_mul(Q, k):
    kb = k.to_bytes(max(1, (k.bit_length() + 7) // 8), "big")
    o = _buf(192)
    lib().orb_g2_mul(Q, kb, len(kb), o)
    return o.raw


def g1_add(a, b):
    o = _buf(96)
    lib().orb_g1_add(a, b, o)
    return o.raw


def g2_add(a, b):
    o = _buf(192)
    lib().orb_g2_add(a, b, o)
    return o.raw


def g1_compress(P):
    o = _buf(48)
    lib().orb_g1_compress(P, o)
    return o.raw


def g2_compress(Q):
    o = _buf(96)
    lib().orb_g2_compress(Q, o)
    return o.raw


def g1_gen():
    o = _buf(96)
    lib().orb_g1_generator(o)
    return o.raw


def g2_gen():
    o = _buf(192)
    lib().orb_g2_generator(o)
    return o.raw


def hard_exponent():
    o = _buf(160)
    lib().orb_hard_exponent(o)
    return int.from_bytes(o.raw, "big")
