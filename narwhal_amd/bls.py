"""ctypes view of the BLS12-381 engine (include/nwv_bls.h, SURVEY.md §8 row f4: the reference's
default signature scheme, crypto/src/lib.rs:29-33 -> fastcrypto 0.1.2 bls12381 / blst min_sig).

Mirrors the fastcrypto trait surface the reference's call sites use (Verifier::verify,
AggregateAuthenticator::{aggregate, verify, batch_verify}, VerifyingKey::verify_batch_empty_fail)
plus the batch entry point (one fast_aggregate_verify per item, exact per-item statuses)."""
import ctypes

import numpy as np

from . import _lib

DST = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"
OK, BAD_ENCODING, NOT_ON_CURVE, NOT_IN_GROUP, AGGR_MISMATCH, VERIFY_FAIL, PK_INFINITY = range(7)

_vp, _sz, _i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32
_SIGS = {
    "nwv_bls_verify_many": ([_vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp], _i32),
    "nwv_bls_verify": ([_vp, _vp, _vp, _sz, _vp], _i32),
    "nwv_bls_aggregate_verify": ([_vp, _vp, _vp, _sz, _vp, _sz], _i32),
    "nwv_bls_verify_batch_empty_fail": ([_vp, _vp, _sz, _vp, _sz, _vp, _sz], _i32),
    "nwv_bls_aggregate_batch_verify": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp, _sz], _i32),
    "nwv_bls_aggregate": ([_vp, _sz, _vp, _vp, _vp], _i32),
    "nwv_bls_keygen_many": ([_vp, _sz, _vp, _vp], _i32),
    "nwv_bls_sign_many": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp, _sz, _vp], _i32),
    "nwv_bls_hash_to_g1_many": ([_vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp], _i32),
    "nwv_bls_pairing_many": ([_vp, _sz, _vp, _vp, _vp], _i32),
    "nwv_bls_last_kernel_ms": ([_vp, _vp], _i32),
    "nwv_bls_last_path": ([_vp], _i32),
    "nwv_bls_last_keys": ([_vp, _vp], _i32),
    "nwv_bls_keycache_register": ([_vp, _sz, _vp], _i32),
    "nwv_bls_keycache_reset": ([_vp], _i32),
    "nwv_bls_keycache_size": ([_vp], _i32),
}
KERNELS = ("keys_new_to_cache", "sig_decode", "hash_to_g1", "key_sums", "pairing_check")
PATHS = ("per_item", "batch_accepted", "batch_rejected_then_per_item", "wave")
_bound = set()


def _bind(lib):
    if id(lib) in _bound:
        return lib
    for name, (args, res) in _SIGS.items():
        f = getattr(lib, name)
        f.argtypes, f.restype = args, res
    _bound.add(id(lib))
    return lib


def _arr(b, dtype=np.uint8):
    a = np.frombuffer(bytes(b) or b"\0", dtype=dtype)
    return a


def _msgs(msgs):
    arena = np.frombuffer(b"".join(msgs) + b"\0" * 8, dtype=np.uint8)
    lens = np.array([len(m) for m in msgs], dtype=np.uint32)
    offs = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return arena, offs, lens


class Bls:
    """BLS12-381 verification on the engine's first device (the context of `engine`)."""

    def __init__(self, engine):
        self.eng = engine
        self.lib = _bind(engine.lib)

    @property
    def _h(self):
        return self.eng._h

    def verify_many(self, keys, sigs, key_lists, msgs, dst=None):
        """item i: fast_aggregate_verify(sigs[i], [keys[k] for k in key_lists[i]], msgs[i]) ->
        numpy int32 statuses (NWV_BLS_*)"""
        n = len(sigs)
        kb = _arr(b"".join(keys))
        sg = _arr(b"".join(sigs))
        cnt = np.array([len(k) for k in key_lists], dtype=np.uint32)
        off = np.zeros(n, dtype=np.uint32)
        if n > 1:
            off[1:] = np.cumsum(cnt[:-1], dtype=np.uint32)
        idx = np.array([k for ks in key_lists for k in ks] or [0], dtype=np.uint32)
        arena, offs, lens = _msgs(msgs)
        st = np.zeros(max(1, n), dtype=np.int32)
        _lib._check(self.lib.nwv_bls_verify_many(
            self._h, len(keys), kb.ctypes.data, n, sg.ctypes.data, off.ctypes.data, cnt.ctypes.data,
            idx.ctypes.data, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, dst,
            len(dst) if dst else 0, st.ctypes.data))
        return st[:n]

    def verify_many_arrays(self, keys, sigs, pk_off, pk_cnt, pk_idx, arena, offs, lens, status, dst=None):
        """the same over prepared numpy arrays (bench / large batches)"""
        _lib._check(self.lib.nwv_bls_verify_many(
            self._h, len(keys) // 96, keys.ctypes.data, len(offs), sigs.ctypes.data, pk_off.ctypes.data,
            pk_cnt.ctypes.data, pk_idx.ctypes.data, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, dst,
            len(dst) if dst else 0, status.ctypes.data))
        return status

    def last_kernel_ms(self):
        """{kernel: device ms} of the last verify_many call"""
        out = np.zeros(5, dtype=np.float64)
        _lib._check(self.lib.nwv_bls_last_kernel_ms(self._h, out.ctypes.data))
        return dict(zip(KERNELS, (float(x) for x in out)))

    def last_keys(self):
        """(key-list entries the last verify_many found in the key cache, keys it decoded itself)"""
        out = np.zeros(2, dtype=np.uint64)
        _lib._check(self.lib.nwv_bls_last_keys(self._h, out.ctypes.data))
        return int(out[0]), int(out[1])

    def last_path(self):
        """how the last verify_many checked its pairings (PATHS)"""
        return PATHS[_lib._check(self.lib.nwv_bls_last_path(self._h), allow=(0, 1, 2, 3))]

    # the committee key cache: register at epoch start, reset at an epoch change
    def register_keys(self, keys):
        kb = _arr(b"".join(keys))
        _lib._check(self.lib.nwv_bls_keycache_register(self._h, len(keys), kb.ctypes.data))

    def reset_keys(self):
        _lib._check(self.lib.nwv_bls_keycache_reset(self._h))

    def cached_keys(self):
        return _lib._check(self.lib.nwv_bls_keycache_size(self._h), allow=range(0, 1 << 20))

    # fastcrypto trait surface: return codes NWV_OK / NWV_ERR_*
    def verify(self, pk, msg, sig):
        return self.lib.nwv_bls_verify(self._h, pk, msg, len(msg), sig)

    def aggregate_verify(self, sig_or_none, pks, msg):
        return self.lib.nwv_bls_aggregate_verify(self._h, sig_or_none, b"".join(pks) or None, len(pks), msg, len(msg))

    def verify_batch_empty_fail(self, msg, pks, sigs):
        return self.lib.nwv_bls_verify_batch_empty_fail(self._h, msg, len(msg), b"".join(pks) or None, len(pks),
                                                        b"".join(sigs) or None, len(sigs))

    def aggregate_batch_verify(self, sigs, pks_lists, msgs):
        n = len(sigs)
        keep = [b"".join(p) or b"\0" for p in pks_lists]
        arr = lambda xs: (ctypes.c_char_p * max(1, len(xs)))(*xs)
        szs = lambda xs: (ctypes.c_size_t * max(1, len(xs)))(*xs)
        return self.lib.nwv_bls_aggregate_batch_verify(
            self._h, n, arr(sigs), arr(keep), szs([len(p) for p in pks_lists]), arr(msgs),
            szs([len(m) for m in msgs]), len(msgs))

    def aggregate(self, sigs):
        """-> (rc, aggregate 48 bytes or None, status)"""
        out = ctypes.create_string_buffer(48)
        st = ctypes.c_int32(0)
        rc = self.lib.nwv_bls_aggregate(self._h, len(sigs), b"".join(sigs) or None, out, ctypes.byref(st))
        return rc, (out.raw if rc == 0 else None), st.value

    # keys, signatures and primitives
    def keygen(self, sks):
        out = np.zeros(96 * len(sks), dtype=np.uint8)
        _lib._check(self.lib.nwv_bls_keygen_many(self._h, len(sks), b"".join(sks), out.ctypes.data))
        return [out[96 * i:96 * (i + 1)].tobytes() for i in range(len(sks))]

    def sign(self, sks, msgs, dst=None):
        arena, offs, lens = _msgs(msgs)
        out = np.zeros(48 * len(sks), dtype=np.uint8)
        _lib._check(self.lib.nwv_bls_sign_many(self._h, len(sks), b"".join(sks), arena.ctypes.data,
                                               offs.ctypes.data, lens.ctypes.data, dst, len(dst) if dst else 0,
                                               out.ctypes.data))
        return [out[48 * i:48 * (i + 1)].tobytes() for i in range(len(sks))]

    def hash_to_g1(self, msgs, dst=None):
        arena, offs, lens = _msgs(msgs)
        out = np.zeros(96 * len(msgs), dtype=np.uint8)
        _lib._check(self.lib.nwv_bls_hash_to_g1_many(self._h, len(msgs), arena.ctypes.data, offs.ctypes.data,
                                                     lens.ctypes.data, dst, len(dst) if dst else 0,
                                                     out.ctypes.data))
        return [out[96 * i:96 * (i + 1)].tobytes() for i in range(len(msgs))]

    def pairing(self, Ps, Qs):
        out = np.zeros(576 * len(Ps), dtype=np.uint8)
        _lib._check(self.lib.nwv_bls_pairing_many(self._h, len(Ps), b"".join(Ps), b"".join(Qs), out.ctypes.data))
        return [out[576 * i:576 * (i + 1)].tobytes() for i in range(len(Ps))]
