"""ctypes binding of the C ABI in include/nwv.h (narwhal_amd/lib/libnwv.so).

This is the Python-side view of the drop-in boundary used by the tests and bench.py.  The
library runs every verification on the GPU; loading fails loudly when the HIP extension has
not been built (there is no CPU fallback anywhere in this package).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NWV_LIB selects an in-tree build variant (e.g. lib/libnwv_exp.so) for A/B measurements
LIB_PATH = os.path.join(_HERE, "lib", os.environ.get("NWV_LIB", "libnwv.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "nwv.h")

NWV_OK = 0
NWV_ERR_SIGNATURE = 1
NWV_ERR_ARG = -1
NWV_ERR_HIP = -2
NWV_ERR_OOM = -3
NWV_ERR_NODEV = -4
NWV_ERR_EMPTY = -5
NWV_ERR_LENGTH = -6
NWV_ERR_REENTRANT = -7
NWV_FLAG_MSM_ALWAYS = 1
NWV_FLAG_MSM_NEVER = 2
NWV_FLAG_MSM_SPLIT_PREP = 4
NWV_FLAG_NO_KEYCACHE = 8
NWV_FLAG_MSM_SORT2 = 16
NWV_FLAG_NO_MSM_REUSE = 32
NWV_FLAG_BLS_PER_ITEM = 64
NWV_FLAG_BLS_BATCH = 128
NWV_FLAG_NO_SIGCACHE = 256
NWV_FLAG_NO_ROW_PREP = 512
NWV_FLAG_NO_EARLY_PREP = 1024
NWV_FLAG_NO_FUSED_KEYSUM = 2048
NWV_FLAG_NO_TINY = 4096
NWV_FLAG_BLS_STAGE_TIMES = 8192  # per-stage timing events on small BLS calls (nwv_bls_last_kernel_ms)
NWV_RUN_TIMED = 0x100


class NwvError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"nwv error {code}: {msg}")
        self.code = code


_lib = None
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i32 = ctypes.c_int


def load():
    """Load libnwv.so (raises if the HIP library was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make lib` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "nwv_init": ([ctypes.POINTER(_vp), _i32, ctypes.c_uint32], _i32),
        "nwv_init_device": ([ctypes.POINTER(_vp), _i32, ctypes.c_uint32], _i32),
        "nwv_free": ([_vp], None),
        "nwv_device_count": ([_vp], _i32),
        "nwv_diag_counters": ([_vp, _vp], _i32),
        "nwv_abi_version": ([], _i32),
        "nwv_last_error": ([], ctypes.c_char_p),
        "nwv_ed25519_verify_each": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp], _i32),
        "nwv_ed25519_verify_batch": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i32),
        "nwv_ed25519_pubkey_verify": ([_vp, _vp, _vp, _sz, _vp], _i32),
        "nwv_keycache_register": ([_vp, _sz, _vp], _i32),
        "nwv_ed25519_verify_batch_empty_fail": ([_vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp], _i32),
        "nwv_ed25519_aggregate_verify": ([_vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp], _i32),
        "nwv_ed25519_aggregate_batch_verify": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp], _i32),
        "nwv_blake2b256_many": ([_vp, _sz, _vp, _vp, _vp, _vp], _i32),
        "nwv_batch_digest_serialized": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp], _i32),
        "nwv_stage_ed25519": ([_vp, _i32, _sz, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)], _i32),
        "nwv_stage_ed25519_keyed": ([_vp, _i32, _sz, _vp, _sz, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)], _i32),
        "nwv_ed25519_verify_batch_keyed": ([_vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i32),
        "nwv_ed25519_verify_batch_keyed_digests": ([_vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp,
                                                    _vp, _vp], _i32),
        "nwv_staged_run": ([_vp, _i32, _vp], _i32),
        "nwv_staged_sync": ([_vp], _i32),
        "nwv_staged_fetch": ([_vp, _vp, ctypes.POINTER(_i32)], _i32),
        "nwv_staged_kernel_ms": ([_vp, _vp, _i32], _i32),
        "nwv_staged_kernel_times": ([_vp, _i32, _i32, _vp, _vp, _i32], _i32),
        "nwv_staged_free": ([_vp], None),
        "nwv_staged_msm_stats": ([_vp, _vp], _i32),
        "nwv_staged_run_tally": ([_vp, _vp], _i32),
        "nwv_staged_mark": ([_vp, _i32], _i32),
        "nwv_staged_mark_elapsed": ([_vp, _i32, _vp, _i32, ctypes.POINTER(ctypes.c_float)], _i32),
        "nwv_ed25519_sign_many": ([_vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp], _i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _lib = lib
    return lib


def bls_source_hash():
    """sha256 (16 hex digits) over the BLS12-381 device sources (nwv_bls.hip, bls*.h and the wave
    tables bls_wave_prog.h): committed BLS rocprofv3 --pmc summaries carry it"""
    import glob
    import hashlib
    h = hashlib.sha256()
    fs = glob.glob(os.path.join(_HERE, "csrc", "bls*.h")) + [os.path.join(_HERE, "csrc", "nwv_bls.hip")]
    for f in sorted(fs):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def kernel_source_hash():
    """sha256 (16 hex digits) over the Ed25519 / BLAKE2b device-code sources (narwhal_amd/csrc/*.hip,
    *.h; the BLS12-381 translation unit nwv_bls.hip and its bls*.h headers are not part of those
    kernels and are left out): committed rocprofv3 --pmc summaries carry it, and bench.py uses a
    summary only while it matches, so counters of kernels that have since changed are never
    priced against today's timings"""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.h"))):
        b = os.path.basename(f)
        if b.startswith("bls") or b == "nwv_bls.hip":
            continue
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def exported_symbols_from_header():
    """Every function name declared in include/*.h (nwv.h and nwv_types.h)."""
    import glob
    import re
    names = set()
    for h in glob.glob(os.path.join(os.path.dirname(HEADER_PATH), "*.h")):
        with open(h) as f:
            names |= set(re.findall(r"\b(nwv_[a-z0-9_]+)\s*\(", f.read()))
    return sorted(names)


def _check(rc, allow=(NWV_OK,)):
    if rc not in allow:
        raise NwvError(rc, load().nwv_last_error().decode(errors="replace"))
    return rc


def _seed(seed):
    """None -> NULL, so the library draws the batch coefficients' key from OS entropy (the
    reference's OsRng).  A given seed must be exactly 32 bytes: the C side reads 32."""
    if seed is None:
        return None
    seed = bytes(seed)
    if len(seed) != 32:
        raise ValueError(f"seed must be 32 bytes, got {len(seed)}")
    return seed


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def pack_messages(msgs):
    """list of bytes -> (arena uint8 (padded), offsets uint64, lengths uint32)"""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint32, count=len(msgs))
    offs = np.zeros(len(msgs), dtype=np.uint64)
    if len(msgs):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
    return arena, offs, lens


class Engine:
    """A context over one device (device=k) or the first n_devices (device=None)."""

    def __init__(self, device=None, n_devices=0, flags=0):
        lib = load()
        h = _vp()
        if device is None:
            _check(lib.nwv_init(ctypes.byref(h), n_devices, flags))
        else:
            _check(lib.nwv_init_device(ctypes.byref(h), device, flags))
        self._h = h
        self.lib = lib
        self.device = device  # the HIP ordinal (None: a context over the first n_devices)

    def close(self):
        if self._h:
            self.lib.nwv_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device_count(self):
        return self.lib.nwv_device_count(self._h)

    def diag_counters(self):
        """{'tiny': one-launch keyed batches, 'msm': batch MSMs, 'each': per-signature passes}"""
        out = np.zeros(3, dtype=np.uint64)
        _check(self.lib.nwv_diag_counters(self._h, out.ctypes.data))
        return {"tiny": int(out[0]), "msm": int(out[1]), "each": int(out[2])}

    def keycache_register(self, keys):
        """nwv_keycache_register: keys, a list of 32-byte keys (the committee, at epoch start)"""
        kb = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
        _check(self.lib.nwv_keycache_register(self._h, len(keys), _ptr(kb)))

    # ---- Ed25519 ---------------------------------------------------------------------
    def verify_each_arrays(self, pk, sig, arena, offs, lens):
        """pk: uint8 [n*32], sig: uint8 [n*64] -> bool array of per-signature verdicts"""
        n = len(offs)
        bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
        _check(self.lib.nwv_ed25519_verify_each(self._h, n, _ptr(pk), _ptr(sig), _ptr(arena),
                                                _ptr(offs), _ptr(lens), _ptr(bits)))
        return unpack_bits(bits, n)

    def verify_each(self, items):
        """items: list of (pk32, sig64, msg) -> list of bool"""
        pk, sig, arena, offs, lens = soa(items)
        return list(self.verify_each_arrays(pk, sig, arena, offs, lens))

    def verify_batch(self, items, seed=None, want_bits=True):
        pk, sig, arena, offs, lens = soa(items)
        n = len(items)
        bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
        allv = _i32(0)
        _check(self.lib.nwv_ed25519_verify_batch(self._h, n, _ptr(pk), _ptr(sig), _ptr(arena),
                                                 _ptr(offs), _ptr(lens), _seed(seed), ctypes.byref(allv),
                                                 _ptr(bits) if want_bits else None))
        return bool(allv.value), (list(unpack_bits(bits, n)) if want_bits else None)

    def verify_batch_keyed(self, keys, key_idx, sigs, msgs, seed=None, want_bits=True):
        """keys: list of distinct 32-byte keys; key_idx[i]: key of signature i; sigs, msgs: per
        signature -> (all_valid, per-signature verdicts or None)"""
        n = len(sigs)
        kb = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
        ki = np.asarray(key_idx, dtype=np.uint32)
        sg = np.frombuffer(b"".join(sigs) or b"\0", dtype=np.uint8)
        arena, offs, lens = pack_messages(list(msgs))
        bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
        allv = _i32(0)
        _check(self.lib.nwv_ed25519_verify_batch_keyed(self._h, len(keys), _ptr(kb), n, _ptr(ki), _ptr(sg),
                                                       _ptr(arena), _ptr(offs), _ptr(lens), _seed(seed),
                                                       ctypes.byref(allv), _ptr(bits) if want_bits else None))
        return bool(allv.value), (list(unpack_bits(bits, n)) if want_bits else None)

    def verify_batch_keyed_digests(self, preimages, keys, key_idx, sigs, digest_idx, seed=None):
        """BLAKE2b-256 of every preimage on the device, then signature i over digest digest_idx[i]
        -> (digests, all_valid, per-signature verdicts)"""
        n, m = len(sigs), len(preimages)
        lens = np.fromiter((len(x) for x in preimages), dtype=np.uint64, count=m)
        offs = np.zeros(m, dtype=np.uint64)
        if m:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(preimages) + b"\0" * 16, dtype=np.uint8)
        dig = np.zeros(32 * max(m, 1), dtype=np.uint8)
        kb = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
        ki = np.asarray(key_idx, dtype=np.uint32)
        di = np.asarray(digest_idx, dtype=np.uint32)
        sg = np.frombuffer(b"".join(sigs) or b"\0", dtype=np.uint8)
        bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
        allv = _i32(0)
        _check(self.lib.nwv_ed25519_verify_batch_keyed_digests(
            self._h, m, _ptr(arena), _ptr(offs), _ptr(lens), _ptr(dig), len(keys), _ptr(kb), n, _ptr(ki),
            _ptr(sg), _ptr(di), _seed(seed), ctypes.byref(allv), _ptr(bits)))
        return [dig[32 * i:32 * i + 32].tobytes() for i in range(m)], bool(allv.value), list(unpack_bits(bits, n))

    def stage_keyed(self, keys, key_idx, sig, arena, offs, lens, device_index=0):
        """keys: uint8 [m*32]; key_idx: uint32 [n]; sig uint8 [n*64]"""
        st = _vp()
        m = len(keys) // 32
        _check(self.lib.nwv_stage_ed25519_keyed(self._h, device_index, m, _ptr(keys), len(offs), _ptr(key_idx),
                                                _ptr(sig), _ptr(arena), _ptr(offs), _ptr(lens), ctypes.byref(st)))
        return Staged(self, st, len(offs))

    def sign_many(self, seeds, msgs):
        n = len(seeds)
        arena, offs, lens = pack_messages(msgs)
        sd = np.frombuffer(b"".join(seeds), dtype=np.uint8)
        pk = np.zeros(32 * n, dtype=np.uint8)
        sg = np.zeros(64 * n, dtype=np.uint8)
        _check(self.lib.nwv_ed25519_sign_many(self._h, n, _ptr(sd), _ptr(arena), _ptr(offs),
                                              _ptr(lens), _ptr(pk), _ptr(sg)))
        return pk, sg

    def sign_many_arrays(self, seeds, arena, offs, lens):
        n = len(offs)
        pk = np.zeros(32 * n, dtype=np.uint8)
        sg = np.zeros(64 * n, dtype=np.uint8)
        _check(self.lib.nwv_ed25519_sign_many(self._h, n, _ptr(seeds), _ptr(arena), _ptr(offs),
                                              _ptr(lens), _ptr(pk), _ptr(sg)))
        return pk, sg

    def stage(self, pk, sig, arena, offs, lens, device_index=0):
        st = _vp()
        _check(self.lib.nwv_stage_ed25519(self._h, device_index, len(offs), _ptr(pk), _ptr(sig),
                                          _ptr(arena), _ptr(offs), _ptr(lens), ctypes.byref(st)))
        return Staged(self, st, len(offs))

    # ---- BLAKE2b ---------------------------------------------------------------------
    def blake2b256_many(self, msgs):
        n = len(msgs)
        lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n)
        offs = np.zeros(n, dtype=np.uint64)
        if n:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
        out = np.zeros(32 * max(n, 1), dtype=np.uint8)
        _check(self.lib.nwv_blake2b256_many(self._h, n, _ptr(arena), _ptr(offs), _ptr(lens), _ptr(out)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]

    def batch_digest_serialized(self, bufs):
        """-> list of (digest or None, err_offset)"""
        n = len(bufs)
        lens = np.fromiter((len(m) for m in bufs), dtype=np.uint64, count=n)
        offs = np.zeros(n, dtype=np.uint64)
        if n:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(bufs) + b"\0" * 16, dtype=np.uint8)
        out = np.zeros(32 * max(n, 1), dtype=np.uint8)
        err = np.zeros(max(n, 1), dtype=np.int64)
        _check(self.lib.nwv_batch_digest_serialized(self._h, n, _ptr(arena), _ptr(offs), _ptr(lens),
                                                    _ptr(out), _ptr(err)),
               allow=(NWV_OK, NWV_ERR_ARG))
        return [(out[32 * i:32 * i + 32].tobytes() if err[i] < 0 else None, int(err[i])) for i in range(n)]


class Staged:
    """Device-resident Ed25519 batch (inputs already in HBM)."""

    def __init__(self, eng, h, n):
        self.eng, self._h, self.n = eng, h, n

    def run(self, mode=0, seed=None, timed=False):
        """mode 0 per-signature pipeline, 1 batch MSM (graph replay); timed: kernel-by-kernel
        launches bracketed by HIP events (feeds kernel_ms / kernel_times)"""
        _check(self.eng.lib.nwv_staged_run(self._h, mode | (NWV_RUN_TIMED if timed else 0), _seed(seed)))

    def sync(self):
        _check(self.eng.lib.nwv_staged_sync(self._h))

    def fetch(self):
        bits = np.zeros((self.n + 63) // 64 + 1, dtype=np.uint64)
        allv = _i32(0)
        _check(self.eng.lib.nwv_staged_fetch(self._h, _ptr(bits), ctypes.byref(allv)))
        return bool(allv.value), unpack_bits(bits, self.n)

    def kernel_ms(self, reset=True):
        out = np.zeros(3, dtype=np.float64)
        _check(self.eng.lib.nwv_staged_kernel_ms(self._h, _ptr(out), 1 if reset else 0))
        return out

    def kernel_times(self, mode, reset=True):
        """{kernel name: average device ms} of the mode-`mode` pipeline since the last reset"""
        cap = 32
        names = (ctypes.c_char_p * cap)()
        ms = np.zeros(cap, dtype=np.float64)
        k = self.eng.lib.nwv_staged_kernel_times(self._h, mode, cap, names, _ptr(ms), 1 if reset else 0)
        if k < 0:
            _check(k)
        return {names[i].decode(): float(ms[i]) for i in range(min(k, cap))}

    def msm_stats(self):
        """{points, windows, windows_z, buckets, entries, chunks, seg, a_points} of the batch MSM"""
        out = np.zeros(8, dtype=np.uint64)
        _check(self.eng.lib.nwv_staged_msm_stats(self._h, _ptr(out)))
        keys = ("points", "windows", "windows_z", "buckets", "entries", "chunks", "seg", "a_points")
        return {k: int(v) for k, v in zip(keys, out)}

    def run_tally(self):
        """(accepted, rejected) batch verdicts of every mode-1 run since staging, counted on the
        device by each run (graph replays included)"""
        out = np.zeros(2, dtype=np.uint64)
        _check(self.eng.lib.nwv_staged_run_tally(self._h, _ptr(out)))
        return int(out[0]), int(out[1])

    def mark(self, slot):
        """record step-completion event `slot` on this batch's stream"""
        _check(self.eng.lib.nwv_staged_mark(self._h, slot))

    def mark_elapsed(self, slot, other, other_slot):
        """device ms from this batch's mark `slot` to `other`'s mark `other_slot`"""
        ms = ctypes.c_float(0)
        _check(self.eng.lib.nwv_staged_mark_elapsed(self._h, slot, other._h, other_slot, ctypes.byref(ms)))
        return ms.value

    def free(self):
        if self._h:
            self.eng.lib.nwv_staged_free(self._h)
            self._h = None


def unpack_bits(bits, n):
    b = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n]
    return b.astype(bool)


def soa(items):
    n = len(items)
    pk = np.frombuffer(b"".join(x[0] for x in items) or b"\0", dtype=np.uint8)
    sig = np.frombuffer(b"".join(x[1] for x in items) or b"\0", dtype=np.uint8)
    arena, offs, lens = pack_messages([x[2] for x in items])
    assert pk.size >= 32 * n and sig.size >= 64 * n
    return pk, sig, arena, offs, lens
