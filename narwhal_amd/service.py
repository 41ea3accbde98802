"""Batching verification service (include/nwv_service.h) over ctypes.

Python view of the in-library coalescer in front of Core::sanitize_header / sanitize_vote /
sanitize_certificate (primary/src/core.rs:497-573): threads call verify_header / verify_vote /
verify_certificate (blocking; the GIL is released while waiting) or submit_* with a callback; the
library's flusher threads verify whatever is pending as ONE nwv_verify_mixed_many call and hand
each caller its own DagError code (0 = Ok, types/src/error.rs), exactly what Header::verify,
Vote::verify and Certificate::verify (types/src/primary.rs:150-183, :307-328, :487-537) return.
"""
import ctypes
import itertools

import numpy as np

from . import _lib
from . import types as T

DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32)

_SIGS = {
    "nwv_service_create": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                            ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "nwv_service_set_committee": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_submit_header": ([ctypes.c_void_p, ctypes.c_void_p, DONE_FN, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_submit_vote": ([ctypes.c_void_p, ctypes.c_void_p, DONE_FN, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_submit_certificate": ([ctypes.c_void_p, ctypes.c_void_p, DONE_FN, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_verify_header": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "nwv_service_verify_vote": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "nwv_service_verify_certificate": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)],
                                       ctypes.c_int),
    "nwv_service_create_bls": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "nwv_service_set_committee_bls": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_submit_bls_header": ([ctypes.c_void_p, ctypes.c_void_p, DONE_FN, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_submit_bls_vote": ([ctypes.c_void_p, ctypes.c_void_p, DONE_FN, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_submit_bls_certificate": ([ctypes.c_void_p, ctypes.c_void_p, DONE_FN, ctypes.c_void_p],
                                           ctypes.c_int),
    "nwv_service_verify_bls_header": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)],
                                      ctypes.c_int),
    "nwv_service_verify_bls_vote": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "nwv_service_verify_bls_certificate": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)],
                                           ctypes.c_int),
    "nwv_service_set_idle": ([ctypes.c_void_p, ctypes.c_uint32], ctypes.c_int),
    "nwv_service_flush": ([ctypes.c_void_p], ctypes.c_int),
    "nwv_service_stats": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_service_free": ([ctypes.c_void_p], None),
}


def bind(lib):
    """declare the service entry points on a loaded library (libnwv.so, or the CPU test stub)"""
    if not getattr(lib, "_service_bound", False):
        for name, (args, res) in _SIGS.items():
            f = getattr(lib, name)
            f.argtypes = args
            f.restype = res
        lib._service_bound = True
    return lib


class Service:
    """One batching service over an Engine's context (or any nwv_ctx handle with lib).

    scheme='bls': the reference's default scheme (crypto/src/lib.rs:29-33), BLS12-381 -- items are
    types.Header / Vote with 96-byte keys and 48-byte signatures and types.BlsCertificate; each
    flush is one nwv_bls_verify_mixed_many call (nwv_service_create_bls)."""

    def __init__(self, engine, committee, max_batch=256, max_wait_us=200, lib=None, ctx=None, scheme="ed25519",
                 idle_us=0):
        if scheme not in ("ed25519", "bls"):
            raise ValueError("scheme must be 'ed25519' or 'bls'")
        self.lib = bind(lib if lib is not None else _lib.load())
        self.scheme = scheme
        self._p = "bls_" if scheme == "bls" else ""
        self._keep = T._Keep()
        cc = committee._c(self._keep)
        h = ctypes.c_void_p()
        create = self.lib.nwv_service_create_bls if scheme == "bls" else self.lib.nwv_service_create
        rc = create(ctx if ctx is not None else engine._h, ctypes.byref(cc), max_batch, max_wait_us, ctypes.byref(h))
        if rc:
            raise _lib.NwvError(rc, "nwv_service_create")
        self._h = h
        if idle_us:
            _lib._check(self.lib.nwv_service_set_idle(h, idle_us))
        self._callbacks = {}
        self._keys = itertools.count()

    def close(self):
        if self._h:
            self.lib.nwv_service_free(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_committee(self, committee):
        keep = T._Keep()
        cc = committee._c(keep)
        fn = self.lib.nwv_service_set_committee_bls if self.scheme == "bls" else self.lib.nwv_service_set_committee
        rc = fn(self._h, ctypes.byref(cc))
        if rc:
            raise _lib.NwvError(rc, "nwv_service_set_committee")

    # blocking forms: the DagError code of the item (the structs are copied by the library)
    def _verify(self, fn, st):
        r = ctypes.c_int32(0)
        rc = fn(self._h, ctypes.byref(st), ctypes.byref(r))
        if rc < 0:
            raise _lib.NwvError(rc, "service verify")
        return r.value

    def verify_header(self, header):
        keep = T._Keep()
        return self._verify(getattr(self.lib, f"nwv_service_verify_{self._p}header"), header._c(keep))

    def verify_vote(self, vote):
        keep = T._Keep()
        return self._verify(getattr(self.lib, f"nwv_service_verify_{self._p}vote"), vote._c(keep))

    def verify_certificate(self, cert):
        keep = T._Keep()
        return self._verify(getattr(self.lib, f"nwv_service_verify_{self._p}certificate"), cert._c(keep))

    # asynchronous forms: done(code) runs on a service thread
    def _submit(self, fn, st, done):
        key = next(self._keys)

        def cb(_user, code, key=key):
            f = self._callbacks.pop(key)
            done(code)
            del f

        c = DONE_FN(cb)
        self._callbacks[key] = c
        rc = fn(self._h, ctypes.byref(st), c, None)
        if rc:
            self._callbacks.pop(key, None)
            raise _lib.NwvError(rc, "service submit")

    def submit_header(self, header, done):
        keep = T._Keep()
        self._submit(getattr(self.lib, f"nwv_service_submit_{self._p}header"), header._c(keep), done)

    def submit_vote(self, vote, done):
        keep = T._Keep()
        self._submit(getattr(self.lib, f"nwv_service_submit_{self._p}vote"), vote._c(keep), done)

    def submit_certificate(self, cert, done):
        keep = T._Keep()
        self._submit(getattr(self.lib, f"nwv_service_submit_{self._p}certificate"), cert._c(keep), done)

    def flush(self):
        _lib._check(self.lib.nwv_service_flush(self._h))

    def stats(self):
        out = np.zeros(6, dtype=np.uint64)
        _lib._check(self.lib.nwv_service_stats(self._h, out.ctypes.data))
        keys = ("calls", "items", "max_batch", "by_count", "by_deadline", "by_flush")
        return {k: int(v) for k, v in zip(keys, out)}



class CoreDrain:
    """Single-consumer coalescer for a Core-shaped loop (Core::run, primary/src/core.rs:614-714):
    the drain pattern of rust/narwhal-gpu-crypto/src/core_drain.rs.  On a message, take whatever
    else is already queued (up to max_items, waiting at most max_wait_us for more), verify the lot
    with ONE nwv_verify_mixed_many call (one digest launch, one batch MSM) and hand back each
    message's DagError code (0 = Ok) in arrival order -- what Header::verify / Vote::verify /
    Certificate::verify (types/src/primary.rs:150-183, :307-328, :487-537) return for it.  The
    loop then runs sanitize_*'s state checks and process_* per message as before: verification
    depends only on the committee, never on Core's state, so verifying ahead changes no outcome.

    A message is (kind, item): kind 'header' | 'vote' | 'certificate', item a types.Header / Vote
    / Certificate or its prepared C struct (types._Header / _Vote / _Certificate).

    scheme='bls': the reference's default scheme (crypto/src/lib.rs:29-33), BLS12-381 -- 96-byte
    keys, 48-byte signatures, certificates as types.BlsCertificate (or _BlsCertificate); the call
    is nwv_bls_verify_mixed_many (single-key checks for headers and votes, one
    fast_aggregate_verify per certificate, all in one BLS verification call)."""

    KINDS = ("header", "vote", "certificate")
    _CLS = {"header": T._Header, "vote": T._Vote, "certificate": T._Certificate}
    _CLS_BLS = {"header": T._Header, "vote": T._Vote, "certificate": T._BlsCertificate}

    def __init__(self, engine, committee, max_items=512, max_wait_us=1000, min_items=64, scheme="ed25519",
                 idle_us=0):
        if max_items < 1:
            raise ValueError("max_items must be >= 1")
        if scheme not in ("ed25519", "bls"):
            raise ValueError("scheme must be 'ed25519' or 'bls'")
        self.scheme = scheme
        self.engine = engine
        self.max_items = max_items
        self.max_wait_us = max_wait_us
        self.min_items = min_items
        self.idle_us = idle_us
        self.set_committee(committee)
        self.calls = self.items = self.largest = 0

    def set_committee(self, committee):
        """epoch change (Core::change_epoch, primary/src/core.rs:592-611)"""
        self._ckeep = T._Keep()
        self._cc = committee._c(self._ckeep)

    def drain(self, q, first=None):
        """`first` (or a blocking q.get()) plus whatever q holds, at most max_items messages; when
        q runs dry it waits for more until the deadline while fewer than min_items are taken, and
        (idle_us > 0) for at most idle_us more once min_items are in: a burst still arriving is
        taken whole, while a big enough batch with nothing behind it goes at once (q: a
        queue.Queue standing in for Core's channels)"""
        import queue
        import time
        out = [q.get() if first is None else first]
        deadline = time.perf_counter() + self.max_wait_us * 1e-6
        while len(out) < self.max_items:
            try:
                out.append(q.get_nowait())
                continue
            except queue.Empty:
                pass
            left = deadline - time.perf_counter()
            if len(out) >= self.min_items:
                left = min(left, self.idle_us * 1e-6)
            if left <= 0:
                break
            try:
                out.append(q.get(timeout=left))
            except queue.Empty:
                break
        return out

    def verify(self, msgs):
        """one engine call for every message -> DagError codes in input order"""
        keep = T._Keep()
        structs = {k: [] for k in self.KINDS}
        where = {k: [] for k in self.KINDS}
        for i, (kind, item) in enumerate(msgs):
            structs[kind].append(item if isinstance(item, ctypes.Structure) else item._c(keep))
            where[kind].append(i)
        args, outs = [], []
        cls = self._CLS_BLS if self.scheme == "bls" else self._CLS
        for k in self.KINDS:
            n = len(structs[k])
            arr = (cls[k] * max(n, 1))(*structs[k])
            res = (ctypes.c_int32 * max(n, 1))()
            keep.objs += [arr, res]
            args += [n, ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(res, ctypes.c_void_p)]
            outs.append(res)
        fn = T.lib().nwv_bls_verify_mixed_many if self.scheme == "bls" else T.lib().nwv_verify_mixed_many
        _lib._check(fn(self.engine._h, ctypes.byref(self._cc), *args))
        codes = [0] * len(msgs)
        for k, res in zip(self.KINDS, outs):
            for j, i in enumerate(where[k]):
                codes[i] = res[j]
        self.calls += 1
        self.items += len(msgs)
        self.largest = max(self.largest, len(msgs))
        return codes

    def next_batch(self, q, first=None):
        """drain + verify: [(message, code)] in arrival order"""
        msgs = self.drain(q, first)
        return list(zip(msgs, self.verify(msgs)))
