"""Narwhal's certificate / header / vote types over the GPU engine (include/nwv_types.h).

Python view of the types crate's verification surface (types/src/primary.rs): Header, Vote and
Certificate with digest() and verify(), Certificate.new / new_unsigned (new_unsafe :427-485),
Certificate.genesis, and validate_certificates (primary/src/block_synchronizer/responses.rs:95-141).
Each call marshals plain byte buffers into the C structs of nwv_types.h; the digests and the
signature checks run on the GPU.  Errors come back as DagError subclasses named after the
reference's variants (types/src/error.rs).
"""
import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from . import _lib

_u8p = ctypes.POINTER(ctypes.c_uint8)


class _Committee(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("keys", ctypes.c_void_p), ("stakes", ctypes.c_void_p),
                ("epoch", ctypes.c_uint64), ("n_workers", ctypes.c_void_p), ("worker_ids", ctypes.c_void_p)]


class _Header(ctypes.Structure):
    _fields_ = [("author", ctypes.c_void_p), ("round", ctypes.c_uint64), ("epoch", ctypes.c_uint64),
                ("n_payload", ctypes.c_size_t), ("payload_digests", ctypes.c_void_p),
                ("payload_workers", ctypes.c_void_p), ("n_parents", ctypes.c_size_t),
                ("parents", ctypes.c_void_p), ("id", ctypes.c_void_p), ("signature", ctypes.c_void_p)]


class _Vote(ctypes.Structure):
    _fields_ = [("id", ctypes.c_void_p), ("round", ctypes.c_uint64), ("epoch", ctypes.c_uint64),
                ("origin", ctypes.c_void_p), ("author", ctypes.c_void_p), ("signature", ctypes.c_void_p)]


class _Certificate(ctypes.Structure):
    _fields_ = [("header", _Header), ("n_signed", ctypes.c_size_t), ("signed_authorities", ctypes.c_void_p),
                ("n_sigs", ctypes.c_size_t), ("aggregated_signature", ctypes.c_void_p)]


# ---- DagError (types/src/error.rs) ------------------------------------------------------
class DagError(Exception):
    code = -1


class InvalidEpoch(DagError):
    code = 10


class InvalidHeaderId(DagError):
    code = 11


class UnknownAuthority(DagError):
    code = 12


class MalformedHeader(DagError):
    code = 13


class InvalidSignature(DagError):
    code = 14


class CertificateRequiresQuorum(DagError):
    code = 15


class InvalidBitmap(DagError):
    code = 16


_ERRORS = {c.code: c for c in (InvalidEpoch, InvalidHeaderId, UnknownAuthority, MalformedHeader,
                               InvalidSignature, CertificateRequiresQuorum, InvalidBitmap)}


def error_for(code):
    """DagError class for an NWV_DAG_* code (None for Ok)."""
    return None if code == 0 else _ERRORS[code]


def _raise(code):
    if code < 0:
        _lib._check(code)
    if code:
        raise _ERRORS[code]()


_SIGS = {
    "nwv_header_digest_many": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_vote_digest_many": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_certificate_digest_many": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_header_verify_many": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_vote_verify_many": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_certificate_verify_many": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_verify_mixed_many": ([ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p] * 3,
                              ctypes.c_int),
    "nwv_validate_certificates": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_certificate_new": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_committee_quorum_threshold": ([ctypes.c_void_p], ctypes.c_uint64),
    "nwv_bls_header_digest_many": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_bls_vote_digest_many": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_bls_certificate_digest_many": ([ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p],
                                        ctypes.c_int),
    "nwv_bls_verify_mixed_many": ([ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_size_t, ctypes.c_void_p,
                                                                         ctypes.c_void_p] * 3, ctypes.c_int),
    "nwv_bls_validate_certificates": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "nwv_bls_certificate_new": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
                                ctypes.c_int),
}


def lib():
    l_ = _lib.load()
    if not getattr(l_, "_types_bound", False):
        for name, (args, res) in _SIGS.items():
            f = getattr(l_, name)
            f.argtypes = args
            f.restype = res
        l_._types_bound = True
    return l_


class _Keep:
    """Owns the ctypes buffers a marshalled struct points into."""

    def __init__(self):
        self.objs = []

    def buf(self, data: bytes):
        b = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
        self.objs.append(b)
        return ctypes.cast(b, ctypes.c_void_p)

    def arr(self, ctype, values):
        a = (ctype * max(len(values), 1))(*values)
        self.objs.append(a)
        return ctypes.cast(a, ctypes.c_void_p)


# ---- types ------------------------------------------------------------------------------
@dataclass
class Committee:
    """config::Committee (+ the worker cache's worker ids): authorities ordered by key bytes."""
    keys: List[bytes]
    stakes: List[int]
    epoch: int = 0
    workers: Optional[List[List[int]]] = None  # worker ids per authority

    def __post_init__(self):
        order = sorted(range(len(self.keys)), key=lambda i: self.keys[i])
        self.keys = [self.keys[i] for i in order]
        self.stakes = [self.stakes[i] for i in order]
        if self.workers is not None:
            self.workers = [list(self.workers[i]) for i in order]

    def index(self, pk):
        try:
            return self.keys.index(pk)
        except ValueError:
            return None

    def stake(self, pk):
        i = self.index(pk)
        return 0 if i is None else self.stakes[i]

    def quorum_threshold(self):
        return 2 * sum(self.stakes) // 3 + 1

    def _c(self, keep):
        c = _Committee()
        c.n = len(self.keys)
        c.keys = keep.buf(b"".join(self.keys))
        c.stakes = keep.arr(ctypes.c_uint64, self.stakes)
        c.epoch = self.epoch
        ws = self.workers or [[] for _ in self.keys]
        c.n_workers = keep.arr(ctypes.c_uint32, [len(w) for w in ws])
        ptrs = [keep.arr(ctypes.c_uint32, w) for w in ws]
        c.worker_ids = keep.arr(ctypes.c_void_p, [p.value for p in ptrs])
        return c


@dataclass
class Header:
    author: bytes
    round: int = 0
    epoch: int = 0
    payload: List[Tuple[bytes, int]] = field(default_factory=list)  # IndexMap order
    parents: List[bytes] = field(default_factory=list)  # kept sorted (BTreeSet)
    id: bytes = bytes(32)
    signature: bytes = bytes(64)

    def __post_init__(self):
        self.parents = sorted(set(self.parents))

    def _c(self, keep):
        h = _Header()
        h.author = keep.buf(self.author)
        h.round = self.round
        h.epoch = self.epoch
        h.n_payload = len(self.payload)
        h.payload_digests = keep.buf(b"".join(d for d, _ in self.payload))
        h.payload_workers = keep.arr(ctypes.c_uint32, [w for _, w in self.payload])
        h.n_parents = len(self.parents)
        h.parents = keep.buf(b"".join(self.parents))
        h.id = keep.buf(self.id)
        h.signature = keep.buf(self.signature)
        return h


@dataclass
class Vote:
    id: bytes
    round: int
    epoch: int
    origin: bytes
    author: bytes
    signature: bytes = bytes(64)

    def _c(self, keep):
        v = _Vote()
        v.id, v.origin, v.author, v.signature = (keep.buf(self.id), keep.buf(self.origin),
                                                 keep.buf(self.author), keep.buf(self.signature))
        v.round, v.epoch = self.round, self.epoch
        return v


@dataclass
class Certificate:
    header: Header
    signed_authorities: List[int] = field(default_factory=list)
    aggregated_signature: List[bytes] = field(default_factory=list)

    @staticmethod
    def genesis(committee: Committee) -> List["Certificate"]:
        return [Certificate(Header(author=k, epoch=committee.epoch)) for k in committee.keys]

    @staticmethod
    def _new_unsafe(committee: Committee, header: Header, votes: Sequence[Tuple[bytes, bytes]], check):
        n = len(votes)
        signed = (ctypes.c_uint32 * max(len(committee.keys), 1))()
        sigs = ctypes.create_string_buffer(64 * max(len(committee.keys), 1))
        ns, nsig = ctypes.c_size_t(0), ctypes.c_size_t(0)
        keep = _Keep()
        c = committee._c(keep)
        rc = lib().nwv_certificate_new(ctypes.byref(c), n, b"".join(p for p, _ in votes) or None,
                                       b"".join(s for _, s in votes) or None, 1 if check else 0,
                                       signed, ctypes.byref(ns), sigs, ctypes.byref(nsig))
        _raise(rc)
        return Certificate(header, list(signed[:ns.value]),
                           [sigs.raw[64 * k:64 * k + 64] for k in range(nsig.value)])

    @staticmethod
    def new(committee, header, votes):
        """Certificate::new: votes [(pk, sig)] -> Certificate (UnknownAuthority / RequiresQuorum)"""
        return Certificate._new_unsafe(committee, header, votes, True)

    @staticmethod
    def new_unsigned(committee, header, votes):
        return Certificate._new_unsafe(committee, header, votes, False)

    def _c(self, keep):
        c = _Certificate()
        c.header = self.header._c(keep)
        c.n_signed = len(self.signed_authorities)
        c.signed_authorities = keep.arr(ctypes.c_uint32, self.signed_authorities)
        c.n_sigs = len(self.aggregated_signature)
        c.aggregated_signature = keep.buf(b"".join(self.aggregated_signature))
        return c


# ---- GPU-backed operations (an Engine supplies the device context) -----------------------
def _many(engine, fn, committee, items):
    keep = _Keep()
    n = len(items)
    cls = type(items[0]._c(keep)) if n else _Header
    arr = (cls * max(n, 1))(*[it._c(keep) for it in items])
    res = (ctypes.c_int32 * max(n, 1))()
    if committee is None:
        out = ctypes.create_string_buffer(32 * max(n, 1))
        _lib._check(fn(engine._h, n, arr, out))
        return [out.raw[32 * i:32 * i + 32] for i in range(n)]
    c = committee._c(keep)
    _lib._check(fn(engine._h, ctypes.byref(c), n, arr, res))
    return list(res[:n])


def header_digests(engine, headers: Sequence[Header]) -> List[bytes]:
    return _many(engine, lib().nwv_header_digest_many, None, list(headers))


def vote_digests(engine, votes: Sequence[Vote]) -> List[bytes]:
    return _many(engine, lib().nwv_vote_digest_many, None, list(votes))


def certificate_digests(engine, certs: Sequence[Certificate]) -> List[bytes]:
    return _many(engine, lib().nwv_certificate_digest_many, None, list(certs))


def verify_headers(engine, committee, headers) -> List[int]:
    """Header::verify of every header in one GPU batch -> NWV_DAG_* codes (0 = Ok)"""
    return _many(engine, lib().nwv_header_verify_many, committee, list(headers))


def verify_votes(engine, committee, votes) -> List[int]:
    return _many(engine, lib().nwv_vote_verify_many, committee, list(votes))


def verify_certificates(engine, committee, certs) -> List[int]:
    return _many(engine, lib().nwv_certificate_verify_many, committee, list(certs))


def verify_mixed(engine, committee, headers=(), votes=(), certs=()):
    """One coalesced call for the headers, votes and certificates a Core has queued
    (Core::sanitize_*, primary/src/core.rs:497-573): one digest launch, one batch MSM.
    -> (header codes, vote codes, certificate codes), NWV_DAG_* (0 = Ok)"""
    keep = _Keep()
    c = committee._c(keep)
    args = []
    outs = []
    for items, cls in ((list(headers), _Header), (list(votes), _Vote), (list(certs), _Certificate)):
        n = len(items)
        arr = (cls * max(n, 1))(*[it._c(keep) for it in items])
        res = (ctypes.c_int32 * max(n, 1))()
        keep.objs += [arr, res]
        args += [n, ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(res, ctypes.c_void_p)]
        outs.append((res, n))
    _lib._check(lib().nwv_verify_mixed_many(engine._h, ctypes.byref(c), *args))
    return tuple(list(r[:n]) for r, n in outs)


def verify(engine, committee, item):
    """item.verify(committee): raises the DagError the reference would return"""
    fn = {Header: verify_headers, Vote: verify_votes, Certificate: verify_certificates}[type(item)]
    _raise(fn(engine, committee, [item])[0])


def validate_certificates(engine, committee, certs) -> Tuple[bool, List[int]]:
    """CertificatesResponse::validate_certificates -> (all valid, indices of the invalid ones)"""
    keep = _Keep()
    n = len(certs)
    arr = (_Certificate * max(n, 1))(*[c._c(keep) for c in certs])
    c = committee._c(keep)
    nbad = ctypes.c_size_t(0)
    idx = (ctypes.c_size_t * max(n, 1))()
    rc = lib().nwv_validate_certificates(engine._h, ctypes.byref(c), n, arr, ctypes.byref(nbad), idx)
    _lib._check(rc, allow=(_lib.NWV_OK, _lib.NWV_ERR_SIGNATURE))
    return rc == _lib.NWV_OK, list(idx[:nbad.value])


# ---- BLS12-381, the reference's default scheme (crypto/src/lib.rs:29-33) ------------------
# Committee, Header and Vote are shared with the Ed25519 layer (the C structs have the same
# layout; keys are 96 bytes, signatures 48).  A certificate's aggregate is ONE 48-byte G1 point,
# or None for AggregateSignature::default().
class _BlsCertificate(ctypes.Structure):
    _fields_ = [("header", _Header), ("n_signed", ctypes.c_size_t), ("signed_authorities", ctypes.c_void_p),
                ("aggregated_signature", ctypes.c_void_p)]


@dataclass
class BlsCertificate:
    header: Header
    signed_authorities: List[int] = field(default_factory=list)
    aggregated_signature: Optional[bytes] = None

    @staticmethod
    def genesis(committee: Committee) -> List["BlsCertificate"]:
        return [BlsCertificate(Header(author=k, epoch=committee.epoch, signature=bytes(48))) for k in committee.keys]

    @staticmethod
    def new(engine, committee, header, votes, check_stake=True):
        """Certificate::new under BLS: votes [(pk96, sig48)] -> BlsCertificate (the aggregate is
        summed on the GPU); raises UnknownAuthority / CertificateRequiresQuorum / InvalidSignature"""
        keep = _Keep()
        c = committee._c(keep)
        signed = (ctypes.c_uint32 * max(len(committee.keys), 1))()
        ns, has = ctypes.c_size_t(0), ctypes.c_int(0)
        agg = ctypes.create_string_buffer(48)
        rc = lib().nwv_bls_certificate_new(engine._h, ctypes.byref(c), len(votes), b"".join(p for p, _ in votes) or None,
                                           b"".join(s_ for _, s_ in votes) or None, 1 if check_stake else 0, signed,
                                           ctypes.byref(ns), agg, ctypes.byref(has))
        _raise(rc)
        return BlsCertificate(header, list(signed[:ns.value]), agg.raw if has.value else None)

    def _c(self, keep):
        c = _BlsCertificate()
        c.header = self.header._c(keep)
        c.n_signed = len(self.signed_authorities)
        c.signed_authorities = keep.arr(ctypes.c_uint32, self.signed_authorities)
        c.aggregated_signature = keep.buf(self.aggregated_signature) if self.aggregated_signature is not None else None
        return c


def bls_header_digests(engine, headers):
    return _many(engine, lib().nwv_bls_header_digest_many, None, list(headers))


def bls_vote_digests(engine, votes):
    return _many(engine, lib().nwv_bls_vote_digest_many, None, list(votes))


def bls_certificate_digests(engine, certs):
    return _many(engine, lib().nwv_bls_certificate_digest_many, None, list(certs))


def bls_verify_mixed(engine, committee, headers=(), votes=(), certs=()):
    """nwv_bls_verify_mixed_many: a Core's queued headers, votes and certificates in one call (one
    digest launch, one BLS verification call) -> (header codes, vote codes, certificate codes)"""
    keep = _Keep()
    c = committee._c(keep)
    args, outs = [], []
    for items, cls in ((list(headers), _Header), (list(votes), _Vote), (list(certs), _BlsCertificate)):
        n = len(items)
        arr = (cls * max(n, 1))(*[it._c(keep) for it in items])
        res = (ctypes.c_int32 * max(n, 1))()
        keep.objs += [arr, res]
        args += [n, ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(res, ctypes.c_void_p)]
        outs.append((res, n))
    _lib._check(lib().nwv_bls_verify_mixed_many(engine._h, ctypes.byref(c), *args))
    return tuple(list(r[:n]) for r, n in outs)


def bls_validate_certificates(engine, committee, certs) -> Tuple[bool, List[int]]:
    keep = _Keep()
    n = len(certs)
    arr = (_BlsCertificate * max(n, 1))(*[x._c(keep) for x in certs])
    c = committee._c(keep)
    nbad = ctypes.c_size_t(0)
    idx = (ctypes.c_size_t * max(n, 1))()
    rc = lib().nwv_bls_validate_certificates(engine._h, ctypes.byref(c), n, arr, ctypes.byref(nbad), idx)
    _lib._check(rc, allow=(_lib.NWV_OK, _lib.NWV_ERR_SIGNATURE))
    return rc == _lib.NWV_OK, list(idx[:nbad.value])
