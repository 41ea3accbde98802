"""ctypes wrapper around oracle/build/libnwv_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this (the checker,
never the thing measured)."""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libnwv_oracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        _lib = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_char_p
        _lib.or_ed25519_verify.argtypes = [u8p, u8p, u8p, ctypes.c_size_t]
        _lib.or_ed25519_verify.restype = ctypes.c_int
        _lib.or_ed25519_verify_batch.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_void_p,
                                                 ctypes.c_void_p, u8p]
        _lib.or_ed25519_verify_each_mt.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib.or_ed25519_verify_each_mt.restype = None
        _lib.or_ed25519_verify_batch_mt.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_void_p,
                                                    ctypes.c_void_p, u8p, ctypes.c_int]
        _lib.or_sha512.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.or_blake2b256.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.or_sc_reduce512.argtypes = [u8p, ctypes.c_void_p]
        _lib.or_batch_digest_serialized.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p,
                                                    ctypes.POINTER(ctypes.c_int64)]
        _lib.or_ed25519_pubkey.argtypes = [u8p, ctypes.c_void_p]
        _lib.or_ed25519_sign.argtypes = [u8p, u8p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.or_point_decompress_ok.argtypes = [u8p]
    return _lib


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def verify(pk, sig, msg):
    return bool(lib().or_ed25519_verify(pk, sig, msg, len(msg)))


def sha512(m):
    out = ctypes.create_string_buffer(64)
    lib().or_sha512(m, len(m), out)
    return out.raw


def blake2b256(m):
    out = ctypes.create_string_buffer(32)
    lib().or_blake2b256(m, len(m), out)
    return out.raw


def sc_reduce(b64):
    out = ctypes.create_string_buffer(32)
    lib().or_sc_reduce512(b64, out)
    return out.raw


def pubkey(seed):
    out = ctypes.create_string_buffer(32)
    lib().or_ed25519_pubkey(seed, out)
    return out.raw


def sign(seed, msg):
    out = ctypes.create_string_buffer(64)
    lib().or_ed25519_sign(seed, msg, len(msg), out)
    return out.raw


def batch_digest_serialized(buf):
    out = ctypes.create_string_buffer(32)
    err = ctypes.c_int64(0)
    rc = lib().or_batch_digest_serialized(buf, len(buf), out, ctypes.byref(err))
    return (out.raw if rc == 0 else None), err.value


def pack(items):
    """items: list of (pk, sig, msg) -> contiguous SoA arrays used by both libraries."""
    n = len(items)
    pk = b"".join(x[0] for x in items)
    sig = b"".join(x[1] for x in items)
    lens = np.array([len(x[2]) for x in items], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    msg = b"".join(x[2] for x in items)
    return pk, sig, msg, offs, lens


def verify_batch(items, seed=b"\x07" * 32):
    pk, sig, msg, offs, lens = pack(items)
    return bool(lib().or_ed25519_verify_batch(len(items), pk, sig, msg or b"\0",
                                              offs.ctypes.data, lens.ctypes.data, seed))


def verify_each_mt(pk, sig, msg, offs, lens, threads):
    n = len(offs)
    bits = np.zeros((n + 63) // 64, dtype=np.uint64)
    lib().or_ed25519_verify_each_mt(n, pk, sig, msg or b"\0", offs.ctypes.data, lens.ctypes.data,
                                    bits.ctypes.data, threads)
    return bits


def verify_batch_mt(pk, sig, msg, offs, lens, threads, seed=b"\x09" * 32):
    n = len(offs)
    return bool(lib().or_ed25519_verify_batch_mt(n, pk, sig, msg or b"\0", offs.ctypes.data,
                                                 lens.ctypes.data, seed, threads))
