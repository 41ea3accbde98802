"""Row-parallel field arithmetic of k_msm_final (narwhal_amd/csrc/fe_row.h) on the host wave
emulation (tests/hostemu): every DPP / permlane move emulated with the semantics measured on
gfx950 (tools/probe/dpp_probe.hip) and every 32/64-bit operation checked for overflow.  The
row Horner must give the same point as the lane-local chain (and so the same batch verdict as
the reference's batch::Verifier)."""
import ctypes
import random

import numpy as np
import pytest

from test_msm_hostemu import he  # noqa: F401  (fixture: builds and loads libhostemu.so)

P = 2**255 - 19


def _val(limbs):
    return sum(int(x) << (16 * k) for k, x in enumerate(limbs))


def _row_mul(lib, a, b, use_lds=0):
    A = np.array(a, dtype=np.uint32)
    B = np.array(b, dtype=np.uint32)
    out = np.zeros(16, dtype=np.uint32)
    assert lib.he_row_mul(A.ctypes.data, B.ctypes.data, out.ctypes.data, use_lds) == 1
    return [int(x) for x in out]


@pytest.fixture(scope="module")
def lib(he):  # noqa: F811
    vp = ctypes.c_void_p
    he.he_row_mul.argtypes = [vp, vp, vp, ctypes.c_int]
    he.he_row_horner.argtypes = [ctypes.c_int, vp, vp, vp, vp]
    he.he_decompress.argtypes = [ctypes.c_char_p, vp]
    he.he_row_decompress.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    return he


@pytest.mark.parametrize("use_lds", [0, 1, 2])
@pytest.mark.parametrize("bound", [2**16, 2**16 + 2**11, 2**17, int(2**17.7)])
def test_row_mul_values_and_output_bounds(lib, bound, use_lds):
    """the three operand paths of the row multiply (DPP shifts, the LDS exchange, row rotations)
    give the product mod p with the documented output bounds"""
    rnd = random.Random(bound)
    cases = [[bound - 1] * 16, [0] * 16, [1] + [0] * 15]
    cases += [[rnd.randrange(bound) for _ in range(16)] for _ in range(60)]
    for a in cases:
        for b in (cases[0], cases[3], [rnd.randrange(bound) for _ in range(16)]):
            out = _row_mul(lib, a, b, use_lds)
            assert _val(out) % P == (_val(a) * _val(b)) % P
            assert out[0] < 2**17 and max(out[1:]) < 2**16 + 2**12  # two carry passes (fe_row.h)


def _random_point(lib, rnd):
    out = np.zeros(40, dtype=np.uint32)
    while True:
        b = bytes(rnd.getrandbits(8) for _ in range(32))
        if lib.he_decompress(b, out.ctypes.data):
            return b


# 8-torsion encodings: identity (y = 1), (0, -1) (y = p - 1), the order-4 points (y = 0)
TORSION = [(1).to_bytes(32, "little"), (P - 1).to_bytes(32, "little"), bytes(32),
           bytes(31) + b"\x80"]


def _horner(lib, widths, pts):
    nw = len(widths)
    W = np.array(widths, dtype=np.uint8)
    row = np.zeros(24, dtype=np.uint32)
    ref = np.zeros(24, dtype=np.uint32)
    r = lib.he_row_horner(nw, W.ctypes.data, b"".join(pts), row.ctypes.data, ref.ctypes.data)
    assert r in (0, 1)

    def coords(a):
        return [sum(int(a[8 * c + j]) << (32 * j) for j in range(8)) for c in range(3)]

    return r, coords(row), coords(ref)


def test_row_horner_matches_lane_chain(lib):
    rnd = random.Random(7)
    for trial in range(12):
        nw = rnd.choice([1, 2, 3, 17, 22, 48])
        widths = [rnd.randint(1, 16) for _ in range(nw)]
        pts = [_random_point(lib, rnd) for _ in range(nw)]
        r, (X, Y, Z), (Xr, Yr, Zr) = _horner(lib, widths, pts)
        assert r == 0  # a random combination of random points is not 8-torsion
        assert Z % P and Zr % P
        assert X * Zr % P == Xr * Z % P
        assert Y * Zr % P == Yr * Z % P


def test_row_horner_torsion_is_identity(lib):
    rnd = random.Random(8)
    for nw in (1, 5, 30):
        widths = [rnd.randint(1, 16) for _ in range(nw)]
        pts = [rnd.choice(TORSION) for _ in range(nw)]
        r, (X, Y, Z), _ = _horner(lib, widths, pts)
        assert r == 1 and X % P == 0 and (Y - Z) % P == 0
    # one prime-order component anywhere breaks it
    widths = [12] * 8
    pts = [TORSION[1]] * 8
    pts[3] = _random_point(lib, rnd)
    assert _horner(lib, widths, pts)[0] == 0


@pytest.mark.parametrize("form", [0, 1, 2])
def test_row_decompression_matches_lane_local(lib, form):
    """k_msm_prep's row form (the decompression power on 16-lane rows, small batches) gives the
    same MSM record and decode flag as the lane-local ge_decompress on random encodings (about
    half do not decode), the 8-torsion encodings, y >= p, negative zero and the golden vectors'
    keys and R values"""
    import json
    import os
    rnd = random.Random(11 + form)
    encs = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(40)]
    encs += TORSION + [bytes(31) + b"\x80" * 1, (P).to_bytes(32, "little"), (P + 1).to_bytes(32, "little"),
                       (2**255 - 1).to_bytes(32, "little"), ((1) | (1 << 255)).to_bytes(32, "little")]
    g = os.path.join(os.path.dirname(__file__), "golden", "ed25519_vectors.json")
    with open(g) as f:
        vs = json.load(f)["vectors"]
    for v in vs[:: max(1, len(vs) // 40)]:
        encs += [bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"])[:32]]
    assert lib.he_row_decompress(b"".join(encs), len(encs), form) == 0
