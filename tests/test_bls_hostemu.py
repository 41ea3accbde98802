"""The gfx950 BLS12-381 code (narwhal_amd/csrc/bls381.h, bls_verify.h) compiled for the host
(tests/hostemu/bls_hostemu.cpp) against the oracle, on the CPU: pairing values bit-exact,
hash_to_curve on the RFC 9380 known answers, key generation on the reference's Docker fixtures,
decode / subgroup statuses of adversarial encodings, and fast_aggregate_verify statuses."""
import ctypes
import json
import os
import random
import subprocess

import pytest

import bls_cases as C
import bls_ffi as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


@pytest.fixture(scope="module")
def emu():
    # NWV_BLSEMU_LIB: another build of the same code (the sanitizer build, tools/run_blsemu_asan.sh)
    path = os.environ.get("NWV_BLSEMU_LIB") or os.path.join(ROOT, "tests", "_build", "libblsemu.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", ROOT, "tests/_build/libblsemu.so"], check=True)
    L = ctypes.CDLL(path)
    c, sz, vp = ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p
    L.bh_pairing.argtypes = [c, c, vp]
    L.bh_hash_to_g1.argtypes = [c, sz, c, sz, vp]
    L.bh_key_decode.argtypes = [c, vp]
    L.bh_sig_decode.argtypes = [c, vp]
    L.bh_keygen.argtypes = [c, vp]
    L.bh_sign.argtypes = [c, c, sz, c, sz, vp]
    L.bh_fast_aggregate_verify.argtypes = [c, sz, c, c, sz, c, sz]
    L.bh_rlc_batch.argtypes = [sz, c, c, c, c, c, sz]
    L.bh_g_pairing.argtypes = [c, c, vp]
    L.bh_g_fast_aggregate_verify.argtypes = [c, sz, c, c, sz, c, sz]
    L.bh_w_f12_op.argtypes = [ctypes.c_int, c, c, vp]
    L.bh_w_fast_aggregate_verify.argtypes = [c, sz, c, c, sz, c, sz, ctypes.c_int]
    L.bh_w_hash_to_g1.argtypes = [c, sz, c, sz, vp]
    L.bh_w_sig_status.argtypes = [c]
    L.bh_w2_fast_aggregate_verify.argtypes = [c, sz, c, c, sz, c, sz]
    L.bh_w3_fast_aggregate_verify.argtypes = [c, sz, c, c, sz, c, sz, ctypes.c_int]
    L.bh_w_pc_fast_aggregate_verify.argtypes = [c, sz, c, c, sz, c, sz, ctypes.c_int]
    L.bh_fp_inv_vt.argtypes = [c, vp]
    L.bh_w_aggregate.argtypes = [sz, c, vp, ctypes.c_int]
    L.bh_fp_inv_rows.argtypes = [c, vp]
    return L


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(ROOT, "tests", "golden", "bls12381_kats.json")) as f:
        return json.load(f)


def _buf(n):
    return ctypes.create_string_buffer(n)


def test_pairing_bit_exact(emu):
    rnd = random.Random(21)
    for _ in range(3):
        P = B.g1_mul(B.g1_gen(), rnd.randrange(1, r))
        Q = B.g2_mul(B.g2_gen(), rnd.randrange(1, r))
        o = _buf(576)
        emu.bh_pairing(P, Q, o)
        assert o.raw == B.pairing(P, Q)


def test_hash_to_g1(emu, gold):
    for v in gold["hash_to_g1"]:
        m, d = bytes.fromhex(v["msg"]), v["dst"].encode()
        o = _buf(96)
        emu.bh_hash_to_g1(m, len(m), d, len(d), o)
        assert o.raw.hex() == v["x"] + v["y"]
    rnd = random.Random(22)
    for n in (0, 17, 64, 150):
        m = rnd.randbytes(n)
        o = _buf(96)
        emu.bh_hash_to_g1(m, len(m), B.DST_NUL, len(B.DST_NUL), o)
        assert o.raw == B.hash_to_g1(m)


def test_keygen_and_sign(emu, gold):
    for k in gold["keygen"]:
        o = _buf(96)
        emu.bh_keygen(bytes.fromhex(k["sk"]), o)
        assert o.raw.hex() == k["pk"]
    for s in gold["sign"][:4]:
        sk, m = bytes.fromhex(gold["keygen"][s["sk_index"]]["sk"]), bytes.fromhex(s["msg"])
        o = _buf(48)
        emu.bh_sign(sk, m, len(m), B.DST_NUL, len(B.DST_NUL), o)
        assert o.raw.hex() == s["sig"]


def test_decode_statuses(emu, gold):
    """decode + subgroup statuses equal the oracle's for valid, identity, off-curve, bad-encoding
    and outside-the-subgroup inputs (the endomorphism tests against the oracle's [r]P = O)"""
    pk = bytes.fromhex(gold["keygen"][0]["pk"])
    sig = bytes.fromhex(gold["sign"][0]["sig"])
    o2, o1 = _buf(192), _buf(96)
    assert emu.bh_key_decode(pk, o2) == 0 and o2.raw == B.g2_decompress(pk)[1]
    assert emu.bh_key_decode(C.IDENTITY_G2, o2) == B.ORB_PK_INFINITY
    assert emu.bh_key_decode(C.not_in_g2(), o2) == B.ORB_NOT_IN_GROUP
    assert emu.bh_key_decode(C.not_in_g2(50), o2) == B.ORB_NOT_IN_GROUP
    for s in [sig, C.IDENTITY_G1, C.not_in_g1(), C.not_in_g1(100)] + C.bad_encodings_g1(sig):
        want = B.g1_decompress(s)[0]
        if want == 0 and s != C.IDENTITY_G1 and not B.lib().orb_g1_in_group(s):
            want = B.ORB_NOT_IN_GROUP
        assert emu.bh_sig_decode(s, o1) == want, s.hex()


def test_fast_aggregate_verify_statuses(emu, gold):
    sks = [bytes.fromhex(k["sk"]) for k in gold["keygen"]]
    pks = [bytes.fromhex(k["pk"]) for k in gold["keygen"]]
    m = bytes(range(32))
    sigs = [B.sign(sk, m) for sk in sks]
    _, agg = B.aggregate(sigs[:3])
    dst = B.DST_NUL
    cases = [(agg, pks[:3], m), (agg, pks[:3], m + b"x"), (agg, pks[:2], m), (agg, [], m),
             (agg, [pks[0], C.negate_g2(pks[0])], m), (agg, pks[:2] + [C.not_in_g2()], m),
             (C.IDENTITY_G1, pks[:3], m), (C.not_in_g1(), pks[:3], m), (sigs[0], pks[:1], m)]
    for s, ks, msg in cases:
        got = emu.bh_fast_aggregate_verify(s, len(ks), b"".join(ks), msg, len(msg), dst, len(dst))
        assert got == B.fast_aggregate_verify(s, ks, msg)


def test_rlc_batch_check(emu, gold):
    """the random-linear-combination batch check (bls_verify.h rlc_*): accepts valid items at
    every tree shape, rejects when any one item's pairing equation fails"""
    import os
    sks = [bytes.fromhex(k["sk"]) for k in gold["keygen"]]
    pks = [bytes.fromhex(k["pk"]) for k in gold["keygen"]]
    dst = B.DST_NUL
    seed = os.urandom(32)
    msgs = [bytes([i]) * 32 for i in range(5)]
    sigs = [B.sign(sks[i % 4], m) for i, m in enumerate(msgs)]
    keys = [pks[i % 4] for i in range(5)]
    for n in (1, 2, 3, 5):
        assert emu.bh_rlc_batch(n, b"".join(sigs[:n]), b"".join(keys[:n]), b"".join(msgs[:n]), seed, dst,
                                len(dst)) == 1
        for bad in range(n):
            m2 = list(msgs[:n])
            m2[bad] = bytes([0xee]) * 32
            assert emu.bh_rlc_batch(n, b"".join(sigs[:n]), b"".join(keys[:n]), b"".join(m2), seed, dst,
                                    len(dst)) == 0
        # a signature swapped between two items: each item's equation fails, the sums still match
        if n >= 2:
            s2 = list(sigs[:n])
            s2[0], s2[1] = s2[1], s2[0]
            assert emu.bh_rlc_batch(n, b"".join(s2), b"".join(keys[:n]), b"".join(msgs[:n]), seed, dst,
                                    len(dst)) == 0


def test_group_pairing_matches_single_lane(emu):
    """bls_group.h's Miller loop + final exponentiation (the group arithmetic the kernels run) equal
    bls381.h's single-lane pairing bit for bit, and both equal the oracle"""
    import random
    rnd = random.Random(21)
    for _ in range(3):
        P = B.g1_mul(B.g1_gen(), rnd.randrange(1, r))
        Q = B.g2_mul(B.g2_gen(), rnd.randrange(1, r))
        o1 = ctypes.create_string_buffer(576)
        o2 = ctypes.create_string_buffer(576)
        emu.bh_pairing(P, Q, o1)
        emu.bh_g_pairing(P, Q, o2)
        assert o1.raw == o2.raw == B.pairing(P, Q)


def test_group_fast_aggregate_verify_statuses(emu, gold):
    sks = [bytes.fromhex(k["sk"]) for k in gold["keygen"]]
    pks = [bytes.fromhex(k["pk"]) for k in gold["keygen"]]
    m = bytes(range(32))
    sigs = [B.sign(sk, m) for sk in sks]
    _, agg = B.aggregate(sigs[:3])
    dst = B.DST_NUL
    for s, ks, msg in [(agg, pks[:3], m), (agg, pks[:3], m + b"x"), (sigs[0], pks[:1], m), (C.IDENTITY_G1, pks[:3], m)]:
        got = emu.bh_g_fast_aggregate_verify(s, len(ks), b"".join(ks), msg, len(msg), dst, len(dst))
        assert got == B.fast_aggregate_verify(s, ks, msg)


# ---- the wave engine (bls_wave.h: stage programs of tools/gen_bls_wave.py) on the host --------
def _rand_f12(rnd):
    p = C.p
    return b"".join(rnd.randrange(p).to_bytes(48, "big") for _ in range(12))


def test_wave_f12_ops_match_oracle(emu):
    """the stage programs' Fp12 product and square equal the oracle's Fp12 arithmetic bit for bit
    (canonical outputs), the cyclotomic square on GT elements as well"""
    rnd = random.Random(51)
    for _ in range(3):
        a, b = _rand_f12(rnd), _rand_f12(rnd)
        o = _buf(576)
        emu.bh_w_f12_op(0, a, b, o)
        assert o.raw == B.gt_mul(a, b)
        emu.bh_w_f12_op(2, a, None, o)
        assert o.raw == B.gt_mul(a, a)
    g = B.pairing(B.g1_mul(B.g1_gen(), 7), B.g2_gen())  # in the cyclotomic subgroup
    o = _buf(576)
    emu.bh_w_f12_op(1, g, None, o)
    assert o.raw == B.gt_mul(g, g)


@pytest.mark.parametrize("lines", [0, 1])
def test_wave_fast_aggregate_verify_matches_oracle(emu, lines):
    """fast_aggregate_verify with the pairing check on the wave (Miller loop and final
    exponentiation as stage programs): valid items, wrong message / key set, identity signature,
    pre-pairing failures; the apk's lines computed in the loop (0) or precomputed (1)"""
    rnd = random.Random(52 + lines)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(4)]
    pks = [B.keygen(k)[1] for k in sks]
    m = rnd.randbytes(32)
    sigs = [B.sign(k, m) for k in sks]
    _, agg = B.aggregate(sigs[:3])
    cases = [(agg, pks[:3], m), (sigs[0], pks[:1], m), (agg, pks[:3], m + b"!"), (agg, pks[1:], m),
             (C.IDENTITY_G1, pks[:2], m), (C.not_in_g1(), pks[:2], m), (agg, [], m)]
    for sig, ks, msg in cases:
        got = emu.bh_w_fast_aggregate_verify(sig, len(ks), b"".join(ks) or None, msg, len(msg), B.DST_NUL,
                                             len(B.DST_NUL), lines)
        assert got == B.fast_aggregate_verify(sig, ks, msg), (ks == pks[:3], msg == m)


def test_wave_hash_to_g1_rfc9380(emu, gold):
    """hash to G1 with the isogeny map, the sum and [h_eff] as wave programs (homogeneous, no
    inversion): the RFC 9380 J.9.1 known answers and the oracle on other messages"""
    o = _buf(96)
    for v in gold["hash_to_g1"]:
        m, dst = bytes.fromhex(v["msg"]), v["dst"].encode()
        emu.bh_w_hash_to_g1(m, len(m), dst, len(dst), o)
        assert o.raw.hex() == v["x"] + v["y"]
    rnd = random.Random(53)
    for n in (0, 1, 32, 77, 200):
        m = rnd.randbytes(n)
        emu.bh_w_hash_to_g1(m, len(m), B.DST_NUL, len(B.DST_NUL), o)
        assert o.raw == B.hash_to_g1(m)


def test_wave_g1_membership(emu):
    """the signature's G1 check on the wave: valid signatures, points of E outside G1 (several),
    the identity, bad encodings -- statuses equal the oracle's decode + group check"""
    rnd = random.Random(54)
    sk = rnd.randrange(1, r).to_bytes(32, "big")
    cases = [B.sign(sk, rnd.randbytes(32)) for _ in range(2)] + [C.not_in_g1(s) for s in (5, 50, 500)] + \
        [C.IDENTITY_G1, C.off_curve_g1()] + C.bad_encodings_g1(B.sign(sk, b"x"))
    for sg in cases:
        want = B.g1_decompress(sg)[0] or (0 if sg == C.IDENTITY_G1 or B.lib().orb_g1_in_group(sg) else B.ORB_NOT_IN_GROUP)
        assert emu.bh_w_sig_status(sg) == want


def test_wave_pipeline_fast_aggregate_verify(emu):
    """every step on the wave (decode + wave G1 check, wave hash to G1, wave pairing check)
    against the oracle"""
    rnd = random.Random(55)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(3)]
    pks = [B.keygen(k)[1] for k in sks]
    m = rnd.randbytes(32)
    _, agg = B.aggregate([B.sign(k, m) for k in sks])
    for sig, ks, msg in [(agg, pks, m), (agg, pks, m + b"?"), (agg, pks[:2], m), (C.not_in_g1(), pks, m),
                         (C.IDENTITY_G1, pks, m)]:
        got = emu.bh_w2_fast_aggregate_verify(sig, len(ks), b"".join(ks), msg, len(msg), B.DST_NUL, len(B.DST_NUL))
        assert got == B.fast_aggregate_verify(sig, ks, msg)


def test_fp_inv_variable_time(emu):
    """the batched binary-GCD inversion (variable time: public inputs) against a^(p-2)"""
    rnd = random.Random(56)
    p = C.p
    vals = [1, 2, 3, p - 1, p - 2, (p + 1) // 2, 1 << 62, (1 << 62) - 1, 1 << 380, (1 << 381) % p]
    vals += [rnd.randrange(1, p) for _ in range(500)] + [rnd.randrange(1, 1 << rnd.randrange(1, 380)) for _ in range(100)]
    o = _buf(48)
    for inv in (emu.bh_fp_inv_vt, emu.bh_fp_inv_rows):  # the row form: the wave's (fp_inv_wave) updates
        for a in vals:
            inv(a.to_bytes(48, "big"), o)
            assert int.from_bytes(o.raw, "big") == pow(a, p - 2, p), hex(a)
        inv(bytes(48), o)
        assert o.raw == bytes(48)


def test_wave_cofactor_on_key_side(emu):
    """e(H0, [h_eff] apk) == e([h_eff] H0, apk): the hash's cofactor clearing moved onto the key sum
    (H0 = the two maps' sum, not cleared), with computed lines and with the line table of
    [h_eff] apk -- statuses equal the oracle's on valid items, wrong messages, wrong key sets,
    signatures outside G1 and the identity"""
    rnd = random.Random(58)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(3)]
    pks = [B.keygen(k)[1] for k in sks]
    cases = []
    for t in range(6):
        m = rnd.randbytes(rnd.choice([0, 1, 32, 100]))
        _, agg = B.aggregate([B.sign(k, m) for k in sks])
        cases += [(agg, pks, m), (agg, pks, m + b"?"), (agg, pks[:2], m)]
        one = B.sign(sks[t % 3], m)
        cases += [(one, [pks[t % 3]], m), (one, [pks[(t + 1) % 3]], m)]
    cases += [(C.not_in_g1(), pks, b"m"), (C.IDENTITY_G1, pks, b"m")]
    for sig, ks, msg in cases:
        want = B.fast_aggregate_verify(sig, ks, msg)
        for mode in (1, 2):
            got = emu.bh_w3_fast_aggregate_verify(sig, len(ks), b"".join(ks), msg, len(msg), B.DST_NUL,
                                                  len(B.DST_NUL), mode)
            assert got == want, (mode, len(ks), len(msg))


def test_wave_aggregate_matches_oracle(emu):
    """AggregateAuthenticator::aggregate by the g1_sum trees (nwv_bls.hip k_blsw_g1_sum /
    k_blsw_g1_sum_fin) against the oracle's sum: one point, a partial block, 32 and 33 (two tree
    levels), 67 (the quorum of 100), 1,100 (three levels), repeated and opposite points (the
    complete formulas' doubling and identity cases), the identity signature, and a bad signature
    mid-list; straight records and records read through a position list"""
    rnd = random.Random(31)
    base = [B.g1_compress(B.g1_mul(B.g1_gen(), rnd.randrange(1, r))) for _ in range(40)]
    neg = bytes([base[3][0] ^ 0x20]) + base[3][1:]  # -P: the sign bit flipped
    ident = bytes([0xc0]) + bytes(47)
    cases = [base[:1], base[:5], base[:32], base[:33], (base * 2)[:67], [base[0]] * 4, [base[3], neg],
             [base[3], neg, base[4]], [ident, base[1]], [ident], (base * 28)[:1100]]
    for sigs in cases:
        want_rc, want = B.aggregate(sigs)
        for through in (0, 1):
            o = _buf(48)
            st = emu.bh_w_aggregate(len(sigs), b"".join(sigs), o, through)
            assert st == want_rc and o.raw == want, (len(sigs), through)
    bad = base[:10] + [C.not_in_g1()] + base[10:40]
    o = _buf(48)
    assert emu.bh_w_aggregate(len(bad), b"".join(bad), o, 0) == B.aggregate(bad)[0] == B.ORB_NOT_IN_GROUP


def test_generated_wave_tables_match_generator():
    """narwhal_amd/csrc/bls_wave_prog.h and bls_wave_counts.json are exactly what
    tools/gen_bls_wave.py emits (its --check re-emits into a temporary directory and compares), after
    checking every program against its formulas on Python integers"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_bls_wave.py"), "--check"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "match the generator" in p.stderr


def test_wave_pairing_on_pc_bank(emu):
    """the packed pairing kernel's bank holds only the pairing check's NSLOTS_PC slots (the
    generator lays them out first): the whole pairing check, computed lines and a key's line
    table, run on a bank of exactly that size with a canary behind it -- statuses equal the
    oracle's and nothing past the bank is touched"""
    rnd = random.Random(59)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(3)]
    pks = [B.keygen(k)[1] for k in sks]
    m = rnd.randbytes(32)
    _, agg = B.aggregate([B.sign(k, m) for k in sks])
    one = B.sign(sks[0], m)
    for sig, ks, msg in [(agg, pks, m), (agg, pks, m + b"?"), (one, pks[:1], m), (one, pks[1:2], m),
                         (C.IDENTITY_G1, pks, m)]:
        want = B.fast_aggregate_verify(sig, ks, msg)
        for mode in (1, 2):
            got = emu.bh_w_pc_fast_aggregate_verify(sig, len(ks), b"".join(ks), msg, len(msg), B.DST_NUL,
                                                    len(B.DST_NUL), mode)
            assert got != -1000, "a pairing-check program addressed a slot past NSLOTS_PC"
            assert got == want, (mode, len(ks))


def test_wave_flat_pairing_script(emu):
    """the packed pairing kernel runs one flat script (wave::pairing_script: the Miller loop's line
    loads and programs, the conjugation, the final exponentiation's programs and inversion) in one
    interpreter loop instead of an out-of-line call per program; the script, replayed op by op on
    the host wave, gives the oracle's statuses with computed and with precomputed key lines"""
    import ctypes
    emu.bh_w_script_fast_aggregate_verify.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                      ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                                      ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    rnd = random.Random(73)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(3)]
    pks = [B.keygen(k)[1] for k in sks]
    m = rnd.randbytes(32)
    _, agg = B.aggregate([B.sign(k, m) for k in sks])
    one = B.sign(sks[0], m)
    for sig, ks, msg in [(agg, pks, m), (agg, pks, m + b"?"), (one, pks[:1], m), (one, pks[1:2], m),
                         (C.IDENTITY_G1, pks, m)]:
        want = B.fast_aggregate_verify(sig, ks, msg)
        for mode in (1, 2):
            nops = ctypes.c_int(0)
            got = emu.bh_w_script_fast_aggregate_verify(sig, len(ks), b"".join(ks), msg, len(msg), B.DST_NUL,
                                                        len(B.DST_NUL), mode, ctypes.byref(nops))
            assert got != -2000, "a RUN op's next_run link is wrong"
            assert got == want, (mode, len(ks))
            assert 2 * 68 < nops.value <= 512
