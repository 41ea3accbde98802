"""The BLS12-381 oracle (oracle/bls_oracle.c) against its pins, on the CPU:
the reference's own BLS12381KeyPair fixtures (Docker/validators/validator-*/primary-key.json), the
RFC 9380 Appendix J.9.1 hash_to_curve known answers, a big-integer Python restatement of signing
(oracle/gen_bls_golden.py), and the algebra that pins the pairing (bilinearity, non-degeneracy,
order r, the fast twisted Miller loop + x-chain final exponentiation against a plain affine Miller
loop on the untwisted curve with square-and-multiply final exponentiation)."""
import hashlib
import json
import os
import random

import pytest

import bls_ffi as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(ROOT, "tests", "golden", "bls12381_kats.json")) as f:
        return json.load(f)


def test_keygen_matches_reference_docker_fixtures(gold):
    assert len(gold["keygen"]) == 4
    for k in gold["keygen"]:
        rc, pk = B.keygen(bytes.fromhex(k["sk"]))
        assert rc == B.ORB_OK and pk.hex() == k["pk"], k["source"]
        assert B.lib().orb_pubkey_validate(pk) == B.ORB_OK


def test_hash_to_g1_rfc9380_known_answers(gold):
    assert len(gold["hash_to_g1"]) == 2
    for v in gold["hash_to_g1"]:
        P = B.hash_to_g1(bytes.fromhex(v["msg"]), v["dst"].encode())
        assert P.hex() == v["x"] + v["y"]


def test_sign_matches_python_restatement(gold):
    for s in gold["sign"]:
        sk = bytes.fromhex(gold["keygen"][s["sk_index"]]["sk"])
        m = bytes.fromhex(s["msg"])
        assert B.g1_compress(B.hash_to_g1(m)).hex() == s["h"]
        assert B.sign(sk, m).hex() == s["sig"]


def test_sha256_and_expand_message_xmd():
    rnd = random.Random(1)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 1000):
        m = rnd.randbytes(n)
        assert B.sha256(m) == hashlib.sha256(m).digest()
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    for msg in (b"", b"abc", bytes(200)):
        for n in (32, 128, 48, 255):
            h = lambda x: hashlib.sha256(x).digest()
            ell = (n + 31) // 32
            dp = dst + bytes([len(dst)])
            b0 = h(bytes(64) + msg + n.to_bytes(2, "big") + b"\0" + dp)
            bs = [h(b0 + b"\1" + dp)]
            for i in range(2, ell + 1):
                bs.append(h(bytes(x ^ y for x, y in zip(b0, bs[-1])) + bytes([i]) + dp))
            assert B.expand_xmd(msg, dst, n) == b"".join(bs)[:n]


def test_hard_exponent_constant():
    assert B.hard_exponent() == (p ** 4 - p ** 2 + 1) // r


def test_generators_and_compression(gold):
    assert B.g1_compress(B.g1_gen()).hex() == gold["g1_gen"]
    rc, Q = B.g2_decompress(bytes.fromhex(gold["g2_gen"]))
    assert rc == 0 and Q == B.g2_gen()
    rnd = random.Random(2)
    for _ in range(4):
        P = B.g1_mul(B.g1_gen(), rnd.randrange(1, r))
        Q = B.g2_mul(B.g2_gen(), rnd.randrange(1, r))
        assert B.g1_decompress(B.g1_compress(P)) == (0, P)
        assert B.g2_decompress(B.g2_compress(Q)) == (0, Q)
    assert B.g1_decompress(bytes([0xc0]) + bytes(47)) == (0, bytes(96))
    assert B.g2_decompress(bytes([0xc0]) + bytes(95)) == (0, bytes(192))


def test_pairing_fast_equals_reference_cubed():
    rnd = random.Random(3)
    for _ in range(2):
        P = B.g1_mul(B.g1_gen(), rnd.randrange(1, r))
        Q = B.g2_mul(B.g2_gen(), rnd.randrange(1, r))
        assert B.pairing(P, Q) == B.gt_pow(B.pairing_ref(P, Q), 3)


def test_pairing_bilinear_nondegenerate_order_r():
    rnd = random.Random(4)
    P, Q = B.g1_gen(), B.g2_gen()
    e = B.pairing(P, Q)
    one = B.gt_pow(e, 0)
    assert e != one
    assert B.gt_pow(e, r) == one
    for _ in range(3):
        a, b = rnd.randrange(1, r), rnd.randrange(1, r)
        assert B.pairing(B.g1_mul(P, a), B.g2_mul(Q, b)) == B.gt_pow(e, a * b % r)
    P2 = B.g1_mul(P, 7)
    assert B.gt_mul(B.pairing(P, Q), B.pairing(P2, Q)) == B.pairing(B.g1_add(P, P2), Q)


def _not_in_g1():
    """a point on y^2 = x^3 + 4 outside the order-r subgroup (the cofactor is not cleared)"""
    x = 5
    while True:
        for sign in (0, 0x20):
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80 | sign
            rc, P = B.g1_decompress(bytes(b))
            if rc == 0 and not B.lib().orb_g1_in_group(bytes(b)):
                return bytes(b)
        x += 1


def _not_in_g2():
    x = 3
    while True:
        b = bytearray(bytes(48) + x.to_bytes(48, "big"))
        b[0] |= 0x80
        rc, Q = B.g2_decompress(bytes(b))
        if rc == 0 and not B.lib().orb_g2_in_group(bytes(b)):
            return bytes(b)
        x += 1


def test_verify_semantics(gold):
    sks = [bytes.fromhex(k["sk"]) for k in gold["keygen"]]
    pks = [bytes.fromhex(k["pk"]) for k in gold["keygen"]]
    m = bytes(range(32))
    sigs = [B.sign(sk, m) for sk in sks]
    assert all(B.verify(pk, m, s) == B.ORB_OK for pk, s in zip(pks, sigs))
    assert B.verify(pks[0], m + b"x", sigs[0]) == B.ORB_VERIFY_FAIL
    assert B.verify(pks[1], m, sigs[0]) == B.ORB_VERIFY_FAIL
    # encodings: compression flag, x >= p, infinity with stray bits, off-curve x
    bad = bytearray(sigs[0])
    bad[0] &= 0x7f
    assert B.verify(pks[0], m, bytes(bad)) == B.ORB_BAD_ENCODING
    big = bytearray(p.to_bytes(48, "big"))
    big[0] |= 0x80
    assert B.verify(pks[0], m, bytes(big)) == B.ORB_BAD_ENCODING
    assert B.verify(pks[0], m, bytes([0xc1]) + bytes(47)) == B.ORB_BAD_ENCODING
    assert B.verify(pks[0], m, bytes([0xe0]) + bytes(47)) == B.ORB_BAD_ENCODING
    # the identity signature passes the group check and fails the pairing equation
    assert B.verify(pks[0], m, bytes([0xc0]) + bytes(47)) == B.ORB_VERIFY_FAIL
    assert B.verify(bytes([0xc0]) + bytes(95), m, sigs[0]) == B.ORB_PK_INFINITY
    assert B.verify(pks[0], m, _not_in_g1()) == B.ORB_NOT_IN_GROUP
    assert B.verify(_not_in_g2(), m, sigs[0]) == B.ORB_NOT_IN_GROUP
    # aggregation: AggregateAuthenticator::aggregate + fast_aggregate_verify
    rc, agg = B.aggregate(sigs[:3])
    assert rc == 0
    assert B.fast_aggregate_verify(agg, pks[:3], m) == B.ORB_OK
    assert B.fast_aggregate_verify(agg, pks[:2], m) == B.ORB_VERIFY_FAIL
    assert B.fast_aggregate_verify(agg, [pks[3]] + pks[1:3], m) == B.ORB_VERIFY_FAIL
    assert B.fast_aggregate_verify(agg, [], m) == B.ORB_AGGR_MISMATCH
    assert B.aggregate([])[0] == B.ORB_AGGR_MISMATCH
    assert B.aggregate([sigs[0], _not_in_g1()])[0] == B.ORB_NOT_IN_GROUP
    # apk = identity (pk + (-pk)) is rejected
    rc, q = B.g2_decompress(pks[0])
    negpk = bytearray(pks[0])
    negpk[0] ^= 0x20
    assert B.fast_aggregate_verify(agg, [pks[0], bytes(negpk)], m) == B.ORB_PK_INFINITY
