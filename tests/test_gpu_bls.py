"""GPU parity of the BLS12-381 engine (include/nwv_bls.h) through the C ABI:
key generation against the reference's own BLS12381KeyPair fixtures, hash_to_curve against the
RFC 9380 known answers, signing and pairing values bit-exact against the oracle
(oracle/bls_oracle.c), and per-item verification statuses identical to the oracle's on batches
that mix valid certificates with every adversarial category (bad encodings, off-curve points,
points outside G1 / G2, identities, wrong message / key set, empty key lists)."""
import json
import os
import random

import pytest

import bls_cases as C
import bls_ffi as B

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


@pytest.fixture(scope="module")
def bls():
    import narwhal_amd
    from narwhal_amd.bls import Bls
    e = narwhal_amd.Engine(device=0)
    yield Bls(e)
    e.close()


@pytest.fixture(scope="module")
def bls_batch():
    """a context under NWV_FLAG_BLS_BATCH: the call's pairing equations as one random linear
    combination on the 8-lane group kernels (per item only after a rejection)"""
    import narwhal_amd
    from narwhal_amd import _lib
    from narwhal_amd.bls import Bls
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_BLS_BATCH)
    yield Bls(e)
    e.close()


@pytest.fixture(scope="module")
def bls_per_item():
    """a context under NWV_FLAG_BLS_PER_ITEM: every item's own pairing check, no batch check"""
    import narwhal_amd
    from narwhal_amd import _lib
    from narwhal_amd.bls import Bls
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_BLS_PER_ITEM)
    yield Bls(e)
    e.close()


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(ROOT, "tests", "golden", "bls12381_kats.json")) as f:
        return json.load(f)


def test_keygen_reference_fixtures(bls, gold):
    sks = [bytes.fromhex(k["sk"]) for k in gold["keygen"]]
    assert [pk.hex() for pk in bls.keygen(sks)] == [k["pk"] for k in gold["keygen"]]


def test_hash_to_g1_rfc9380(bls, gold):
    for v in gold["hash_to_g1"]:
        (P,) = bls.hash_to_g1([bytes.fromhex(v["msg"])], v["dst"].encode())
        assert P.hex() == v["x"] + v["y"]
    rnd = random.Random(11)
    msgs = [rnd.randbytes(n) for n in (0, 1, 31, 32, 33, 64, 100, 200, 500)]
    assert bls.hash_to_g1(msgs) == [B.hash_to_g1(m) for m in msgs]


def test_sign_matches_golden_and_oracle(bls, gold):
    sks = [bytes.fromhex(gold["keygen"][s["sk_index"]]["sk"]) for s in gold["sign"]]
    msgs = [bytes.fromhex(s["msg"]) for s in gold["sign"]]
    assert [s.hex() for s in bls.sign(sks, msgs)] == [s["sig"] for s in gold["sign"]]


def test_pairing_values_bit_exact(bls):
    rnd = random.Random(12)
    Ps = [B.g1_mul(B.g1_gen(), rnd.randrange(1, r)) for _ in range(6)] + [bytes(96)]
    Qs = [B.g2_mul(B.g2_gen(), rnd.randrange(1, r)) for _ in range(6)] + [B.g2_gen()]
    assert bls.pairing(Ps, Qs) == [B.pairing(P, Q) for P, Q in zip(Ps, Qs)]


def _committee(bls, n, seed):
    rnd = random.Random(seed)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(n)]
    return sks, bls.keygen(sks)


@pytest.fixture(scope="module")
def bls_nocache():
    """a context under NWV_FLAG_NO_KEYCACHE: every call decodes its keys afresh"""
    import narwhal_amd
    from narwhal_amd import _lib
    from narwhal_amd.bls import Bls
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_NO_KEYCACHE)
    yield Bls(e)
    e.close()


EXPECT_PATH = {"wave": ("wave", "wave"), "nocache": ("wave", "wave"), "per_item": ("per_item", "per_item"),
               "batch": ("batch_rejected_then_per_item", "batch_accepted")}


@pytest.mark.parametrize("path", ["wave", "batch", "per_item", "nocache"])
def test_verify_many_mixed_batch_matches_oracle(bls, bls_batch, bls_per_item, bls_nocache, path):
    """certificates of a 10-node committee (quorum 7 signers, 32-byte digests) plus every
    adversarial category; statuses equal the oracle's codes item by item: on the wave engine
    (default), through the batch check (it rejects, then the per-item check names the failures)
    and under NWV_FLAG_BLS_PER_ITEM"""
    bls = {"wave": bls, "batch": bls_batch, "per_item": bls_per_item, "nocache": bls_nocache}[path]
    sks, pks = _committee(bls, 10, 13)
    keys = pks + [C.not_in_g2(), C.IDENTITY_G2, C.negate_g2(pks[0])]
    if path != "nocache":  # the committee in the key cache; the stray keys decoded per call
        bls.register_keys(pks)
    rnd = random.Random(14)
    items = []  # (sig, key index list, msg)
    for c in range(12):
        d = rnd.randbytes(32)
        who = sorted(rnd.sample(range(10), 7))
        sigs = bls.sign([sks[k] for k in who], [d] * 7)
        _, agg = B.aggregate(sigs)
        items.append((agg, who, d))
    agg, who, d = items[0]
    items += [
        (agg, who, d + b"!"),                  # wrong message
        (agg, who[:-1], d),                    # missing signer
        (agg, who[:-1] + [9 if 9 not in who else 8], d),  # wrong signer
        (agg, [], d),                          # empty key list
        (agg, who + [10], d),                  # a key outside G2
        (agg, who + [11], d),                  # identity key
        (agg, [0, 12], d),                     # apk = identity (pk + (-pk))
        (C.not_in_g1(), who, d),               # signature outside G1
        (C.IDENTITY_G1, who, d),               # identity signature
    ] + [(b, who, d) for b in C.bad_encodings_g1(agg)]
    got = bls.verify_many(keys, [i[0] for i in items], [i[1] for i in items], [i[2] for i in items])
    want = [B.fast_aggregate_verify(s, [keys[k] for k in ks], m) for s, ks, m in items]
    assert list(got) == want
    assert want[:12] == [0] * 12 and all(w != 0 for w in want[12:])
    # the wrong-message / wrong-signer items fail only the pairing equation: the batch check rejects
    assert bls.last_path() == EXPECT_PATH[path][0]
    # the valid certificates alone: the batch check accepts them in one final exponentiation
    got = bls.verify_many(keys, [i[0] for i in items[:12]], [i[1] for i in items[:12]], [i[2] for i in items[:12]])
    assert list(got) == [0] * 12
    assert bls.last_path() == EXPECT_PATH[path][1]
    # valid certificates beside items that fail before the pairing (decode / group / key errors):
    # those stay out of the batch check, which accepts the rest
    pre = [it for it, w in zip(items, want) if w not in (0, B.ORB_VERIFY_FAIL)]
    sub = items[:12] + pre
    got = bls.verify_many(keys, [i[0] for i in sub], [i[1] for i in sub], [i[2] for i in sub])
    assert list(got) == [B.fast_aggregate_verify(s, [keys[k] for k in ks], m) for s, ks, m in sub]
    assert bls.last_path() == EXPECT_PATH[path][1]
    # the same keys in another order and with duplicates (cache hits, repeated slots)
    perm = list(range(len(keys)))[::-1]
    keys2 = [keys[p] for p in perm] + [keys[0]]
    inv = {p: j for j, p in enumerate(perm)}
    items2 = [(s_, [inv[k] for k in ks] + ([len(keys)] if ks and ks[0] == 0 else []), m) for s_, ks, m in items]
    got = bls.verify_many(keys2, [i[0] for i in items2], [i[1] for i in items2], [i[2] for i in items2])
    assert list(got) == [B.fast_aggregate_verify(s_, [keys2[k] for k in ks], m) for s_, ks, m in items2]


def test_trait_contract(bls, gold):
    """BLS analogue of crypto/src/tests/bls12377_tests.rs:138-297 through the fastcrypto surface"""
    from narwhal_amd import _lib
    sks = [bytes.fromhex(k["sk"]) for k in gold["keygen"]]
    pks = [bytes.fromhex(k["pk"]) for k in gold["keygen"]]
    m = bytes(range(32))
    sigs = bls.sign(sks, [m] * 4)
    assert all(bls.verify(pk, m, s) == _lib.NWV_OK for pk, s in zip(pks, sigs))
    assert bls.verify(pks[0], b"Bad message!", sigs[0]) == _lib.NWV_ERR_SIGNATURE
    assert bls.verify_batch_empty_fail(m, pks[:3], sigs[:3]) == _lib.NWV_OK
    assert bls.verify_batch_empty_fail(m, [], []) == _lib.NWV_ERR_EMPTY
    assert bls.verify_batch_empty_fail(m, pks[:2], sigs[:3]) == _lib.NWV_ERR_LENGTH
    assert bls.verify_batch_empty_fail(m, [pks[3]] + pks[1:3], sigs[:3]) == _lib.NWV_ERR_SIGNATURE
    rc, agg, st = bls.aggregate(sigs[:3])
    assert rc == 0 and agg == B.aggregate(sigs[:3])[1]
    assert bls.aggregate([])[0] == _lib.NWV_ERR_SIGNATURE
    assert bls.aggregate([sigs[0], C.not_in_g1()])[2] == B.ORB_NOT_IN_GROUP
    assert bls.aggregate_verify(agg, pks[:3], m) == _lib.NWV_OK
    assert bls.aggregate_verify(agg, pks[:2], m) == _lib.NWV_ERR_SIGNATURE
    assert bls.aggregate_verify(None, pks[:3], m) == _lib.NWV_ERR_SIGNATURE
    m2 = bytes(range(32, 64))
    _, agg2, _ = bls.aggregate(bls.sign(sks[1:], [m2] * 3))
    assert bls.aggregate_batch_verify([agg, agg2], [pks[:3], pks[1:]], [m, m2]) == _lib.NWV_OK
    assert bls.aggregate_batch_verify([agg, agg2], [pks[:3], pks[:3]], [m, m2]) == _lib.NWV_ERR_SIGNATURE
    assert bls.aggregate_batch_verify([agg, agg2], [pks[:3], pks[1:]], [m]) == _lib.NWV_ERR_LENGTH


def test_key_sums_many_keys(bls):
    """items naming many keys (the key sum runs on 8 lanes and a tree): 1..20 signers, a bad key at
    every position of the list (the first bad key's status wins), against the oracle"""
    sks, pks = _committee(bls, 20, 16)
    keys = pks + [C.not_in_g2(), C.IDENTITY_G2]
    rnd = random.Random(17)
    items = []
    for q in (1, 2, 7, 8, 9, 15, 16, 17, 20):
        who = sorted(rnd.sample(range(20), q))
        d = rnd.randbytes(32)
        _, agg = B.aggregate(bls.sign([sks[k] for k in who], [d] * q))
        items.append((agg, who, d))
        for pos in (0, q // 2, q - 1):
            bad = list(who)
            bad.insert(pos, 20)
            items.append((agg, bad, d))
            bad2 = list(bad)
            bad2.insert(0 if pos else 1, 21)  # an identity key before / after the subgroup failure
            items.append((agg, bad2, d))
    got = bls.verify_many(keys, [i[0] for i in items], [i[1] for i in items], [i[2] for i in items])
    assert list(got) == [B.fast_aggregate_verify(s, [keys[k] for k in ks], m) for s, ks, m in items]


@pytest.mark.parametrize("engine", ["wave", "batch"])
@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 200])
def test_batch_sizes(bls, bls_batch, n, engine):
    """batch tails around the 64-lane wave and the product tree's odd levels; every other item
    corrupted (message flipped), then the same items all valid (one accepted batch check)"""
    bls = {"wave": bls, "batch": bls_batch}[engine]
    sks, pks = _committee(bls, 4, 15)
    rnd = random.Random(n)
    msgs = [rnd.randbytes(32) for _ in range(n)]
    flat = bls.sign(sks[:3] * n, [m for m in msgs for _ in range(3)])
    sigs = [B.aggregate(flat[3 * i:3 * i + 3])[1] for i in range(n)]
    bad = [i % 2 == 1 for i in range(n)]
    msgs2 = [m + b"x" if b else m for m, b in zip(msgs, bad)]
    got = bls.verify_many(pks, sigs, [[0, 1, 2]] * n, msgs2)
    assert list(got) == [B.ORB_VERIFY_FAIL if b else 0 for b in bad]
    if engine == "wave":
        assert bls.last_path() == "wave"
    else:
        assert bls.last_path() == ("batch_accepted" if n == 1 else "batch_rejected_then_per_item")
    got = bls.verify_many(pks, sigs, [[0, 1, 2]] * n, msgs)
    assert list(got) == [0] * n and bls.last_path() == ("wave" if engine == "wave" else "batch_accepted")


def test_stage_times_small_and_large_calls(bls):
    """nwv_bls_last_kernel_ms: a call of at most 1,024 items records its per-stage timing events
    only on a NWV_FLAG_BLS_STAGE_TIMES context (zeros otherwise: the events cost a single
    verification ~0.1 ms); a larger call always records them.  Statuses are the same either way."""
    import narwhal_amd
    from narwhal_amd import _lib
    from narwhal_amd.bls import Bls
    sks, pks = _committee(bls, 4, 16)
    rnd = random.Random(5)
    msgs = [rnd.randbytes(32) for _ in range(1100)]
    sigs = bls.sign([sks[i % 4] for i in range(1100)], msgs)
    keys = [[i % 4] for i in range(1100)]
    assert not bls.verify_many(pks, sigs[:2], keys[:2], msgs[:2]).any()
    assert all(v == 0.0 for v in bls.last_kernel_ms().values())
    assert not bls.verify_many(pks, sigs, keys, msgs).any()  # > 1,024 items
    assert bls.last_kernel_ms()["pairing_check"] > 0.0
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_BLS_STAGE_TIMES)
    try:
        bt = Bls(e)
        assert not bt.verify_many(pks, sigs[:2], keys[:2], msgs[:2]).any()
        km = bt.last_kernel_ms()
        assert km["pairing_check"] > 0.0 and km["hash_to_g1"] > 0.0 and km["sig_decode"] > 0.0
    finally:
        e.close()


def test_keycache_register_only(bls):
    """the key cache takes only registered (committee) keys that validate: 70,000 stray keys named
    by verify calls (undecodable, off-curve, outside G2, and valid keys of outsiders) never take a
    slot, an invalid key passed to register takes none either, and the committee's keys still hit
    the cache afterwards with statuses equal to the oracle's"""
    bls.reset_keys()
    assert bls.cached_keys() == 0
    sks, pks = _committee(bls, 10, 21)
    bad_key = C.not_in_g2()
    bls.register_keys(pks + [bad_key, C.IDENTITY_G2])
    assert bls.cached_keys() == 10
    rnd = random.Random(22)
    d = rnd.randbytes(32)
    who = sorted(rnd.sample(range(10), 7))
    _, agg = B.aggregate(bls.sign([sks[k] for k in who], [d] * 7))
    # 70,000 distinct stray keys in verify calls: mostly undecodable (cheap to make and check), plus
    # invalid points and valid keys of outsiders signing their own messages
    osk, opk = _committee(bls, 16, 23)
    om = [rnd.randbytes(32) for _ in range(16)]
    osig = bls.sign(osk, om)
    stray = [bytes([0x80 | (i & 0x1f)]) + i.to_bytes(4, "big") + bytes(91) for i in range(70000 - 20)]
    stray = [bytes([k[0] & 0x7f]) + k[1:] if i % 3 == 0 else k for i, k in enumerate(stray)]
    stray += [C.not_in_g2(1000 * (i + 1)) for i in range(4)] + opk
    n0 = len(stray)
    items = [(C.IDENTITY_G1, [i], d) for i in range(n0 - 16)] + [(osig[j], [n0 - 16 + j], om[j]) for j in range(16)]
    for lo in range(0, len(items), 20000):
        part = items[lo:lo + 20000]
        got = bls.verify_many(stray, [i[0] for i in part], [i[1] for i in part], [i[2] for i in part])
        assert bls.last_keys()[0] == 0  # nothing found in the cache: none of them were registered
        want_tail = [0] * 16 if lo + 20000 >= len(items) else []
        if want_tail:
            assert list(got[-16:]) == want_tail  # the outsiders' valid single signatures verify
        sample = rnd.sample(range(len(part) - len(want_tail)), 40)
        sub_keys = [stray[part[k][1][0]] for k in sample]  # the oracle validates only these
        assert [int(got[k]) for k in sample] == B.verify_items(sub_keys, [part[k][0] for k in sample],
                                                               [[j] for j in range(len(sample))],
                                                               [part[k][2] for k in sample])
    assert bls.cached_keys() == 10  # no stray key took a slot
    # the committee's keys still come from the cache, statuses as the oracle's
    keys = pks + [bad_key]
    its = [(agg, who, d), (agg, who, d + b"!"), (agg, who + [10], d), (agg, who[:-1], d)]
    got = bls.verify_many(keys, [i[0] for i in its], [i[1] for i in its], [i[2] for i in its])
    assert list(got) == B.verify_items(keys, [i[0] for i in its], [i[1] for i in its], [i[2] for i in its])
    assert list(got)[0] == 0
    assert bls.last_keys() == (10, 1)  # the committee from the cache; the bad key decoded by the call
    bls.reset_keys()
    assert bls.cached_keys() == 0


@pytest.mark.parametrize("path", ["wave", "batch", "per_item"])
def test_committee_shape_100(bls, bls_batch, bls_per_item, path):
    """the reference's committee shape: a 100-key committee (registered), certificates of 67 and
    100 signers (the key-sum tree at full depth) mixed with every adversarial category, on the wave
    engine, through the batch check and per item, against the oracle"""
    bls = {"wave": bls, "batch": bls_batch, "per_item": bls_per_item}[path]
    sks, pks = _committee(bls, 100, 31)
    bls.register_keys(pks)
    keys = pks + [C.not_in_g2(), C.IDENTITY_G2, C.negate_g2(pks[5])]
    rnd = random.Random(32)
    items = []
    for q in (67, 100, 67, 68, 99, 100):
        d = rnd.randbytes(32)
        who = sorted(rnd.sample(range(100), q))
        _, agg = B.aggregate(bls.sign([sks[k] for k in who], [d] * q))
        items.append((agg, who, d))
    agg, who, d = items[0]
    agg2, who2, d2 = items[1]
    items += [
        (agg, who, d + b"!"),                                  # wrong message
        (agg, who[:-1], d),                                    # missing signer
        (agg, who[:-1] + [next(k for k in range(100) if k not in who)], d),  # wrong signer
        (agg2, who2[1:], d2),                                  # 99 of the 100 signers
        (agg, [], d),                                          # empty key list
        (agg, who[:30] + [100] + who[30:], d),                 # a key outside G2 mid-list
        (agg, who + [101], d),                                 # identity key last
        (agg, [5, 102], d),                                    # apk = identity (pk + (-pk))
        (C.not_in_g1(), who, d),                               # signature outside G1
        (C.IDENTITY_G1, who, d),                               # identity signature
        (agg2, who, d),                                        # another certificate's aggregate
    ] + [(b, who, d) for b in C.bad_encodings_g1(agg)]
    got = bls.verify_many(keys, [i[0] for i in items], [i[1] for i in items], [i[2] for i in items])
    want = B.verify_items(keys, [i[0] for i in items], [i[1] for i in items], [i[2] for i in items])
    assert list(got) == want
    assert want[:6] == [0] * 6 and all(w != 0 for w in want[6:])
    assert bls.last_path() == EXPECT_PATH[path][0]
    got = bls.verify_many(keys, [i[0] for i in items[:6]], [i[1] for i in items[:6]], [i[2] for i in items[:6]])
    assert list(got) == [0] * 6


@pytest.fixture(scope="module")
def bls_nosig():
    """a context under NWV_FLAG_NO_SIGCACHE: every aggregate decodes and G1-checks its signatures"""
    import narwhal_amd
    from narwhal_amd import _lib
    from narwhal_amd.bls import Bls
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_NO_SIGCACHE)
    yield Bls(e)
    e.close()


def test_aggregate_verified_signatures(bls, bls_nosig):
    """AggregateAuthenticator::aggregate over votes already verified (the Core's quorum of 67 of
    100): signatures that passed a verify call are summed from the device's ring (k_blsw_g1_sum
    through the ring positions), others are decoded and checked first; both equal the oracle, as
    do a context without the ring, repeated signatures, a not-yet-verified signature among
    verified ones, a bad one, and 1,100 signatures (three tree levels)"""
    from narwhal_amd import _lib
    sks, pks = _committee(bls, 100, 41)
    d = bytes(range(7, 39))
    sigs = bls.sign(sks, [d] * 100)
    got = bls.verify_many(pks, sigs[:67], [[k] for k in range(67)], [d] * 67)
    assert list(got) == [0] * 67
    for b in (bls, bls_nosig):
        for sub in (sigs[:67], sigs[:1], sigs[:32], sigs[:33], sigs[5:9] * 3, sigs[:66] + [sigs[80]]):
            rc, agg, st = b.aggregate(sub)
            want_rc, want = B.aggregate(sub)
            assert (rc, st) == (_lib.NWV_OK, want_rc) and agg == want
        rc, _, st = b.aggregate(sigs[:20] + [C.not_in_g1()] + sigs[20:40])
        assert rc == _lib.NWV_ERR_SIGNATURE and st == B.ORB_NOT_IN_GROUP
    rnd = random.Random(43)
    many = bls.sign([sks[k % 100] for k in range(1100)], [bytes([k % 251]) * 32 for k in range(1100)])
    for lo in range(0, 1100, 550):
        keys = [[k % 100] for k in range(lo, lo + 550)]
        assert list(bls.verify_many(pks, many[lo:lo + 550], keys,
                                    [bytes([k % 251]) * 32 for k in range(lo, lo + 550)])) == [0] * 550
    order = list(range(1100))
    rnd.shuffle(order)
    sub = [many[k] for k in order]
    rc, agg, st = bls.aggregate(sub)
    assert rc == _lib.NWV_OK and agg == B.aggregate(sub)[1]


def test_ring_wraps_under_concurrent_verifies_and_aggregates(bls):
    """the verified-signature ring (BlsSigCache, 65,536 slots) under load: 8 threads verify
    1,024-signature calls until the ring has wrapped (73,728 reservations) while 2 threads
    aggregate 67-signature subsets; every verify status is OK and every aggregate equals the
    oracle's (a slot re-reserved while a call or an aggregate still used it would show up as a
    wrong sum)"""
    import threading
    from narwhal_amd import _lib
    sks, pks = _committee(bls, 100, 51)
    msgs = [bytes([k % 251, k // 251]) * 16 for k in range(1024)]
    sigs = bls.sign([sks[k % 100] for k in range(1024)], msgs)
    keys = [[k % 100] for k in range(1024)]
    errs = []
    stop = threading.Event()

    def verifier():
        try:
            for _ in range(9):
                st = bls.verify_many(pks, sigs, keys, msgs)
                if list(st) != [0] * 1024:
                    errs.append(("verify", [int(x) for x in st if x][:4]))
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(("verify", repr(e)))

    def aggregator(seed):
        rnd = random.Random(seed)
        try:
            while not stop.is_set():
                sub = [sigs[k] for k in rnd.sample(range(1024), 67)]
                rc, agg, st = bls.aggregate(sub)
                want_rc, want = B.aggregate(sub)
                if (rc, st, agg) != (_lib.NWV_OK, want_rc, want):
                    errs.append(("aggregate", rc, st))
        except Exception as e:  # noqa: BLE001
            errs.append(("aggregate", repr(e)))

    vs = [threading.Thread(target=verifier) for _ in range(8)]
    ags = [threading.Thread(target=aggregator, args=(s,)) for s in (1, 2)]
    for t in vs + ags:
        t.start()
    for t in vs:
        t.join()
    stop.set()
    for t in ags:
        t.join()
    assert not errs, errs[:5]


def test_verify_many_sharded_over_devices():
    """nwv_bls_verify_many over a multi-device context: the items split by index over three BLS
    shards on this GPU (NWV_BLS_DEVICE_REPLICAS, the test hook of bls_shard.h), keys registered on
    every shard, statuses merged in item order -- equal to the oracle with and without the cache"""
    import subprocess
    import sys
    env = dict(os.environ, NWV_BLS_DEVICE_REPLICAS="3", NWV_BLS_SHARD_MIN="8")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "bls_shard_gpu_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["shards"] == 3 and out["items"] > 48 and out["want_nonzero"] >= 7
    assert out["registered_on_shard0"] == 100
    assert out["cached_equal"] and out["uncached_equal"], out


@pytest.mark.parametrize("pack", ["1", "2", "3", "4"])
def test_verify_many_packed_waves(pack):
    """the throughput path's pairing kernel with `pack` items per wave (k_blsw_pair_k, one LDS bank
    per item; NWV_BLS_WAVE_MAX=0 sends every call there): the 100-key committee round with every
    adversarial category, with and without the key cache (precomputed vs computed key lines), equal
    to the oracle -- including a last wave holding fewer items"""
    import subprocess
    import sys
    env = dict(os.environ, NWV_BLS_WAVE_MAX="0", NWV_BLS_PACK=pack, NWV_BLS_DEVICE_REPLICAS="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "bls_shard_gpu_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["items"] % 3 != 0 and out["want_nonzero"] >= 7
    assert out["cached_equal"] and out["uncached_equal"], out
