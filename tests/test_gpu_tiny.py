"""The one-launch path for tiny keyed batches (narwhal_amd/csrc/tiny_kernels.hip k_ed_tiny): a keyed
batch of at most 64 signatures whose keys were registered (nwv_keycache_register: each key gets a
fixed-base comb table) is checked signature by signature in one kernel.  Its verdict bits must equal
the oracle's ZIP-215 verdicts (types/src/primary.rs:150-183, 307-328, 487-537 call sites) and those
of the batch MSM path (NWV_FLAG_NO_TINY) on every size 1..64, on forgeries of every kind, on every
golden / ZIP-215 vector (undecodable and small-order keys registered too), and through the types
layer (which registers its committee)."""
import random

import numpy as np
import pytest

import oracle_ffi as of
from narwhal_amd import _lib

pytestmark = pytest.mark.gpu
L_ORDER = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def engs():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    m = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_NO_TINY)
    yield e, m
    e.close()
    m.close()


def _committee(eng, n, seed):
    rnd = random.Random(seed)
    seeds = [rnd.randbytes(32) for _ in range(n)]
    pk, _ = eng.sign_many(seeds, [b""] * n)
    return seeds, [pk[32 * i:32 * i + 32].tobytes() for i in range(n)]


def _forge(sig, msg, kind):
    s = bytearray(sig)
    if kind == 0:
        s[3] ^= 0x10  # R
    elif kind == 1:
        s[40] ^= 0x01  # s
    elif kind == 2:
        msg = bytes([msg[0] ^ 0x80]) + msg[1:] if msg else b"\x01"
    else:
        v = int.from_bytes(bytes(s[32:]), "little") + L_ORDER  # s + l
        s[32:] = v.to_bytes(32, "little")
    return bytes(s), msg


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 17, 33, 63, 64])
def test_tiny_sizes_and_forgeries_match_oracle(engs, n):
    e, m = engs
    seeds, keys = _committee(e, 10, 1000 + n)
    for eng in (e, m):
        eng.keycache_register(keys)
    rnd = random.Random(n)
    kidx = [rnd.randrange(10) for _ in range(n)]
    msgs = [rnd.randbytes(rnd.choice([0, 1, 32, 200])) for _ in range(n)]
    _, sg = e.sign_many([seeds[k] for k in kidx], msgs)
    sigs = [sg[64 * i:64 * i + 64].tobytes() for i in range(n)]
    before = e.diag_counters()
    ok, bits = e.verify_batch_keyed(keys, kidx, sigs, msgs)
    assert ok and all(bits)
    assert e.diag_counters()["tiny"] == before["tiny"] + 1  # the one-launch path ran
    ok, _ = e.verify_batch_keyed(keys, kidx, sigs, msgs, want_bits=False)
    assert ok
    bad = sorted(rnd.sample(range(n), min(n, 1 + n // 5)))
    for j, i in enumerate(bad):
        sigs[i], msgs[i] = _forge(sigs[i], msgs[i], j % 4)
    want = [of.verify(keys[kidx[i]], sigs[i], msgs[i]) for i in range(n)]
    assert [i for i, w in enumerate(want) if not w] == bad
    ok, bits = e.verify_batch_keyed(keys, kidx, sigs, msgs)
    assert not ok and bits == want
    ok2, _ = e.verify_batch_keyed(keys, kidx, sigs, msgs, want_bits=False)
    assert not ok2
    okm, bm = m.verify_batch_keyed(keys, kidx, sigs, msgs)
    assert not okm and bm == want
    assert m.diag_counters()["tiny"] == 0


def test_tiny_golden_and_zip215_vectors(engs):
    """every committed vector (Appendix-B categories, the 196-case small-order table) as keyed
    batches of up to 64 over registered keys, undecodable and small-order keys included"""
    e, m = engs
    vecs = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]))
            for v in of.load_golden("ed25519_vectors.json")["vectors"]]
    vecs += [(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]))
             for v in of.load_golden("zip215_small_order.json")["vectors"]]
    keys = sorted({p for p, _, _ in vecs})
    kpos = {k: i for i, k in enumerate(keys)}
    for eng in (e, m):
        eng.keycache_register(keys)
    want = [of.verify(*v) for v in vecs]
    assert set(want) == {True, False}
    t0 = e.diag_counters()["tiny"]
    got = []
    for a in range(0, len(vecs), 64):
        chunk = vecs[a:a + 64]
        ok, bits = e.verify_batch_keyed(keys, [kpos[p] for p, _, _ in chunk], [s for _, s, _ in chunk],
                                        [x for _, _, x in chunk])
        assert ok == all(bits)
        got += bits
    assert got == want
    assert e.diag_counters()["tiny"] > t0
    # one signature at a time (Verifier::verify through nwv_ed25519_pubkey_verify)
    for (p, s, x), w in zip(vecs, want):
        rc = e.lib.nwv_ed25519_pubkey_verify(e._h, p, x, len(x), s)
        assert rc == (_lib.NWV_OK if w else _lib.NWV_ERR_SIGNATURE), (p.hex(), s.hex())


def test_unregistered_keys_take_the_msm(engs):
    """keys the call caches itself (not registered) have no comb table: the batch MSM runs"""
    e, _ = engs
    seeds, keys = _committee(e, 6, 77)
    msgs = [b"m%d" % i for i in range(6)]
    _, sg = e.sign_many(seeds, msgs)
    before = e.diag_counters()
    ok, bits = e.verify_batch_keyed(keys, list(range(6)), [sg[64 * i:64 * i + 64].tobytes() for i in range(6)], msgs)
    assert ok and all(bits)
    after = e.diag_counters()
    assert after["tiny"] == before["tiny"] and after["msm"] == before["msm"] + 1


def test_types_layer_certificates_take_the_tiny_path(engs):
    """Certificate::verify over a registered committee (the types layer registers it): one digest
    launch and k_ed_tiny; codes equal the oracle restatement, forged votes included"""
    import types_util as tu
    from types_util import nt
    from narwhal_amd import types as T
    e, _ = engs
    fx = nt.CommitteeFixture(7, of.pubkey, of.sign, seed=17)
    c = tu.committee(fx.committee)
    h = fx.header()
    q = fx.committee.quorum_threshold()
    cert = tu.oracle_certificate(fx, h, list(range(1, q + 1)))
    t0 = e.diag_counters()["tiny"]
    assert T.verify_certificates(e, c, [tu.certificate(cert)]) == [0]
    s = cert["sigs"][2]
    bad = dict(cert, sigs=cert["sigs"][:2] + [s[:5] + bytes([s[5] ^ 2]) + s[6:]] + cert["sigs"][3:])
    got = T.verify_certificates(e, c, [tu.certificate(bad)])
    assert got == [nt.certificate_verify(fx.committee, bad, of.verify)] and got[0] != 0
    assert e.diag_counters()["tiny"] >= t0 + 2
