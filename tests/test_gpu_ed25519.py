"""GPU parity: per-signature verdicts of the HIP engine (through the C ABI) are identical to
the oracle's / the golden fixtures' on the same inputs, including adversarial mixes, and the
batch / fastcrypto trait entry points follow the reference's error behaviour."""
import os
import random

import numpy as np
import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    yield e
    e.close()


def _v(v):
    return bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])


def test_golden_vectors_bit_exact(eng):
    g = of.load_golden("ed25519_vectors.json")
    items = [_v(v) for v in g["vectors"]]
    got = eng.verify_each(items)
    assert got == [v["expect"] for v in g["vectors"]]


def test_zip215_small_order_196(eng):
    g = of.load_golden("zip215_small_order.json")
    assert all(eng.verify_each([_v(v) for v in g["vectors"]]))


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 1000])
def test_sizes_and_tails(eng, n):
    g = of.load_golden("ed25519_vectors.json")
    vecs = [_v(v) for v in g["vectors"]]
    rnd = random.Random(n)
    items = [rnd.choice(vecs) for _ in range(n)]
    assert eng.verify_each(items) == [of.verify(*it) for it in items]


def test_empty(eng):
    assert eng.verify_each([]) == []


def _synthetic(eng, n, mlen, seed=1):
    rnd = np.random.default_rng(seed)
    seeds = [rnd.bytes(32) for _ in range(n)]
    msgs = [rnd.bytes(mlen) for _ in range(n)]
    pk, sg = eng.sign_many(seeds, msgs)
    return seeds, msgs, pk, sg


def test_gpu_signer_matches_rfc8032(eng):
    seeds, msgs, pk, sg = _synthetic(eng, 300, 77)
    for i in range(0, 300, 7):
        assert pk[32 * i:32 * i + 32].tobytes() == of.pubkey(seeds[i])
        assert sg[64 * i:64 * i + 64].tobytes() == of.sign(seeds[i], msgs[i])


def test_adversarial_mix_fallback_pinpoints_bad_indices(eng):
    # config 4 shape at test size: 1% corrupted (seeded positions), every category
    n = 20000
    seeds, msgs, pk, sg = _synthetic(eng, n, 32, seed=4)
    pk = pk.copy()
    sg = sg.copy()
    rnd = random.Random(4)
    bad = sorted(rnd.sample(range(n), n // 100))
    g = of.load_golden("ed25519_vectors.json")
    adv = [_v(v) for v in g["vectors"] if v["category"] != "honest"]
    msgs = list(msgs)
    for j, i in enumerate(bad):
        if j % 2 == 0:
            sg[64 * i + rnd.randrange(64)] ^= 1 << rnd.randrange(8)
        else:
            a = adv[j % len(adv)]
            pk[32 * i:32 * i + 32] = np.frombuffer(a[0], dtype=np.uint8)
            sg[64 * i:64 * i + 64] = np.frombuffer(a[1], dtype=np.uint8)
            msgs[i] = a[2]
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    all_valid, bits = eng.verify_batch(items)
    want = [True] * n
    for i in bad:
        want[i] = of.verify(*items[i])
    assert bits == want
    assert all_valid == all(want)
    assert not all_valid
    assert [i for i in range(n) if not bits[i]] == [i for i in range(n) if not want[i]]


def test_unaligned_and_shared_messages(eng):
    g = of.load_golden("ed25519_vectors.json")
    vecs = [_v(v) for v in g["vectors"]][:40]
    from narwhal_amd import _lib
    pk, sig, arena, offs, lens = _lib.soa(vecs)
    # shift the whole arena by 3 bytes: every message becomes unaligned
    arena2 = np.concatenate([np.zeros(3, dtype=np.uint8), arena])
    got = eng.verify_each_arrays(pk, sig, arena2, offs + 3, lens)
    assert list(got) == [of.verify(*v) for v in vecs]
    # certificate shape: one shared 32-byte digest, all offsets 0
    seeds = [bytes([i]) * 32 for i in range(10)]
    digest = bytes(range(32))
    items = [(of.pubkey(s), of.sign(s, digest), digest) for s in seeds]
    pk, sig, _, _, _ = _lib.soa(items)
    arena = np.frombuffer(digest + bytes(16), dtype=np.uint8)
    got = eng.verify_each_arrays(pk, sig, arena, np.zeros(10, np.uint64), np.full(10, 32, np.uint32))
    assert got.all()


def test_trait_contract(eng):
    """Ed25519 analogue of crypto/src/tests/bls12377_tests.rs:138-297."""
    import ctypes
    from narwhal_amd import _lib
    lib = eng.lib
    keys = [bytes([i + 1]) * 32 for i in range(4)]
    digest = bytes(range(32))
    pks = b"".join(of.pubkey(k) for k in keys[:3])
    sigs = b"".join(of.sign(k, digest) for k in keys[:3])
    seed = b"\x11" * 32
    ok = lib.nwv_ed25519_verify_batch_empty_fail(eng._h, digest, 32, pks, 3, sigs, 3, seed)
    assert ok == _lib.NWV_OK
    assert lib.nwv_ed25519_verify_batch_empty_fail(eng._h, digest, 32, None, 0, None, 0, seed) == _lib.NWV_ERR_EMPTY
    assert lib.nwv_ed25519_verify_batch_empty_fail(eng._h, digest, 32, pks[32:], 2, sigs, 3, seed) == _lib.NWV_ERR_LENGTH
    bad = bytearray(sigs)
    bad[0:64] = bytes(64)
    assert lib.nwv_ed25519_verify_batch_empty_fail(eng._h, digest, 32, pks, 3, bytes(bad), 3, seed) == _lib.NWV_ERR_SIGNATURE
    assert lib.nwv_ed25519_aggregate_verify(eng._h, sigs, 3, pks, 3, digest, 32, seed) == _lib.NWV_OK
    assert lib.nwv_ed25519_aggregate_verify(eng._h, sigs, 3, pks[:64], 2, digest, 32, seed) == _lib.NWV_ERR_LENGTH
    swapped = of.pubkey(keys[3]) + pks[32:]
    assert lib.nwv_ed25519_aggregate_verify(eng._h, sigs, 3, swapped, 3, digest, 32, seed) == _lib.NWV_ERR_SIGNATURE
    assert lib.nwv_ed25519_pubkey_verify(eng._h, pks[:32], digest, 32, sigs[:64]) == _lib.NWV_OK
    assert lib.nwv_ed25519_pubkey_verify(eng._h, pks[:32], b"Bad message!", 12, sigs[:64]) == _lib.NWV_ERR_SIGNATURE
    # batch_verify over two aggregates with different messages
    d2 = bytes(range(32, 64))
    sigs2 = b"".join(of.sign(k, d2) for k in keys[1:4])
    pks2 = b"".join(of.pubkey(k) for k in keys[1:4])
    arr = lambda *xs: (ctypes.c_char_p * len(xs))(*xs)
    sz = lambda *xs: (ctypes.c_size_t * len(xs))(*xs)
    rc = lib.nwv_ed25519_aggregate_batch_verify(eng._h, 2, arr(sigs, sigs2), sz(3, 3), arr(pks, pks2),
                                                sz(3, 3), arr(digest, d2), sz(32, 32), 2, seed)
    assert rc == _lib.NWV_OK
    rc = lib.nwv_ed25519_aggregate_batch_verify(eng._h, 2, arr(sigs, sigs2), sz(3, 3), arr(pks, pks2),
                                                sz(3, 2), arr(digest, d2), sz(32, 32), 2, seed)
    assert rc == _lib.NWV_ERR_LENGTH
    rc = lib.nwv_ed25519_aggregate_batch_verify(eng._h, 2, arr(sigs, sigs2), sz(3, 3), arr(pks, pks2),
                                                sz(3, 3), arr(digest), sz(32), 1, seed)
    assert rc == _lib.NWV_ERR_LENGTH


@pytest.mark.parametrize("golden", ["ed25519_vectors.json", "zip215_small_order.json"])
def test_single_verify_each_vector_alone(golden):
    """Verifier::verify (nwv_ed25519_pubkey_verify, a one-signature keyed MSM) on every golden and
    ZIP-215 small-order vector on its own, so no batch AND can hide a wrong individual verdict:
    first with the key unseen (uncached form: single verifies only look the key cache up), then
    after nwv_keycache_register (cache hit, 128-bit scalars), then on a context without the key
    cache -- each verdict equal to the oracle's."""
    import narwhal_amd
    from narwhal_amd import _lib
    vecs = [_v(v) for v in of.load_golden(golden)["vectors"]]
    want = [of.verify(*it) for it in vecs]
    e = narwhal_amd.Engine(device=0)
    e2 = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_NO_KEYCACHE)
    try:
        def run(engine):
            return [engine.lib.nwv_ed25519_pubkey_verify(engine._h, pk, m, len(m), sg) == _lib.NWV_OK
                    for pk, sg, m in vecs]
        assert run(e) == want                       # keys not in the cache
        keys = b"".join(sorted({pk for pk, _, _ in vecs}))
        _check = e.lib.nwv_keycache_register(e._h, len(keys) // 32, keys)
        assert _check == _lib.NWV_OK
        assert run(e) == want                       # every key cached (undecodable ones flagged)
        assert run(e2) == want                      # key cache disabled
    finally:
        e.close()
        e2.close()


def test_staged_resident_batch(eng):
    seeds, msgs, pk, sg = _synthetic(eng, 4096, 512, seed=9)
    from narwhal_amd import _lib
    arena, offs, lens = _lib.pack_messages(msgs)
    st = eng.stage(pk, sg, arena, offs, lens)
    for _ in range(3):
        st.run(mode=0, timed=True)
    allv, bits = st.fetch()
    ms = st.kernel_ms()
    st.free()
    assert allv and bits.all()
    assert (ms > 0).all()
