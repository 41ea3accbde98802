"""GPU parity of batch verification through the Pippenger MSM (K5, msm_kernels.hip) via the C
ABI: the batch verdict equals the AND of the oracle's per-signature ZIP-215 verdicts on valid,
invalid and adversarial batches of every size class (window widths 6..15 are chosen from n),
and a rejected batch's fallback pinpoints exactly the oracle's bad indices (config 4)."""
import random

import numpy as np
import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    from narwhal_amd import _lib
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_ALWAYS)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng_nokc():
    """keyed calls without the committee key cache (full-width scalars, keys decompressed per call)"""
    import narwhal_amd
    from narwhal_amd import _lib
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_ALWAYS | _lib.NWV_FLAG_NO_KEYCACHE)
    yield e
    e.close()


@pytest.fixture(scope="module")
def eng_sort2():
    """the two-level counting sort (coarse bins, then k_msm_lsort) forced whenever the sort has
    more than one chunk; by default only windows of 2^20+ points use it"""
    import narwhal_amd
    from narwhal_amd import _lib
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_ALWAYS | _lib.NWV_FLAG_MSM_SORT2)
    yield e
    e.close()


@pytest.mark.parametrize("n", [5000, 40000])
def test_two_level_sort(eng, eng_sort2, n):
    """batches through the two-level sort: valid batches accept, three forged signatures are
    pinpointed exactly, and every golden / ZIP-215 vector inside a batch gives the oracle's
    verdict"""
    items = _synthetic(eng, n, 32, seed=300 + n)
    ok, bits = eng_sort2.verify_batch(items, seed=b"\x09" * 32)
    assert ok and all(bits)
    bad = [0, n // 3, n - 1]
    forged = list(items)
    for i in bad:
        p, s_, m = forged[i]
        forged[i] = (p, s_[:10] + bytes([s_[10] ^ 0x40]) + s_[11:], m)
    ok, bits = eng_sort2.verify_batch(forged)
    assert not ok and [i for i in range(n) if not bits[i]] == bad
    if n == 5000:
        g = of.load_golden("ed25519_vectors.json")["vectors"]
        z = of.load_golden("zip215_small_order.json")["vectors"]
        vecs = [_v(v) for v in g + z]
        batch = items[:n - len(vecs)] + vecs
        want = all(of.verify(*v) for v in vecs)
        ok, _ = eng_sort2.verify_batch(batch)
        assert ok == want


@pytest.fixture(params=["keycache", "nokeycache"])
def keng(request, eng, eng_nokc):
    return eng if request.param == "keycache" else eng_nokc


def _v(v):
    return bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])


def _synthetic(eng, n, mlen, seed=1):
    rnd = np.random.default_rng(seed)
    seeds = [rnd.bytes(32) for _ in range(n)]
    msgs = [rnd.bytes(mlen) for _ in range(n)]
    pk, sg = eng.sign_many(seeds, msgs)
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    return items


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 300, 1024, 5000, 40000])
def test_valid_batches_accept(eng, n):
    items = _synthetic(eng, n, 32 if n > 1000 else 77, seed=n)
    ok, bits = eng.verify_batch(items, seed=bytes([n % 251]) * 32)
    assert ok and all(bits)


@pytest.mark.parametrize("n", [1, 64, 1000, 5000])
def test_one_bad_signature_rejects_and_is_pinpointed(eng, n):
    items = _synthetic(eng, n, 32, seed=100 + n)
    rnd = random.Random(n)
    i = rnd.randrange(n)
    pk, sg, m = items[i]
    sg = bytearray(sg)
    sg[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
    items[i] = (pk, bytes(sg), m)
    ok, bits = eng.verify_batch(items)
    want = [of.verify(*it) for it in items] if n <= 1000 else None
    assert not ok
    assert [k for k in range(n) if not bits[k]] == [i]
    if want is not None:
        assert bits == want


def test_golden_and_zip215_vectors_in_batches(eng):
    g = of.load_golden("ed25519_vectors.json")["vectors"]
    z = of.load_golden("zip215_small_order.json")["vectors"]
    honest = _synthetic(eng, 40, 32, seed=3)
    for k, v in enumerate(g + z):
        items = honest[: k % 7] + [_v(v)] + honest[k % 7:]
        want = [of.verify(*it) for it in items]
        ok, bits = eng.verify_batch(items, seed=bytes([k % 256]) * 32)
        assert ok == all(want), (k, v.get("category"))
        assert bits == want


@pytest.fixture(scope="module")
def eng_noreuse():
    """the per-signature pass after a rejected MSM decompresses again (k_ed_points) instead of
    building its tables from the MSM's point records (k_ed_points_msm, the default)"""
    import narwhal_amd
    from narwhal_amd import _lib
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_ALWAYS | _lib.NWV_FLAG_NO_MSM_REUSE)
    yield e
    e.close()


def test_fallback_reuses_msm_points_exactly(eng, eng_noreuse):
    """a rejected batch holding every golden / ZIP-215 vector (undecodable R and A, non-canonical
    encodings, small-order points, negative zero) plus forged signatures: the fallback built from
    the MSM's decompressed records and the one that decompresses again both give the oracle's
    bits"""
    g = of.load_golden("ed25519_vectors.json")["vectors"]
    z = of.load_golden("zip215_small_order.json")["vectors"]
    items = _synthetic(eng, 300, 32, seed=11)
    for i in (5, 77, 299):
        p, s_, m = items[i]
        items[i] = (p, s_[:3] + bytes([s_[3] ^ 1]) + s_[4:], m)
    vecs = [_v(v) for v in g + z]
    batch = items[:150] + vecs + items[150:]
    want = [of.verify(*it) for it in batch]
    assert not all(want)
    for e in (eng, eng_noreuse):
        ok, bits = e.verify_batch(batch, seed=b"\x21" * 32)
        assert not ok and bits == want


def test_all_small_order_vectors_one_batch(eng):
    z = [_v(v) for v in of.load_golden("zip215_small_order.json")["vectors"]]
    ok, bits = eng.verify_batch(z)
    assert ok and all(bits)


def test_adversarial_mix_config4(eng):
    """config 4 shape: 1% invalid / non-canonical / small-order, batch false, exact bad set"""
    n = 20000
    items = _synthetic(eng, n, 32, seed=4)
    rnd = random.Random(4)
    bad = sorted(rnd.sample(range(n), n // 100))
    adv = [_v(v) for v in of.load_golden("ed25519_vectors.json")["vectors"] if v["category"] != "honest"]
    for j, i in enumerate(bad):
        if j % 2 == 0:
            pk, sg, m = items[i]
            sg = bytearray(sg)
            sg[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
            items[i] = (pk, bytes(sg), m)
        else:
            items[i] = adv[j % len(adv)]
    want = [True] * n
    for i in bad:
        want[i] = of.verify(*items[i])
    ok, bits = eng.verify_batch(items)
    assert not ok
    assert bits == want


@pytest.mark.parametrize("split", [False, True])
def test_staged_msm_runs_and_times(eng, split):
    """timed runs report every kernel of the batch MSM: k_msm_prep (hash + decompression in one
    grid) by default, k_msm_scalars and k_msm_points under NWV_FLAG_MSM_SPLIT_PREP; both launch
    shapes give the same verdicts, including the exact bad set"""
    from narwhal_amd import _lib
    e = _lib.Engine(device=0, flags=_lib.NWV_FLAG_MSM_ALWAYS | _lib.NWV_FLAG_MSM_SPLIT_PREP) if split else eng
    items = _synthetic(eng, 8192, 512, seed=9)
    pk, sg, arena, offs, lens = _lib.soa(items)
    st = e.stage(pk, sg, arena, offs, lens)
    for r in range(3):
        st.run(mode=1, seed=bytes([r]) * 32, timed=True)
    allv, bits = st.fetch()
    t = st.kernel_times(1)
    st.free()
    assert allv and bits.all()
    want = (["k_msm_scalars", "k_msm_points"] if split else ["k_msm_prep"]) + [
        "k_msm_hist", "k_msm_wscan", "k_msm_scatter", "k_msm_bucket", "k_msm_tail"]
    assert list(t) == want and all(v > 0 for v in t.values())
    bad = [5, 4000, 8191]
    for i in bad:
        p, s_, m = items[i]
        items[i] = (p, s_, m + b"x")
    ok, vb = e.verify_batch(items)
    if split:
        e.close()
    assert not ok and [i for i in range(len(items)) if not vb[i]] == bad


@pytest.mark.parametrize("chain", ["0", "1", "3"])
def test_staged_graph_replay_valid_and_invalid(eng, monkeypatch, chain):
    """untimed mode-1 runs replay with a fresh seed each time -- a captured HIP graph
    (NWV_STAGE_CHAIN=0) or direct launches whose preps are chained across runs (depth 1, 3 =
    default): verdicts stay exact for a valid batch and for one with a forged signature
    (fallback after fetch)"""
    from narwhal_amd import _lib
    monkeypatch.setenv("NWV_STAGE_CHAIN", chain)
    items = _synthetic(eng, 3000, 64, seed=21)
    pk, sg, arena, offs, lens = _lib.soa(items)
    st = eng.stage(pk, sg, arena, offs, lens)
    for r in range(5):
        st.run(mode=1, seed=bytes([r + 9]) * 32)
        allv, bits = st.fetch()
        assert allv and bits.all()
    # back-to-back replays with no host read in between: the device-side tally sees every one
    for r in range(7):
        st.run(mode=1)
    assert st.run_tally() == (12, 0)
    st.free()
    sg2 = sg.copy()
    sg2[64 * 1234 + 50] ^= 8
    st = eng.stage(pk, sg2, arena, offs, lens)
    for r in range(4):
        st.run(mode=1, seed=bytes([r + 1]) * 32)
        allv, bits = st.fetch()
        assert not allv and list(np.flatnonzero(~bits)) == [1234]
    assert st.run_tally() == (0, 4)
    st.free()


@pytest.mark.parametrize("chain", ["1", "2", "3"])
def test_staged_chain_across_batches(eng, monkeypatch, chain):
    """staged runs issued round-robin over five resident batches (one holding a forged signature)
    with no host read in between, each prep waiting for the prep `chain` runs earlier on another
    batch's stream: every run completes and each batch's device tally is exact"""
    from narwhal_amd import _lib
    monkeypatch.setenv("NWV_STAGE_CHAIN", chain)
    stages = []
    for b in range(5):
        items = _synthetic(eng, 1500 + 300 * b, 48, seed=40 + b)
        pk, sg, arena, offs, lens = _lib.soa(items)
        if b == 2:
            sg = sg.copy()
            sg[64 * 777 + 40] ^= 2
        st = eng.stage(pk, sg, arena, offs, lens)
        st.run(mode=1)  # first run: buffers (and, unchained, the graph)
        stages.append(st)
    for r in range(4):
        for st in stages:
            st.run(mode=1, seed=bytes([r + 3]) * 32)
    for b, st in enumerate(stages):
        assert st.run_tally() == ((0, 5) if b == 2 else (5, 0)), b
    allv, bits = stages[2].fetch()
    assert not allv and list(np.flatnonzero(~bits)) == [777]
    for st in stages:
        st.free()


def _keyed(items):
    keys, idx = [], {}
    kidx = []
    for pk, _, _ in items:
        if pk not in idx:
            idx[pk] = len(keys)
            keys.append(pk)
        kidx.append(idx[pk])
    return keys, kidx


@pytest.mark.parametrize("n,m", [(1, 1), (300, 4), (5000, 100), (20000, 7)])
def test_keyed_batches_committee(keng, n, m):
    """one MSM point per distinct key (configs[1] m = 100 variant, committee batches): valid
    batches accept; one forged signature is pinpointed exactly"""
    eng = keng
    rnd = np.random.default_rng(n + m)
    kseeds = [rnd.bytes(32) for _ in range(m)]
    msgs = [rnd.bytes(32) for _ in range(n)]
    pk, sg = eng.sign_many([kseeds[i % m] for i in range(n)], msgs)
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    keys, kidx = _keyed(items)
    assert len(keys) == m
    ok, bits = eng.verify_batch_keyed(keys, kidx, [s for _, s, _ in items], msgs, seed=b"\x03" * 32)
    assert ok and all(bits)
    bad = n // 2
    s = bytearray(items[bad][1])
    s[33] ^= 2
    sigs = [x[1] for x in items]
    sigs[bad] = bytes(s)
    ok, bits = eng.verify_batch_keyed(keys, kidx, sigs, msgs)
    assert not ok and [i for i in range(n) if not bits[i]] == [bad]
    # the same keys again (cache hits), in another order and with a subset of the committee
    perm = list(range(m))[::-1]
    keys2 = [keys[j] for j in perm]
    kidx2 = [perm.index(k) for k in kidx]
    ok, bits = eng.verify_batch_keyed(keys2, kidx2, [x[1] for x in items], msgs)
    assert ok and all(bits)


@pytest.mark.parametrize("fused", [True, False])
def test_keyed_small_batches_fused_keysum(eng, eng_nokc, fused):
    """keyed batches whose hashes fit one k_msm_prep workgroup sum their keys' scalars in that
    workgroup (no k_msm_keysum launch; NWV_FLAG_NO_FUSED_KEYSUM keeps the launch): key cache on
    and off, one signature per key, several per key, 64 signatures, and a forged signature or a
    signature over the wrong message pinpointed -- the oracle's verdicts either way"""
    import narwhal_amd
    from narwhal_amd import _lib
    engines = [eng, eng_nokc]
    if not fused:
        engines = [narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_ALWAYS | _lib.NWV_FLAG_NO_FUSED_KEYSUM | f)
                   for f in (0, _lib.NWV_FLAG_NO_KEYCACHE)]
    try:
        for e in engines:
            for n, m in [(1, 1), (4, 4), (7, 3), (17, 17), (64, 5), (64, 64)]:
                rnd = np.random.default_rng(1000 * n + m)
                kseeds = [rnd.bytes(32) for _ in range(m)]
                msgs = [rnd.bytes(32) for _ in range(n)]
                pk, sg = e.sign_many([kseeds[i % m] for i in range(n)], msgs)
                items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i])
                         for i in range(n)]
                keys, kidx = _keyed(items)
                sigs = [x[1] for x in items]
                ok, bits = e.verify_batch_keyed(keys, kidx, sigs, msgs, seed=bytes([n]) * 32)
                assert ok and all(bits), (n, m)
                bad = n - 1
                s = bytearray(sigs[bad])
                s[40] ^= 4
                sigs2 = list(sigs)
                sigs2[bad] = bytes(s)
                ok, bits = e.verify_batch_keyed(keys, kidx, sigs2, msgs)
                assert not ok and [i for i in range(n) if not bits[i]] == [bad], (n, m)
                msgs2 = list(msgs)
                msgs2[0] = msgs2[0][:-1] + bytes([msgs2[0][-1] ^ 1])
                ok, bits = e.verify_batch_keyed(keys, kidx, sigs, msgs2)
                assert not ok and [i for i in range(n) if not bits[i]] == [0], (n, m)
    finally:
        if not fused:
            for e in engines:
                e.close()


def test_keyed_many_keys_bypass_cache(eng):
    """a keyed call with more distinct keys than NWV_KEYCACHE_MAX_KEYS (4,096) goes uncached
    (full-width scalars); the same keys in a call of 3,000 distinct keys go through the cache:
    both give the oracle's verdicts, including one forged signature"""
    n = 6000
    items = _synthetic(eng, n, 32, seed=77)
    keys, kidx = _keyed(items)
    assert len(keys) == n
    sigs = [s for _, s, _ in items]
    msgs = [m for _, _, m in items]
    ok, bits = eng.verify_batch_keyed(keys, kidx, sigs, msgs)
    assert ok and all(bits)
    s = bytearray(sigs[4321])
    s[50] ^= 0x10
    sigs[4321] = bytes(s)
    ok, bits = eng.verify_batch_keyed(keys, kidx, sigs, msgs)
    assert not ok and [i for i in range(n) if not bits[i]] == [4321]
    sub = list(range(2000, 5000))  # 3,000 distinct keys: cached, including the forged signature
    ok, bits = eng.verify_batch_keyed([keys[i] for i in sub], list(range(len(sub))), [sigs[i] for i in sub],
                                      [msgs[i] for i in sub])
    assert not ok and [sub[i] for i in range(len(sub)) if not bits[i]] == [4321]


def test_keyed_golden_and_bad_keys(keng):
    """golden / ZIP-215 vectors (small-order, non-canonical and undecodable keys) keyed by their
    raw key bytes: verdicts equal the oracle's, and an unused undecodable key changes nothing"""
    g = of.load_golden("ed25519_vectors.json")["vectors"]
    z = of.load_golden("zip215_small_order.json")["vectors"]
    items = [_v(v) for v in g + z]
    keys, kidx = _keyed(items)
    want = [of.verify(*it) for it in items]
    eng = keng
    ok, bits = eng.verify_batch_keyed(keys, kidx, [s for _, s, _ in items], [m for _, _, m in items])
    assert bits == want and ok == all(want)
    good = [it for it, w in zip(items, want) if w]
    keys, kidx = _keyed(good)
    undecodable = bytes.fromhex("02" + "00" * 31)  # y = 2 is not on the curve
    assert not of.lib().or_point_decompress_ok(undecodable)
    ok, bits = eng.verify_batch_keyed(keys + [undecodable], kidx, [s for _, s, _ in good], [m for _, _, m in good])
    assert ok and all(bits)
    # every signature valid but one signer's key undecodable (cached with its failure flag on the
    # first call, a cache hit on the second): the batch rejects, the fallback pinpoints exactly it
    for _ in range(2):
        ok, bits = eng.verify_batch_keyed(keys + [undecodable], kidx + [len(keys)],
                                          [s for _, s, _ in good] + [good[0][1]], [m for _, _, m in good] + [b"x"])
        assert not ok and [i for i in range(len(bits)) if not bits[i]] == [len(good)]


def test_staged_keyed_msm(eng):
    from narwhal_amd import _lib
    rnd = np.random.default_rng(12)
    m, n = 100, 8192
    kseeds = [rnd.bytes(32) for _ in range(m)]
    msgs = [rnd.bytes(512) for _ in range(n)]
    pk, sg = eng.sign_many([kseeds[i % m] for i in range(n)], msgs)
    keys = np.concatenate([pk[32 * i:32 * i + 32] for i in range(m)])
    kidx = np.arange(n, dtype=np.uint32) % m
    arena, offs, lens = _lib.pack_messages(msgs)
    st = eng.stage_keyed(keys, kidx, sg, arena, offs, lens)
    for r in range(2):
        st.run(mode=1, seed=bytes([r + 1]) * 32)
    allv, bits = st.fetch()
    st.free()
    assert allv and bits.all()


@pytest.mark.parametrize("n_pre,n_sig", [(1, 1), (40, 700), (300, 7000)])
def test_keyed_digests_hash_then_verify(eng, n_pre, n_sig):
    """nwv_ed25519_verify_batch_keyed_digests: the preimages' BLAKE2b-256 digests
    come back equal to the oracle's, and signature i is checked over digest digest_idx[i] from
    device memory: verdicts equal the oracle's over the same bytes, a forged signature and a
    signature over another digest are pinpointed, an out-of-range digest index is an argument
    error"""
    rnd = random.Random(n_pre * 7 + n_sig)
    pre = [rnd.randbytes(rnd.choice([80, 127, 128, 129, 2200])) for _ in range(n_pre)]
    want_dig = [of.blake2b256(x) for x in pre]
    m = min(100, n_sig)
    kseeds = [rnd.randbytes(32) for _ in range(m)]
    didx = [rnd.randrange(n_pre) for _ in range(n_sig)]
    msgs = [want_dig[j] for j in didx]
    pk, sg = eng.sign_many([kseeds[i % m] for i in range(n_sig)], msgs)
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n_sig)]
    keys, kidx = _keyed(items)
    sigs = [s for _, s, _ in items]
    dig, ok, bits = eng.verify_batch_keyed_digests(pre, keys, kidx, sigs, didx, seed=b"\x05" * 32)
    assert dig == want_dig and ok and all(bits)
    bad = {n_sig // 2}
    s = bytearray(sigs[n_sig // 2])
    s[40] ^= 1
    sigs[n_sig // 2] = bytes(s)
    didx2 = list(didx)
    if n_pre > 1:  # signature 0 now points at a digest it did not sign
        didx2[0] = (didx[0] + 1) % n_pre
        bad.add(0)
    dig, ok, bits = eng.verify_batch_keyed_digests(pre, keys, kidx, sigs, didx2)
    assert dig == want_dig and not ok
    assert {i for i in range(n_sig) if not bits[i]} == bad
    if n_sig <= 700:
        want = [of.verify(items[i][0], sigs[i], want_dig[didx2[i]]) for i in range(n_sig)]
        assert bits == want
    with pytest.raises(Exception):
        eng.verify_batch_keyed_digests(pre, keys, kidx, sigs, [n_pre] * n_sig)
