"""GPU parity at BASELINE.json's own sizes (configs C1-C4), through the C ABI, against the oracle.

  C1  Certificate::verify of a 4-node committee (header + 3 votes) and verify_batch of 1,024
      random signatures over 32-byte messages, distinct keys
  C2  verify_batch of 65,536 valid signatures over 512-byte messages, distinct keys (and the
      100-key committee variant): batch verdict, and the per-signature pipeline's bits against the
      oracle's per-signature verdicts for all 65,536
  C3  one firehose shard of 2,097,152 signatures (the 8-GPU share of 16M, 32-byte messages) with
      seeded corrupted indices: the shard's merged verdict bitmap has exactly those bad indices
  C4  65,536 x 512 B with 1 % adversarial entries over every SURVEY Appendix-B category: GPU bits
      equal the oracle's bits for all 65,536 signatures (MSM path with fallback and per-signature
      path), batch verdict false, bad set identical

Semantics: ed25519_consensus (ZIP-215) as called from types/src/primary.rs:150-183, :487-537 and
primary/src/block_synchronizer/responses.rs:95-141 (exact invalid set).  The oracle runs on the
box's CPU share (at most 16 threads)."""
import os
import sys

import numpy as np
import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    yield e
    e.close()


def _synth_arrays(eng, n, mlen, seed, keys=0):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    if keys:
        seeds = np.tile(seeds[:32 * keys], (n + keys - 1) // keys)[:32 * n].copy()
    msgs = rng.integers(0, 256, size=n * mlen + 64, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(mlen)
    lens = np.full(n, mlen, dtype=np.uint32)
    pk, sg = eng.sign_many_arrays(seeds, msgs, offs, lens)
    return pk, sg, msgs, offs, lens


def _oracle_bits(pk, sg, msgs, offs, lens):
    n = len(offs)
    words = of.verify_each_mt(bytes(pk[:32 * n]), bytes(sg[:64 * n]), bytes(msgs), offs.copy(), lens.copy(),
                              _threads())
    return np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)


def _gpu_batch(eng, pk, sg, msgs, offs, lens):
    from narwhal_amd import _lib
    import ctypes
    n = len(offs)
    bits = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
    allv = _lib._i32(0)
    _lib._check(eng.lib.nwv_ed25519_verify_batch(eng._h, n, _lib._ptr(pk), _lib._ptr(sg), _lib._ptr(msgs),
                                                 _lib._ptr(offs), _lib._ptr(lens), None, ctypes.byref(allv),
                                                 _lib._ptr(bits)))
    return bool(allv.value), _lib.unpack_bits(bits, n)


def test_c1_certificate_n4_and_batch_1024(eng):
    import config_legs as CL
    from types_util import nt
    from narwhal_amd import types as T
    seeds, keys, com = CL.committee_fixture(eng, 4, b"nwv-test-c1")
    headers, votes, certs = CL.dag_round(eng, seeds, keys, com)
    ocom = nt.Committee(list(com.keys), list(com.stakes), com.epoch, [list(w) for w in com.workers])
    for cert in certs:
        assert len(cert.aggregated_signature) == 3
        T.verify(eng, com, cert)  # raises on any DagError
        h = cert.header
        hd = {"author": h.author, "round": h.round, "epoch": h.epoch, "payload": list(h.payload),
              "parents": list(h.parents), "id": h.id, "signature": h.signature}
        assert nt.header_verify(ocom, hd, of.verify) == 0
        d = nt.certificate_digest(h.id, h.round, h.epoch, h.author)
        pks = [com.keys[a] for a in cert.signed_authorities]
        assert all(of.verify(pk, s, d) for pk, s in zip(pks, cert.aggregated_signature))
    # a forged vote signature: the GPU rejects it as the oracle does
    bad = certs[0]
    s = bytearray(bad.aggregated_signature[1])
    s[7] ^= 4
    bad.aggregated_signature[1] = bytes(s)
    with pytest.raises(T.InvalidSignature):
        T.verify(eng, com, bad)
    pk, sg, msgs, offs, lens = _synth_arrays(eng, 1024, 32, seed=11)
    ok, bits = _gpu_batch(eng, pk, sg, msgs, offs, lens)
    want = _oracle_bits(pk, sg, msgs, offs, lens)
    assert ok and bits.all() and want.all()
    sg2 = sg.copy()
    for i in (0, 500, 1023):
        sg2[64 * i + 33] ^= 1
    ok, bits = _gpu_batch(eng, pk, sg2, msgs, offs, lens)
    want = _oracle_bits(pk, sg2, msgs, offs, lens)
    assert not ok and (bits == want).all() and list(np.flatnonzero(~bits)) == [0, 500, 1023]


@pytest.mark.parametrize("keys", [0, 100])
def test_c2_65536_x_512(eng, keys):
    n = 65536
    pk, sg, msgs, offs, lens = _synth_arrays(eng, n, 512, seed=2000 + keys, keys=keys)
    want = _oracle_bits(pk, sg, msgs, offs, lens)
    assert want.all()
    if keys:
        kidx = list(np.arange(n) % keys)
        keyl = [pk[32 * k:32 * k + 32].tobytes() for k in range(keys)]
        sigl = [sg[64 * i:64 * i + 64].tobytes() for i in range(n)]
        msgl = [msgs[512 * i:512 * i + 512].tobytes() for i in range(n)]
        ok, bits = eng.verify_batch_keyed(keyl, kidx, sigl, msgl)
        assert ok and all(bits)
        # the same keyed batch with forged entries (R / s / message bit flips, s + l): the batch
        # rejects and the per-signature bits equal the oracle's on every signature
        rng = np.random.default_rng(keys)
        forged = sorted(int(x) for x in rng.choice(n, size=64, replace=False))
        sg2, m2 = sg.copy(), msgs.copy()
        L_ORDER = 2**252 + 27742317777372353535851937790883648493
        for j, i in enumerate(forged):
            if j % 4 == 0:
                sg2[64 * i + 7] ^= 0x10
            elif j % 4 == 1:
                sg2[64 * i + 40] ^= 0x01
            elif j % 4 == 2:
                m2[512 * i + 300] ^= 0x80
            else:
                sv = int.from_bytes(sg2[64 * i + 32:64 * i + 64].tobytes(), "little") + L_ORDER
                sg2[64 * i + 32:64 * i + 64] = np.frombuffer(sv.to_bytes(32, "little"), dtype=np.uint8)
        ok, bits = eng.verify_batch_keyed(keyl, kidx, [sg2[64 * i:64 * i + 64].tobytes() for i in range(n)],
                                          [m2[512 * i:512 * i + 512].tobytes() for i in range(n)])
        want2 = _oracle_bits(pk, sg2, m2, offs, lens)
        assert not ok and list(bits) == list(want2)
        assert list(np.flatnonzero(~want2)) == forged
        return
    ok, bits = _gpu_batch(eng, pk, sg, msgs, offs, lens)
    assert ok and bits.all()
    each = eng.verify_each_arrays(pk, sg, msgs, offs, lens)
    assert (each == want).all()
    # resident batch: repeated graph-replayed MSM runs with fresh seeds all accept
    st = eng.stage(pk, sg, msgs, offs, lens)
    try:
        for _ in range(3):
            st.run(mode=1)
            allv, b = st.fetch()
            assert allv and b.all()
    finally:
        st.free()


def test_c3_firehose_shard_2m(eng):
    """the 8-GPU share of configs[2]: 2,097,152 signatures verified as one resident shard (batch MSM,
    fallback only because the shard holds bad entries); the merged bitmap's bad set is exactly the
    injected one, and the oracle's per-signature bits equal the GPU's on all 2,097,152"""
    from narwhal_amd import firehose as fh
    n_total, world = 16777216, 8
    lo, hi = fh.shard_range(n_total, world, 3)
    m = hi - lo
    assert m == 2097152
    idx = np.arange(lo, hi, dtype=np.uint64)
    seeds = np.zeros((m, 32), dtype=np.uint8)
    seeds[:, :8] = idx.view(np.uint8).reshape(m, 8)
    seeds[:, 8] = 0xA5
    msgs = np.zeros((m, 32), dtype=np.uint8)
    msgs[:, :8] = (idx * np.uint64(0x9E3779B97F4A7C15)).view(np.uint8).reshape(m, 8)
    msgs = np.concatenate([msgs.reshape(-1), np.zeros(64, np.uint8)])
    offs = np.arange(m, dtype=np.uint64) * np.uint64(32)
    lens = np.full(m, 32, dtype=np.uint32)
    pk, sg = eng.sign_many_arrays(seeds.reshape(-1), msgs, offs, lens)
    rng = np.random.default_rng(3)
    bad = sorted(int(x) for x in rng.choice(m, size=41, replace=False))
    L_ORDER = 2**252 + 27742317777372353535851937790883648493
    for j, i in enumerate(bad):
        k = j % 4
        if k == 0:
            sg[64 * i + 5] ^= 0x40          # R bit flip
        elif k == 1:
            sg[64 * i + 50] ^= 0x02         # s bit flip
        elif k == 2:
            msgs[32 * i + 31] ^= 0x01       # message bit flip
        else:                               # s + l: non-canonical scalar
            s = int.from_bytes(sg[64 * i + 32:64 * i + 64].tobytes(), "little") + L_ORDER
            sg[64 * i + 32:64 * i + 64] = np.frombuffer(s.to_bytes(32, "little"), dtype=np.uint8)
    verify = fh.gpu_shard_verifier(eng, pk, sg, msgs, offs, lens)
    ok, words = fh.merge_verdicts([(0, m) + verify(0, m)], m)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:m].astype(bool)
    assert not ok
    assert list(np.flatnonzero(~bits)) == bad
    want = _oracle_bits(pk, sg, msgs, offs, lens)
    assert (want == bits).all()


def test_c4_adversarial_65536_every_category(eng):
    import config_legs as CL
    from narwhal_amd import _lib
    items, pos, cats, expect_bad = CL.adversarial_batch(eng)
    n = len(items)
    assert n == 65536 and len(pos) == 655
    assert len(set(cats)) == len(CL.INPLACE) + len(CL._golden_adversarial())
    pk, sg, arena, offs, lens = _lib.soa(items)
    want = _oracle_bits(pk, sg, arena, offs, lens)
    assert sorted(np.flatnonzero(~want).tolist()) == expect_bad
    # every category is present, and both verdicts occur among the adversarial entries
    acc = {bool(want[i]) for i in pos}
    assert acc == {True, False}
    ok, bits = _gpu_batch(eng, pk, sg, arena, offs, lens)
    assert not ok
    assert (bits == want).all()
    each = eng.verify_each_arrays(pk, sg, arena, offs, lens)
    assert (each == want).all()


@pytest.mark.parametrize("forge", ["equation", "decode", "none"])
def test_early_prep_equals_one_stream_order(eng, forge):
    """a host-staged 65,536 x 512 B batch takes msm_launch's early form (decompressions and the
    fallback's tables on the lane's second stream while the messages cross PCIe, the Straus pass
    gated on the MSM's verdict word).  Forged entries that all decode (message and s bit flips: the
    MSM rejects at its final sum, not at the prep's early reject); entries whose R or A does not
    decode or whose s >= l (the decode-failure and non-canonical-s flags that k_msm_scalars on the
    main stream and k_ed_points_msm on the aux stream set in the same flag words); and an all-valid
    batch: the bits equal the oracle's and those of an engine kept on the one-stream order
    (NWV_FLAG_NO_EARLY_PREP), call after call on the same buffers"""
    import narwhal_amd
    from narwhal_amd import _lib
    n = 65536
    pk, sg, msgs, offs, lens = _synth_arrays(eng, n, 512, seed=4242)
    forged = []
    if forge == "equation":
        rng = np.random.default_rng(7)
        forged = sorted(int(x) for x in rng.choice(n, size=48, replace=False))
        for j, i in enumerate(forged):
            if j % 2:
                msgs[512 * i + 17] ^= 0x04
            else:
                sg[64 * i + 40] ^= 0x01  # s bit flip (s stays < l: top byte untouched)
    elif forge == "decode":
        g = of.load_golden("ed25519_vectors.json")["vectors"]
        r_bad = [bytes.fromhex(v["sig"])[:32] for v in g if v["category"] == "B7_R_undecodable"]
        a_bad = [bytes.fromhex(v["pk"]) for v in g if v["category"] == "B7_A_undecodable"]
        L_ORDER = 2**252 + 27742317777372353535851937790883648493
        rng = np.random.default_rng(8)
        forged = sorted(int(x) for x in rng.choice(n, size=30, replace=False))
        for j, i in enumerate(forged):
            if j % 3 == 0:
                sg[64 * i:64 * i + 32] = np.frombuffer(r_bad[j % len(r_bad)], dtype=np.uint8)
            elif j % 3 == 1:
                pk[32 * i:32 * i + 32] = np.frombuffer(a_bad[j % len(a_bad)], dtype=np.uint8)
            else:
                v = int.from_bytes(sg[64 * i + 32:64 * i + 64].tobytes(), "little") + L_ORDER
                sg[64 * i + 32:64 * i + 64] = np.frombuffer(v.to_bytes(32, "little"), dtype=np.uint8)
    want = _oracle_bits(pk, sg, msgs, offs, lens)
    assert list(np.flatnonzero(~want)) == forged
    one = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_NO_EARLY_PREP)
    try:
        for _ in range(2):
            ok, bits = _gpu_batch(eng, pk, sg, msgs, offs, lens)
            assert ok == (not forged) and (bits == want).all()
            ok1, bits1 = _gpu_batch(one, pk, sg, msgs, offs, lens)
            assert ok1 == ok and (bits1 == bits).all()
    finally:
        one.close()
