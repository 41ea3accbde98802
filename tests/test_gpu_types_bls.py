"""The types layer under BLS12-381, the reference's default scheme (crypto/src/lib.rs:29-33),
through the C ABI (include/nwv_types.h nwv_bls_*): a 100-node DAG round -- 100 headers, 99 votes,
100 certificates of 67 signers -- plus every DagError path (forged aggregate, wrong digest, below
quorum, unknown signer index, an aggregate holding no signature, undecodable aggregate, wrong
epoch, bad header id / signature / author / worker id, genesis), verified in ONE
nwv_bls_verify_mixed_many call and item by item against oracle/narwhal_types.py with the BLS
oracle (oracle/bls_oracle.c) deciding every signature check.  Also the Core drain in BLS mode."""
import random

import pytest

import bls_ffi as B
from types_util import nt as NT  # oracle/narwhal_types.py (the checker)

pytestmark = pytest.mark.gpu
r_order = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


@pytest.fixture(scope="module")
def env():
    import narwhal_amd
    from narwhal_amd import types as T
    from narwhal_amd.bls import Bls
    eng = narwhal_amd.Engine(device=0)
    bls = Bls(eng)
    rnd = random.Random(41)
    n = 100
    sks = [rnd.randrange(1, r_order).to_bytes(32, "big") for _ in range(n)]
    pks = bls.keygen(sks)
    sk_of = dict(zip(pks, sks))
    com = T.Committee(list(pks), [1] * n, 0, [[0, 1, 2, 3]] * n)
    q = com.quorum_threshold()
    parents = T.bls_certificate_digests(eng, T.BlsCertificate.genesis(com))
    headers = [T.Header(author=k, round=1, epoch=0, payload=[(rnd.randbytes(32), a % 4)], parents=list(parents),
                        signature=bytes(48)) for a, k in enumerate(com.keys)]
    for h, d in zip(headers, T.bls_header_digests(eng, headers)):
        h.id = d
    for h, s in zip(headers, bls.sign([sk_of[h.author] for h in headers], [h.id for h in headers])):
        h.signature = s
    voters = [[i for i in range(n) if i != a][:q] for a in range(n)]
    votes = [T.Vote(headers[a].id, 1, 0, com.keys[a], com.keys[v], bytes(48)) for a in range(n) for v in voters[a]]
    for v, s in zip(votes, bls.sign([sk_of[v.author] for v in votes], T.bls_vote_digests(eng, votes))):
        v.signature = s
    certs = [T.BlsCertificate.new(eng, com, headers[a], [(v.author, v.signature) for v in votes[a * q:(a + 1) * q]])
             for a in range(n)]
    yield dict(eng=eng, bls=bls, T=T, com=com, sk_of=sk_of, headers=headers, votes=votes, certs=certs, rnd=rnd, q=q)
    eng.close()


def _oracle_codes(env, headers, votes, certs):
    """oracle/narwhal_types.py's control flow; every signature check it needs decided by the BLS
    oracle (collected in a first pass, computed in one multi-threaded call, then looked up)"""
    com = env["com"]
    oc = NT.Committee(list(com.keys), list(com.stakes), com.epoch, [list(w) for w in com.workers])
    want = {}

    def hd(h):
        return {"author": h.author, "round": h.round, "epoch": h.epoch, "payload": list(h.payload),
                "parents": list(h.parents), "id": h.id, "signature": h.signature}

    def run(ver, agg):
        hc = [NT.header_verify(oc, hd(h), ver) for h in headers]
        vc = [NT.vote_verify(oc, {"id": v.id, "round": v.round, "epoch": v.epoch, "origin": v.origin,
                                  "author": v.author, "signature": v.signature}, ver) for v in votes]
        cc = [NT.certificate_verify_bls(oc, {"header": hd(c.header), "signed": list(c.signed_authorities),
                                             "agg": c.aggregated_signature}, ver, agg) for c in certs]
        return hc, vc, cc

    run(lambda pk, s, m: want.setdefault(((pk,), s, m), None) is None,
        lambda pks, s, m: want.setdefault((tuple(pks), s, m), None) is None)
    keys = list(com.keys)
    extra = sorted({pk for ks, _, _ in want for pk in ks if pk not in keys})
    keys += extra
    kidx = {k: i for i, k in enumerate(keys)}
    checks = list(want)
    st = B.verify_items(keys, [s for _, s, _ in checks], [[kidx[k] for k in ks] for ks, _, _ in checks],
                        [m for _, _, m in checks])
    res = dict(zip(checks, st))
    return run(lambda pk, s, m: res[((pk,), s, m)] == 0, lambda pks, s, m: res[(tuple(pks), s, m)] == 0)


def _adversarial(env):
    T, com, bls, rnd, q = env["T"], env["com"], env["bls"], env["rnd"], env["q"]
    H, V, C = env["headers"], env["votes"], env["certs"]
    import copy
    certs = list(C)
    forged = copy.deepcopy(C[0])
    forged.aggregated_signature = C[1].aggregated_signature          # another certificate's aggregate
    wrong_digest = copy.deepcopy(C[2])
    wrong_digest.header.id = bytes([C[2].header.id[0] ^ 1]) + C[2].header.id[1:]  # InvalidHeaderId
    below = copy.deepcopy(C[3])
    below.signed_authorities = below.signed_authorities[:q - 1]       # CertificateRequiresQuorum
    unknown_idx = copy.deepcopy(C[4])
    unknown_idx.signed_authorities = unknown_idx.signed_authorities[:q - 1] + [150]  # filtered out: below quorum
    missing_one = copy.deepcopy(C[5])
    missing_one.signed_authorities = [i for i in range(100) if i != C[5].signed_authorities[0]][:q]  # other signers
    none_agg = copy.deepcopy(C[6])
    none_agg.aggregated_signature = None
    garbage = copy.deepcopy(C[7])
    garbage.aggregated_signature = bytes([0x9f]) + bytes(47)
    wrong_epoch = copy.deepcopy(C[8])
    wrong_epoch.header.epoch = 1
    bad_hsig = copy.deepcopy(C[9])
    bad_hsig.header.signature = H[10].signature
    genesis = T.BlsCertificate.genesis(com)[3]
    certs += [forged, wrong_digest, below, unknown_idx, missing_one, none_agg, garbage, wrong_epoch, bad_hsig, genesis]
    headers = list(H)
    h_badsig = copy.deepcopy(H[0])
    h_badsig.signature = H[1].signature
    h_unknown = copy.deepcopy(H[2])
    h_unknown.author = env["bls"].keygen([(7).to_bytes(32, "big")])[0]
    h_unknown.id = T.bls_header_digests(env["eng"], [h_unknown])[0]
    h_worker = copy.deepcopy(H[3])
    h_worker.payload = [(H[3].payload[0][0], 9)]
    h_worker.id = T.bls_header_digests(env["eng"], [h_worker])[0]
    h_epoch = copy.deepcopy(H[4])
    h_epoch.epoch = 3
    h_badid = copy.deepcopy(H[5])
    h_badid.round = 2
    headers += [h_badsig, h_unknown, h_worker, h_epoch, h_badid]
    votes = list(V[:99])
    v_bad = copy.deepcopy(V[0])
    v_bad.signature = V[1].signature
    v_epoch = copy.deepcopy(V[2])
    v_epoch.epoch = 5
    v_unknown = copy.deepcopy(V[3])
    v_unknown.author = h_unknown.author
    v_garbage = copy.deepcopy(V[4])
    v_garbage.signature = bytes(48)
    votes += [v_bad, v_epoch, v_unknown, v_garbage]
    return headers, votes, certs


def test_bls_round_valid(env):
    """the honest 100-node round in one call: every code Ok, as the oracle's"""
    T = env["T"]
    hc, vc, cc = T.bls_verify_mixed(env["eng"], env["com"], env["headers"], env["votes"][:99], env["certs"])
    assert hc == [0] * 100 and vc == [0] * 99 and cc == [0] * 100
    ok, bad = T.bls_validate_certificates(env["eng"], env["com"], env["certs"])
    assert ok and bad == []


def test_bls_round_adversarial_matches_oracle(env):
    T = env["T"]
    headers, votes, certs = _adversarial(env)
    got = T.bls_verify_mixed(env["eng"], env["com"], headers, votes, certs)
    want = _oracle_codes(env, headers, votes, certs)
    assert got == want
    hc, vc, cc = got
    assert hc[:100] == [0] * 100 and hc[100:] == [NT.INVALID_SIGNATURE, NT.UNKNOWN_AUTHORITY, NT.MALFORMED_HEADER,
                                                   NT.INVALID_EPOCH, NT.INVALID_HEADER_ID]
    assert vc[99:] == [NT.INVALID_SIGNATURE, NT.INVALID_EPOCH, NT.UNKNOWN_AUTHORITY, NT.INVALID_SIGNATURE]
    assert cc[:100] == [0] * 100
    assert cc[100:] == [NT.INVALID_SIGNATURE, NT.INVALID_HEADER_ID, NT.REQUIRES_QUORUM, NT.REQUIRES_QUORUM,
                        NT.INVALID_SIGNATURE, NT.INVALID_SIGNATURE, NT.INVALID_SIGNATURE, NT.INVALID_EPOCH,
                        NT.INVALID_SIGNATURE, NT.OK]
    ok, bad = T.bls_validate_certificates(env["eng"], env["com"], certs)
    assert not ok and bad == [i for i, c in enumerate(cc) if c]


def test_bls_certificate_new_contract(env):
    """Certificate::new under BLS: unknown voter, below quorum, repeats dropped, aggregate = the
    oracle's sum of the kept signatures"""
    T, com, V, q = env["T"], env["com"], env["votes"], env["q"]
    h = env["headers"][0]
    vs = [(v.author, v.signature) for v in V[:q]]
    c = T.BlsCertificate.new(env["eng"], com, h, vs + vs[:3])  # repeats dropped
    assert c.aggregated_signature == B.aggregate([s for _, s in sorted(vs)])[1]
    assert c.signed_authorities == sorted(com.keys.index(p) for p, _ in vs)
    with pytest.raises(T.CertificateRequiresQuorum):
        T.BlsCertificate.new(env["eng"], com, h, vs[:q - 1])
    stranger = env["bls"].keygen([(9).to_bytes(32, "big")])[0]
    with pytest.raises(T.UnknownAuthority):
        T.BlsCertificate.new(env["eng"], com, h, vs + [(stranger, vs[0][1])])
    c0 = T.BlsCertificate.new(env["eng"], com, h, [], check_stake=False)
    assert c0.aggregated_signature is None and c0.signed_authorities == []
    with pytest.raises(T.InvalidSignature):
        T.BlsCertificate.new(env["eng"], com, h, [(vs[0][0], bytes(48))], check_stake=False)


def test_bls_core_drain(env):
    """the Core drain in BLS mode: one engine call per drained batch, codes per message in arrival
    order, equal to the oracle's"""
    import queue
    from narwhal_amd.service import CoreDrain
    headers, votes, certs = _adversarial(env)
    want_h, want_v, want_c = _oracle_codes(env, headers, votes, certs)
    msgs = [("header", h) for h in headers] + [("vote", v) for v in votes] + [("certificate", c) for c in certs]
    want = list(want_h) + list(want_v) + list(want_c)
    order = list(range(len(msgs)))
    env["rnd"].shuffle(order)
    q = queue.Queue()
    for i in order:
        q.put((i, msgs[i]))
    d = CoreDrain(env["eng"], env["com"], max_items=512, max_wait_us=100, min_items=1, scheme="bls")
    got = {}
    while len(got) < len(msgs):
        batch = d.drain(q)
        for (i, _), code in zip(batch, d.verify([m for _, m in batch])):
            got[i] = code
    assert [got[i] for i in range(len(msgs))] == want
    assert d.calls >= 1 and d.largest <= 512


def test_bls_service_concurrent_submitters(env):
    """the in-library batching service in BLS mode (nwv_service_create_bls): 8 threads submit the
    adversarial round's headers, votes and certificates with the blocking calls; each gets the
    oracle's code for its own message, and the service coalesced them into few engine calls"""
    import threading
    from narwhal_amd.service import Service
    headers, votes, certs = _adversarial(env)
    want_h, want_v, want_c = _oracle_codes(env, headers, votes, certs)
    msgs = [(h, w) for h, w in zip(headers, want_h)] + [(v, w) for v, w in zip(votes, want_v)] + \
           [(c, w) for c, w in zip(certs, want_c)]
    got = [None] * len(msgs)
    with Service(env["eng"], env["com"], max_batch=64, max_wait_us=2000, scheme="bls") as svc:
        def worker(lo):
            for k in range(lo, len(msgs), 8):
                m = msgs[k][0]
                got[k] = (svc.verify_certificate(m) if isinstance(m, env["T"].BlsCertificate) else
                          svc.verify_vote(m) if isinstance(m, env["T"].Vote) else svc.verify_header(m))

        th = [threading.Thread(target=worker, args=(lo,)) for lo in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        st = svc.stats()
    assert got == [w for _, w in msgs]
    assert st["items"] == len(msgs) and st["calls"] < len(msgs)
