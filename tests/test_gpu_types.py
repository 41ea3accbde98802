"""GPU parity of the types layer (include/nwv_types.h): Header / Vote / Certificate digests and
verify results equal the oracle restatement (oracle/narwhal_types.py) check by check, the
reference's certificate tests (primary/src/tests/certificate_tests.rs:12-144) pass, and
validate_certificates pinpoints exactly the invalid certificates of a 100-node committee round
(BASELINE.json configs[4] shape)."""
import random

import pytest

import oracle_ffi as of
import types_util as tu
from types_util import nt

from narwhal_amd import types as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    yield e
    e.close()


def _ver(pk, sig, msg):
    return of.verify(pk, sig, msg)


def test_digests_match_oracle(eng):
    rnd = random.Random(1)
    hs, vs = [], []
    for _ in range(50):
        h = T.Header(rnd.randbytes(32), rnd.getrandbits(64), rnd.getrandbits(64),
                     [(rnd.randbytes(32), rnd.getrandbits(32)) for _ in range(rnd.randint(0, 5))],
                     [rnd.randbytes(32) for _ in range(rnd.randint(0, 110))], rnd.randbytes(32))
        hs.append(h)
        vs.append(T.Vote(h.id, h.round, h.epoch, h.author, rnd.randbytes(32)))
    got = T.header_digests(eng, hs)
    assert got == [nt.header_digest(h.author, h.round, h.epoch, h.payload, h.parents) for h in hs]
    assert T.vote_digests(eng, vs) == [nt.vote_digest(v.id, v.round, v.epoch, v.origin) for v in vs]
    certs = [T.Certificate(h) for h in hs]
    assert T.certificate_digests(eng, certs) == [nt.certificate_digest(h.id, h.round, h.epoch, h.author) for h in hs]


def test_reference_certificate_tests(eng):
    fx = nt.CommitteeFixture(4, of.pubkey, of.sign)
    c = tu.committee(fx.committee)
    h = fx.header()
    th = tu.header(h)
    votes = [(v["author"], v["signature"]) for v in fx.votes(h)]
    # test_empty_certificate_verification
    with pytest.raises(T.CertificateRequiresQuorum):
        T.verify(eng, c, T.Certificate.new_unsigned(c, th, []))
    # test_valid_certificate_verification
    T.verify(eng, c, T.Certificate.new(c, th, votes))
    # test_certificate_insufficient_signatures
    with pytest.raises(T.CertificateRequiresQuorum):
        T.verify(eng, c, T.Certificate.new_unsigned(c, th, votes[:2]))
    # test_certificate_validly_repeated_public_keys
    T.verify(eng, c, T.Certificate.new(c, th, [v for v in votes for _ in range(2)]))


@pytest.mark.parametrize("size", [4, 5, 7, 10, 16, 22, 34])
def test_certificate_verification_sizes(eng, size):
    """proptest test_certificate_verification(committee_size in 4..35): a quorum of votes verifies"""
    fx = nt.CommitteeFixture(size, of.pubkey, of.sign, seed=size)
    c = tu.committee(fx.committee)
    h = fx.header()
    q = fx.committee.quorum_threshold()
    votes = [(fx.authorities[i], fx.vote(i, h)["signature"]) for i in range(q)]
    T.verify(eng, c, T.Certificate.new(c, tu.header(h), votes))


def _mutations(fx, rnd):
    """(header dict, certificate dict) pairs covering every DagError path, plus valid ones"""
    c = fx.committee
    out = []
    for k in range(24):
        a = rnd.randrange(len(fx.authorities))
        h = fx.header(author_idx=a, round_=rnd.randint(1, 9),
                      payload=[(rnd.randbytes(32), rnd.randint(0, 3)) for _ in range(rnd.randint(0, 3))])
        signers = [i for i in range(len(fx.authorities)) if i != a]
        rnd.shuffle(signers)
        cert = tu.oracle_certificate(fx, h, signers[:c.quorum_threshold()])
        kind = k % 12
        h2 = dict(h)
        if kind == 1:
            h2["epoch"] = c.epoch + 1
        elif kind == 2:
            h2["id"] = bytes([h["id"][0] ^ 1]) + h["id"][1:]
        elif kind == 3:
            h2["payload"] = h["payload"] + [(bytes(32), 9)]  # unknown worker id
            h2["id"] = nt.header_digest(h2["author"], h2["round"], h2["epoch"], h2["payload"], h2["parents"])
            h2["signature"] = fx.sign(fx.seeds[a], h2["id"])
        elif kind == 4:
            h2["signature"] = bytes([h["signature"][0] ^ 4]) + h["signature"][1:]
        elif kind == 5:
            cert = dict(cert, sigs=[cert["sigs"][0][:-1] + bytes([cert["sigs"][0][-1] ^ 1])] + cert["sigs"][1:])
        elif kind == 6:
            cert = dict(cert, signed=cert["signed"][:-1], sigs=cert["sigs"][:-1])  # below quorum
        elif kind == 7:
            cert = dict(cert, sigs=cert["sigs"][:-1])  # |pks| != |sigs|
        elif kind == 8:
            cert = dict(cert, signed=cert["signed"] + [len(c.keys) + 3])  # out-of-range index ignored
        elif kind == 9:  # bad header signature AND no quorum: Header::verify's error wins
            h2["signature"] = bytes(64)
            cert = dict(cert, signed=cert["signed"][:1], sigs=cert["sigs"][:1])
        elif kind == 10:  # genesis certificate
            out.append((None, {"header": {"author": c.keys[k % len(c.keys)], "round": 0, "epoch": c.epoch,
                                          "payload": [], "parents": [], "id": bytes(32),
                                          "signature": bytes(64)}, "signed": [], "sigs": []}))
            continue
        elif kind == 11:  # unknown author
            h2["author"] = of.pubkey(b"\x42" * 32)
            h2["id"] = nt.header_digest(h2["author"], h2["round"], h2["epoch"], h2["payload"], h2["parents"])
            h2["signature"] = of.sign(b"\x42" * 32, h2["id"])
        out.append((h2, dict(cert, header=h2)))
    return out


def test_header_vote_certificate_codes_match_oracle(eng):
    rnd = random.Random(7)
    fx = nt.CommitteeFixture(10, of.pubkey, of.sign, seed=3)
    c = tu.committee(fx.committee)
    cases = _mutations(fx, rnd)
    heads = [h for h, _ in cases if h is not None]
    got = T.verify_headers(eng, c, [tu.header(h) for h in heads])
    assert got == [nt.header_verify(fx.committee, h, _ver) for h in heads]
    certs = [cert for _, cert in cases]
    got = T.verify_certificates(eng, c, [tu.certificate(x) for x in certs])
    want = [nt.certificate_verify(fx.committee, x, _ver) for x in certs]
    assert got == want
    assert set(want) >= {0, 10, 11, 12, 13, 14, 15}
    # votes: valid, wrong epoch, unknown author, bad signature
    h = fx.header()
    vs = fx.votes(h)
    vs[1] = dict(vs[1], epoch=5)
    vs[2] = dict(vs[2], author=of.pubkey(b"\x01" * 32))
    vs[3] = dict(vs[3], signature=bytes(64))
    got = T.verify_votes(eng, c, [tu.vote(v) for v in vs])
    assert got == [nt.vote_verify(fx.committee, v, _ver) for v in vs]
    assert got[:4] == [0, 10, 12, 14]


def test_validate_certificates_dag_round_100(eng):
    """configs[4] shape: a 100-node committee round, one certificate per authority, each with the
    header signature + 67 votes; a few corrupted -> exactly those are reported invalid."""
    rnd = random.Random(100)
    fx = nt.CommitteeFixture(100, of.pubkey, of.sign, seed=100)
    c = tu.committee(fx.committee)
    q = fx.committee.quorum_threshold()
    assert q == 67
    parents = [rnd.randbytes(32) for _ in range(q)]
    certs = []
    for a in range(100):
        h = fx.header(author_idx=a, parents=parents, payload=[(rnd.randbytes(32), a % 4)])
        signers = [i for i in range(100) if i != a][:q]
        certs.append(tu.oracle_certificate(fx, h, signers))
    bad = {3: "vote", 41: "header", 77: "vote"}
    for i, what in bad.items():
        x = certs[i]
        if what == "vote":
            s = x["sigs"][5]
            certs[i] = dict(x, sigs=x["sigs"][:5] + [s[:10] + bytes([s[10] ^ 8]) + s[11:]] + x["sigs"][6:])
        else:
            hh = dict(x["header"], signature=bytes(64))
            certs[i] = dict(x, header=hh)
    ok, idx = T.validate_certificates(eng, c, [tu.certificate(x) for x in certs])
    assert not ok and idx == sorted(bad)
    good = [x for i, x in enumerate(certs) if i not in bad]
    ok, idx = T.validate_certificates(eng, c, [tu.certificate(x) for x in good])
    assert ok and idx == []
    assert T.validate_certificates(eng, c, []) == (True, [])


def test_verify_mixed_matches_oracle(eng):
    """nwv_verify_mixed_many: headers, votes and certificates of every DagError kind in ONE call
    (one digest launch, one batch MSM) give the codes the reference's per-item verify returns,
    and the same codes as the per-kind *_many calls; empty kinds are allowed."""
    rnd = random.Random(11)
    fx = nt.CommitteeFixture(10, of.pubkey, of.sign, seed=5)
    c = tu.committee(fx.committee)
    cases = _mutations(fx, rnd)
    heads = [h for h, _ in cases if h is not None]
    certs = [cert for _, cert in cases]
    h = fx.header()
    vs = fx.votes(h)
    vs[1] = dict(vs[1], epoch=5)
    vs[2] = dict(vs[2], author=of.pubkey(b"\x02" * 32))
    vs[3] = dict(vs[3], signature=bytes(64))
    H = [tu.header(x) for x in heads]
    V = [tu.vote(v) for v in vs]
    C = [tu.certificate(x) for x in certs]
    gh, gv, gc = T.verify_mixed(eng, c, H, V, C)
    assert gh == [nt.header_verify(fx.committee, x, _ver) for x in heads]
    assert gv == [nt.vote_verify(fx.committee, v, _ver) for v in vs]
    assert gc == [nt.certificate_verify(fx.committee, x, _ver) for x in certs]
    assert gh == T.verify_headers(eng, c, H) and gv == T.verify_votes(eng, c, V)
    assert gc == T.verify_certificates(eng, c, C)
    # all-valid mix (the MSM accepts without fallback), and empty kinds
    good_h = [x for x, code in zip(H, gh) if code == 0]
    good_c = [x for x, code in zip(C, gc) if code == 0]
    good_v = [x for x, code in zip(V, gv) if code == 0]
    assert good_h and good_c and good_v
    assert T.verify_mixed(eng, c, good_h, good_v, good_c) == ([0] * len(good_h), [0] * len(good_v),
                                                               [0] * len(good_c))
    assert T.verify_mixed(eng, c, votes=good_v) == ([], [0] * len(good_v), [])
    assert T.verify_mixed(eng, c) == ([], [], [])


def test_verify_mixed_concurrent_threads(eng):
    """nwv_verify_mixed_many from 6 host threads on one context (per-thread batch buffers, the
    device lock around each engine call): every thread gets the codes of the serial call"""
    from concurrent.futures import ThreadPoolExecutor
    rnd = random.Random(21)
    fx = nt.CommitteeFixture(10, of.pubkey, of.sign, seed=9)
    c = tu.committee(fx.committee)
    cases = _mutations(fx, rnd)
    H = [tu.header(h) for h, _ in cases if h is not None]
    C = [tu.certificate(x) for _, x in cases]
    h = fx.header()
    vs = fx.votes(h)
    vs[2] = dict(vs[2], signature=bytes(64))
    V = [tu.vote(v) for v in vs]
    want = T.verify_mixed(eng, c, H, V, C)

    def run(k):
        # thread k verifies a rotation of the item lists, so the batches differ between threads
        r = k % max(1, len(C))
        got = T.verify_mixed(eng, c, H, V, C[r:] + C[:r])
        return got == (want[0], want[1], want[2][r:] + want[2][:r])

    with ThreadPoolExecutor(6) as ex:
        assert all(ex.map(run, range(24)))
