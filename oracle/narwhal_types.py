"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the verification half of Narwhal's types crate,
the checker for narwhal_amd.types / include/nwv_types.h.  Never imported by the product.

Restates, check by check and in the reference's order:
  Header::digest      types/src/primary.rs:209-227   (BLAKE2b-256: author, round_le, epoch_le,
                                                       (digest, worker_le)*, parents*)
  Vote::digest        types/src/primary.rs:351-364   (id, round_le, epoch_le, origin)
  Certificate::digest types/src/primary.rs:594-607   (header id, round_le, epoch_le, origin)
  Header::verify      types/src/primary.rs:150-183
  Vote::verify        types/src/primary.rs:307-328
  Certificate::new_unsafe types/src/primary.rs:427-485
  Certificate::verify types/src/primary.rs:487-537  (genesis :392-405, PartialEq :615-623)
  Committee::quorum_threshold config/src/lib.rs:537-542, WorkerCache::worker :410-423
  CommitteeFixture header/votes/certificate  test_utils/src/lib.rs:719-780, 850-872
Signature checks call a supplied per-signature verifier (the Ed25519 oracle); the digests use
hashlib's BLAKE2b with digest_size = 32 (= fastcrypto::blake2b_256).
"""
import hashlib

OK, INVALID_EPOCH, INVALID_HEADER_ID, UNKNOWN_AUTHORITY = 0, 10, 11, 12
MALFORMED_HEADER, INVALID_SIGNATURE, REQUIRES_QUORUM = 13, 14, 15


def b2(data):
    return hashlib.blake2b(data, digest_size=32).digest()


def le64(x):
    return x.to_bytes(8, "little")


def header_digest(author, round_, epoch, payload, parents):
    pre = author + le64(round_) + le64(epoch)
    for d, w in payload:
        pre += d + w.to_bytes(4, "little")
    for p in sorted(set(parents)):
        pre += p
    return b2(pre)


def vote_digest(id_, round_, epoch, origin):
    return b2(id_ + le64(round_) + le64(epoch) + origin)


certificate_digest = vote_digest  # same preimage: header id, round, epoch, origin


class Committee:
    def __init__(self, keys, stakes, epoch=0, workers=None):
        order = sorted(range(len(keys)), key=lambda i: keys[i])
        self.keys = [keys[i] for i in order]
        self.stakes = [stakes[i] for i in order]
        self.epoch = epoch
        self.workers = [list(workers[i]) for i in order] if workers else [[] for _ in keys]

    def stake(self, pk):
        return self.stakes[self.keys.index(pk)] if pk in self.keys else 0

    def quorum_threshold(self):
        return 2 * sum(self.stakes) // 3 + 1

    def worker_known(self, pk, wid):
        return pk in self.keys and wid in self.workers[self.keys.index(pk)]


def header_verify(c, h, verify):
    """h: dict(author, round, epoch, payload, parents, id, signature) -> DagError code"""
    if h["epoch"] != c.epoch:
        return INVALID_EPOCH
    if header_digest(h["author"], h["round"], h["epoch"], h["payload"], h["parents"]) != h["id"]:
        return INVALID_HEADER_ID
    if c.stake(h["author"]) <= 0:
        return UNKNOWN_AUTHORITY
    for _, w in h["payload"]:
        if not c.worker_known(h["author"], w):
            return MALFORMED_HEADER
    return OK if verify(h["author"], h["signature"], h["id"]) else INVALID_SIGNATURE


def vote_verify(c, v, verify):
    if v["epoch"] != c.epoch:
        return INVALID_EPOCH
    if c.stake(v["author"]) <= 0:
        return UNKNOWN_AUTHORITY
    d = vote_digest(v["id"], v["round"], v["epoch"], v["origin"])
    return OK if verify(v["author"], v["signature"], d) else INVALID_SIGNATURE


def is_genesis(c, cert):
    h = cert["header"]
    return h["id"] == bytes(32) and h["round"] == 0 and h["epoch"] == c.epoch and h["author"] in c.keys


def certificate_verify(c, cert, verify):
    h = cert["header"]
    if h["epoch"] != c.epoch:
        return INVALID_EPOCH
    if is_genesis(c, cert):
        return OK
    r = header_verify(c, h, verify)
    if r:
        return r
    weight, it, pks = 0, 0, []
    idx = cert["signed"]
    for a, pk in enumerate(c.keys):
        if it < len(idx) and idx[it] == a:
            weight += c.stakes[a]
            it += 1
            pks.append(pk)
    if weight < c.quorum_threshold():
        return REQUIRES_QUORUM
    sigs = cert["sigs"]
    if len(pks) != len(sigs):
        return INVALID_SIGNATURE
    d = certificate_digest(h["id"], h["round"], h["epoch"], h["author"])
    return OK if all(verify(pk, s, d) for pk, s in zip(pks, sigs)) else INVALID_SIGNATURE


def certificate_verify_bls(c, cert, verify, agg_verify):
    """Certificate::verify under BLS12-381 (crypto/src/lib.rs:29-33): cert["agg"] is ONE aggregate
    (48 bytes) or None (AggregateSignature::default(): sig None -> signature::Error); the check is
    agg_verify(pks, agg, digest) = fast_aggregate_verify, with no |pks| = |sigs| test"""
    h = cert["header"]
    if h["epoch"] != c.epoch:
        return INVALID_EPOCH
    if is_genesis(c, cert):
        return OK
    r = header_verify(c, h, verify)
    if r:
        return r
    weight, it, pks = 0, 0, []
    idx = cert["signed"]
    for a, pk in enumerate(c.keys):
        if it < len(idx) and idx[it] == a:
            weight += c.stakes[a]
            it += 1
            pks.append(pk)
    if weight < c.quorum_threshold():
        return REQUIRES_QUORUM
    if cert["agg"] is None:
        return INVALID_SIGNATURE
    d = certificate_digest(h["id"], h["round"], h["epoch"], h["author"])
    return OK if agg_verify(pks, cert["agg"], d) else INVALID_SIGNATURE


def certificate_new(c, votes, check_stake=True):
    """-> (code, signed indices, aggregated signature list)"""
    votes = sorted(votes, key=lambda v: v[0])  # stable, by pk
    front, weight, signed, taken = 0, 0, [], []
    for k, pk in enumerate(c.keys):
        if front < len(votes) and votes[front][0] == pk:
            taken.append(votes[front])
            front += 1
            weight += c.stakes[k]
            while front < len(votes) and votes[front] == taken[-1]:
                front += 1
            signed.append(k)
    if front < len(votes):
        return UNKNOWN_AUTHORITY, None, None
    if check_stake and weight < c.quorum_threshold():
        return REQUIRES_QUORUM, None, None
    return OK, signed, [s for _, s in taken]


class CommitteeFixture:
    """test_utils::CommitteeFixture: seeded Ed25519 authorities (stake 1, workers 0..3, epoch 0).
    `authorities` keeps generation order; the committee orders them by key bytes."""

    def __init__(self, size, pubkey, sign, seed=0, epoch=0, workers=4):
        self.seeds = [hashlib.sha256(b"nwv-fixture" + seed.to_bytes(4, "little") + i.to_bytes(4, "little")).digest()
                      for i in range(size)]
        self.pubkey, self.sign = pubkey, sign
        self.authorities = [pubkey(s) for s in self.seeds]
        self.committee = Committee(self.authorities, [1] * size, epoch, [list(range(workers))] * size)

    def header(self, author_idx=-1, round_=1, parents=None, payload=()):
        """AuthorityFixture::header: round 1, parents = genesis digests, empty payload"""
        c = self.committee
        seed = self.seeds[author_idx]
        pk = self.authorities[author_idx]
        if parents is None:
            parents = [certificate_digest(bytes(32), 0, c.epoch, k) for k in c.keys]
        hid = header_digest(pk, round_, c.epoch, list(payload), parents)
        return {"author": pk, "round": round_, "epoch": c.epoch, "payload": list(payload),
                "parents": sorted(set(parents)), "id": hid, "signature": self.sign(seed, hid)}

    def vote(self, idx, h):
        d = vote_digest(h["id"], h["round"], h["epoch"], h["author"])
        return {"id": h["id"], "round": h["round"], "epoch": h["epoch"], "origin": h["author"],
                "author": self.authorities[idx], "signature": self.sign(self.seeds[idx], d)}

    def votes(self, h):
        return [self.vote(i, h) for i, pk in enumerate(self.authorities) if pk != h["author"]]
