#!/usr/bin/env python3
"""Golden-fixture generator -- TEST INFRASTRUCTURE ONLY, run in the build container.

A small pure-Python (big-integer) restatement of the reference's Ed25519 verdict semantics,
used to produce the committed fixtures under tests/golden/.  The reference path is Rust in
crates that are not vendored: ed25519-consensus 2.0.1 over
curve25519-dalek-ng 4.1.1 and sha2 0.9.9, wrapped by fastcrypto 0.1.2
(/root/reference/Cargo.lock:1428,1166,3845,1534).  Nothing of the reference is imported or run;
this restates the published ZIP-215 contract written out in SURVEY.md Appendix A:

  decode(P):  y = LE(P) mod 2^255 (values >= p accepted), x = sqrt_ratio_i(y^2-1, d y^2+1)
              (non-square -> reject), negate on sign bit, "negative zero" accepted;
  verify:     A decodes, s < l, R decodes, k = SHA-512(R_bytes||A_bytes||M) mod l,
              accept iff [8]([s]B - [k]A - R) == identity.

Independent pins applied before anything is written (the script aborts on any mismatch):
  * libsodium 1.0.18 (/opt/conda/lib/libsodium.so.23): seed->pk, deterministic signatures,
    crypto_core_ed25519_scalar_reduce, and crypto_sign_verify_detached on every canonical,
    torsion-free vector (strict cofactorless verification must agree there);
  * node / OpenSSL 1.1.1 crypto.verify on the same subset;
  * hashlib sha512 / blake2b(digest_size=32) for the hash vectors;
  * the reference's own Ed25519 key fixtures Docker/validators/validator-*/network-key.json
    (seed -> public key), copied here as data.
Run:  python3 oracle/gen_golden.py   (writes tests/golden/*.json; deterministic, seed 2025)
"""
import base64
import ctypes
import hashlib
import json
import os
import random
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")

p = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
d = (-121665 * pow(121666, p - 2, p)) % p
SQRTM1 = pow(2, (p - 1) // 4, p)
D2 = 2 * d % p


def inv(x):
    return pow(x, p - 2, p)


# ---------------------------------------------------------------- field / decoding
def is_negative(x):
    return (x % p) & 1


def sqrt_ratio_i(u, v):
    """FieldElement::sqrt_ratio_i (dalek): (was_nonzero_square, nonnegative r)."""
    u %= p
    v %= p
    v3 = v * v * v % p
    v7 = v3 * v3 * v % p
    r = (u * v3) * pow(u * v7 % p, (p - 5) // 8, p) % p
    check = v * r * r % p
    correct = check == u
    flipped = check == (-u) % p
    flipped_i = check == (-u * SQRTM1) % p
    if flipped or flipped_i:
        r = r * SQRTM1 % p
    if is_negative(r):
        r = (-r) % p
    return (correct or flipped), r


def decompress(b):
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    sign = b[31] >> 7
    yy = y * y % p
    ok, x = sqrt_ratio_i(yy - 1, d * yy + 1)
    if not ok:
        return None
    if sign:
        x = (-x) % p
    y %= p
    return (x, y, 1, x * y % p)


def compress(P):
    X, Y, Z, _ = P
    zi = inv(Z)
    x, y = X * zi % p, Y * zi % p
    return (y | (is_negative(x) << 255)).to_bytes(32, "little")


IDENT = (0, 1, 1, 0)


def padd(P, Q):
    X1, Y1, Z1, T1 = P
    X2, Y2, Z2, T2 = Q
    A = (Y1 - X1) * (Y2 - X2) % p
    B = (Y1 + X1) * (Y2 + X2) % p
    C = T1 * D2 * T2 % p
    Dd = Z1 * 2 * Z2 % p
    E, F, G, H = B - A, Dd - C, Dd + C, B + A
    return (E * F % p, G * H % p, F * G % p, E * H % p)


def pneg(P):
    X, Y, Z, T = P
    return ((-X) % p, Y, Z, (-T) % p)


def pmul(n, P):
    Q = IDENT
    for bit in bin(n)[2:] if n > 0 else "":
        Q = padd(Q, Q)
        if bit == "1":
            Q = padd(Q, P)
    return Q


def is_identity(P):
    X, Y, Z, _ = P
    return X % p == 0 and (Y - Z) % p == 0


BY = 4 * inv(5) % p
B = decompress(BY.to_bytes(32, "little"))
assert compress(B).hex() == "58" + "66" * 31


def H(*parts):
    h = hashlib.sha512()
    for x in parts:
        h.update(x)
    return int.from_bytes(h.digest(), "little")


def verify(pk, sig, msg):
    """ed25519_consensus::VerificationKey::verify semantics."""
    A = decompress(pk)
    if A is None:
        return False
    s = int.from_bytes(sig[32:], "little")
    if s >= L:
        return False
    R = decompress(sig[:32])
    if R is None:
        return False
    k = H(sig[:32], pk, msg) % L
    chk = padd(padd(pmul(s, B), pneg(pmul(k, A))), pneg(R))
    return is_identity(pmul(8, chk))


def expand(seed):
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def pubkey(seed):
    a, _ = expand(seed)
    return compress(pmul(a, B))


def sign(seed, msg):
    a, prefix = expand(seed)
    pk = compress(pmul(a, B))
    r = H(prefix, msg) % L
    Rb = compress(pmul(r, B))
    k = H(Rb, pk, msg) % L
    return Rb + ((r + k * a) % L).to_bytes(32, "little")


# ---------------------------------------------------------------- torsion points
def torsion_points():
    """All 8 points of E[8] (affine x, y)."""
    # find a point of order 8: x^2 solutions with y s.t. 8P = 0, 4P != 0
    pts = set()
    # order-8 points satisfy ... brute force via the known construction: take any point Q,
    # multiply by l to kill the prime-order part; repeat until order 8 found.
    rnd = random.Random(7)
    T8 = None
    while T8 is None:
        yb = rnd.getrandbits(255).to_bytes(32, "little")
        Q = decompress(yb)
        if Q is None:
            continue
        T = pmul(L, Q)
        if not is_identity(pmul(4, T)):
            T8 = T
    acc = IDENT
    for _ in range(8):
        zi = inv(acc[2])
        pts.add((acc[0] * zi % p, acc[1] * zi % p))
        acc = padd(acc, T8)
    assert len(pts) == 8
    return sorted(pts), T8


def encodings_of(x, y):
    """Every 32-byte string that decodes to (x, y) under the ZIP-215 rules."""
    encs = []
    for yy in (y, y + p):
        if yy >= 2**255:
            continue
        for sign in (0, 1):
            b = (yy | (sign << 255)).to_bytes(32, "little")
            P = decompress(b)
            if P is None:
                continue
            if (P[0] % p, P[1] % p) == (x, y):
                encs.append(b)
    return encs


# ---------------------------------------------------------------- independent checkers
def load_sodium():
    for path in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
        try:
            lib = ctypes.CDLL(path)
            if lib.sodium_init() < 0:
                continue
            return lib
        except OSError:
            continue
    return None


SODIUM = load_sodium()


def sodium_seed_keypair(seed):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    assert SODIUM.crypto_sign_seed_keypair(pk, sk, seed) == 0
    return pk.raw, sk.raw


def sodium_sign(seed, msg):
    _, sk = sodium_seed_keypair(seed)
    sig = ctypes.create_string_buffer(64)
    siglen = ctypes.c_ulonglong(0)
    assert SODIUM.crypto_sign_detached(sig, ctypes.byref(siglen), msg, ctypes.c_ulonglong(len(msg)), sk) == 0
    return sig.raw


def sodium_verify(pk, sig, msg):
    return SODIUM.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def sodium_reduce(b64):
    out = ctypes.create_string_buffer(32)
    SODIUM.crypto_core_ed25519_scalar_reduce(out, b64)
    return out.raw


NODE_VERIFY = r"""
const crypto = require('crypto');
const items = JSON.parse(require('fs').readFileSync(0, 'utf8'));
const prefix = Buffer.from('302a300506032b6570032100', 'hex');
const out = items.map(([pk, sig, msg]) => {
  const key = crypto.createPublicKey({key: Buffer.concat([prefix, Buffer.from(pk, 'hex')]), format: 'der', type: 'spki'});
  return crypto.verify(null, Buffer.from(msg, 'hex'), key, Buffer.from(sig, 'hex'));
});
process.stdout.write(JSON.stringify(out));
"""


def node_verify_many(items):
    try:
        r = subprocess.run(["node", "-e", NODE_VERIFY], input=json.dumps(items).encode(),
                           capture_output=True, timeout=600)
    except (OSError, subprocess.TimeoutExpired):
        return None
    if r.returncode != 0:
        return None
    return json.loads(r.stdout)


# ---------------------------------------------------------------- vector construction
def main():
    os.makedirs(OUT, exist_ok=True)
    rnd = random.Random(2025)
    rb = lambda n: bytes(rnd.getrandbits(8) for _ in range(n))
    pins = {"libsodium": SODIUM is not None}

    # ---- reference key fixtures: Docker/validators/validator-*/network-key.json (data copy)
    docker = [
        ("TVvqbV9LvRfPslOSMFUNxm0w0PfH9ytSVkZuqKN0DtU=", "2kRrHl/taJiAd+xzt0yykxexiqh0wOJ0NhpUYyZG280="),
        ("5EpwzXiTL8B2OuazfuHC9S9Hp0uRZFYElYj25ilVljM=", "yP3ZZjwX0njXV5l4vgbXzErOizcVskF4xzrJZwfJRUQ="),
        ("Rd6StTmpiACXs/wN/pv5DtG9h+OImvplxD/xTU2sV0I=", "KPigXDOul6tXan2pmfIk0J4wEYee+TQBB/siF6P5nTI="),
        ("6BHCB8duL285+IiyvcbLnozof/jElGmjYef5wHN9MXk=", "ifdVHBnI9J6bMbcbLZwzRb4T1fIzkGc2+LWitrGTwAM="),
    ]
    keys = []
    for name, secret in docker:
        seed = base64.b64decode(secret)
        pk = pubkey(seed)
        assert pk == base64.b64decode(name), "Docker key fixture mismatch"
        if SODIUM:
            assert sodium_seed_keypair(seed)[0] == pk
        keys.append({"seed": seed.hex(), "pk": pk.hex(), "source": "Docker/validators network-key.json"})

    vectors = []

    def add(pk, sig, msg, cat, note=""):
        exp = verify(pk, sig, msg)
        vectors.append({"pk": pk.hex(), "sig": sig.hex(), "msg": msg.hex(), "expect": exp,
                        "category": cat, "note": note})
        return exp

    # ---- honest signatures: message lengths across SHA-512 block boundaries
    lengths = [0, 1, 31, 32, 33, 46, 47, 48, 49, 63, 64, 65, 111, 112, 113, 127, 128, 129,
               174, 175, 176, 239, 240, 255, 256, 300, 511, 512, 513, 1000]
    seeds = [rb(32) for _ in range(24)] + [bytes.fromhex(k["seed"]) for k in keys]
    honest = []
    for i, n in enumerate(lengths * 2):
        seed = seeds[i % len(seeds)]
        msg = rb(n)
        sig = sign(seed, msg)
        pk = pubkey(seed)
        if SODIUM:
            assert sodium_sign(seed, msg) == sig, "RFC 8032 signature mismatch vs libsodium"
        assert add(pk, sig, msg, "honest")
        honest.append((seed, pk, msg, sig))

    torsion, T8 = torsion_points()
    small_encs = []
    for (x, y) in torsion:
        small_encs.extend(encodings_of(x, y))
    small_set = sorted(set(small_encs))

    # ---- B1: bit flips in R, s or message
    for i in range(40):
        seed, pk, msg, sig = honest[i % len(honest)]
        which = i % 3
        if which == 0:
            bit = rnd.randrange(255)
            s2 = bytearray(sig); s2[bit // 8] ^= 1 << (bit % 8)
            add(pk, bytes(s2), msg, "B1_flip_R")
        elif which == 1:
            bit = rnd.randrange(252)
            s2 = bytearray(sig); s2[32 + bit // 8] ^= 1 << (bit % 8)
            add(pk, bytes(s2), msg, "B1_flip_s")
        else:
            m2 = bytearray(msg if msg else b"\x00")
            bit = rnd.randrange(len(m2) * 8)
            m2[bit // 8] ^= 1 << (bit % 8)
            add(pk, sig, bytes(m2), "B1_flip_msg")
    # ---- B2: s + l, s with top bit set, s = l, s = l-1 (with honest R)
    for i in range(12):
        seed, pk, msg, sig = honest[i]
        s = int.from_bytes(sig[32:], "little")
        variants = [s + L, s | (1 << 255), L, L - 1, s + 2 * L, 2**256 - 1]
        sv = variants[i % len(variants)]
        if sv < 2**256:
            add(pk, sig[:32] + sv.to_bytes(32, "little"), msg, "B2_s_noncanonical")
    # ---- B3 / B8 (as R): small-order R (every decodable encoding, canonical or not),
    #      honest key, s = k*a  => accept
    for i, Renc in enumerate(small_set):
        seed = seeds[i % len(seeds)]
        a, _ = expand(seed)
        pk = pubkey(seed)
        msg = rb(32)
        k = H(Renc, pk, msg) % L
        s = (k * a) % L
        y = int.from_bytes(Renc, "little") & ((1 << 255) - 1)
        cat = "B3_R_noncanonical" if y >= p else ("B8_R_negzero" if (decompress(Renc)[0] == 0 and Renc[31] >> 7) else "B5_R_small_order")
        assert add(pk, Renc + s.to_bytes(32, "little"), msg, cat)
        # and a wrong s => reject
        add(pk, Renc + ((s + 1) % L).to_bytes(32, "little"), msg, cat + "_bad")
    # ---- B4 / B8 (as A): small-order A (all encodings), R = [s]B  => accept; wrong R => reject
    for i, Aenc in enumerate(small_set):
        s = rnd.randrange(L)
        Renc = compress(pmul(s, B))
        msg = rb(rnd.choice([0, 32, 100]))
        y = int.from_bytes(Aenc, "little") & ((1 << 255) - 1)
        cat = "B4_A_noncanonical" if y >= p else ("B8_A_negzero" if (decompress(Aenc)[0] == 0 and Aenc[31] >> 7) else "B5_A_small_order")
        assert add(Aenc, Renc + s.to_bytes(32, "little"), msg, cat)
        R2 = compress(pmul(s + 1, B))
        add(Aenc, R2 + s.to_bytes(32, "little"), msg, cat + "_bad")
    # ---- B6: honest signature with a torsion component in R (s recomputed over the new R bytes)
    for i in range(16):
        seed = seeds[i % len(seeds)]
        a, prefix = expand(seed)
        pk = pubkey(seed)
        msg = rb(rnd.choice([32, 64, 512]))
        r = rnd.randrange(L)
        T = pmul(1 + (i % 7), T8)
        Rp = padd(pmul(r, B), T)
        Renc = compress(Rp)
        k = H(Renc, pk, msg) % L
        s = (r + k * a) % L
        assert add(pk, Renc + s.to_bytes(32, "little"), msg, "B6_R_torsion")
        # torsion on A instead: A' = A + T, signature made for A' with the same secret
        Ap = padd(pmul(a, B), T)
        Aenc = compress(Ap)
        k2 = H(compress(pmul(r, B)), Aenc, msg) % L
        s2 = (r + k2 * a) % L
        add(Aenc, compress(pmul(r, B)) + s2.to_bytes(32, "little"), msg, "B6_A_torsion")
    # ---- B7: non-decodable R or A
    nd = 0
    while nd < 16:
        yb = bytearray(rb(32))
        if decompress(bytes(yb)) is not None:
            continue
        seed, pk, msg, sig = honest[nd]
        if nd % 2 == 0:
            assert not add(pk, bytes(yb) + sig[32:], msg, "B7_R_undecodable")
        else:
            assert not add(bytes(yb), sig, msg, "B7_A_undecodable")
        nd += 1
    # ---- ZIP-215 small-order table: every small-order A x every small-order R, s = 0
    zip215 = []
    for Aenc in small_set:
        for Renc in small_set:
            msg = b"Zcash"
            sig = Renc + bytes(32)
            ok = verify(Aenc, sig, msg)
            assert ok, "ZIP-215 small-order case must verify"
            zip215.append({"pk": Aenc.hex(), "sig": sig.hex(), "msg": msg.hex(), "expect": True})

    # ---- independent pins: libsodium + OpenSSL on canonical, torsion-free vectors
    def canonical_torsion_free(v):
        pk, sig = bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"])
        for enc in (pk, sig[:32]):
            y = int.from_bytes(enc, "little") & ((1 << 255) - 1)
            P = decompress(enc)
            if P is None or y >= p:
                return False
            if not is_identity(pmul(L, P)) or is_identity(pmul(8, P)):
                return False  # torsion component, or small order (libsodium rejects those)
            if compress(P) != enc:
                return False
        return int.from_bytes(sig[32:], "little") < L

    subset = [v for v in vectors if canonical_torsion_free(v)]
    if SODIUM:
        for v in subset:
            sv = sodium_verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]))
            assert sv == v["expect"], ("libsodium disagrees", v)
        lib_small = [sodium_verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]))
                     for v in vectors if v["category"].startswith(("B5", "B6")) and v["expect"]]
        pins["libsodium_checked"] = len(subset)
        pins["libsodium_rejects_cofactored_only_accepts"] = sum(1 for x in lib_small if not x)
    nv = node_verify_many([[v["pk"], v["sig"], v["msg"]] for v in subset])
    if nv is not None:
        for v, ok in zip(subset, nv):
            assert ok == v["expect"], ("OpenSSL disagrees", v)
        pins["openssl_checked"] = len(subset)

    # ---- batches: index lists into vectors with the expected batch verdict
    batches = []
    good = [i for i, v in enumerate(vectors) if v["expect"]]
    bad = [i for i, v in enumerate(vectors) if not v["expect"]]
    for t in range(40):
        n = rnd.choice([1, 2, 3, 7, 33, 64, 65, 130])
        items = [rnd.choice(good) for _ in range(n)]
        if t % 2 == 1:
            items[rnd.randrange(n)] = rnd.choice(bad)
        batches.append({"items": items, "expect": all(vectors[i]["expect"] for i in items)})

    # ---- hashes / scalar reduction
    hashv = {"sha512": [], "blake2b256": [], "sc_reduce": []}
    for n in [0, 1, 3, 111, 112, 127, 128, 129, 239, 240, 1000]:
        m = rb(n)
        hashv["sha512"].append({"msg": m.hex(), "digest": hashlib.sha512(m).hexdigest()})
    for n in [0, 1, 3, 64, 127, 128, 129, 255, 256, 257, 1000, 4096]:
        m = rb(n)
        hashv["blake2b256"].append({"msg": m.hex(), "digest": hashlib.blake2b(m, digest_size=32).hexdigest()})
    hashv["blake2b256_empty"] = hashlib.blake2b(b"", digest_size=32).hexdigest()
    for i in range(40):
        x = rb(64) if i > 3 else [bytes(64), b"\xff" * 64, L.to_bytes(64, "little"), (L - 1).to_bytes(64, "little")][i]
        red = (int.from_bytes(x, "little") % L).to_bytes(32, "little")
        if SODIUM:
            assert sodium_reduce(x) == red
        hashv["sc_reduce"].append({"in": x.hex(), "out": red.hex()})

    # ---- worker batches: bincode WorkerMessage::Batch layout (types/src/tests/batch_serde.rs:39-86)
    def bincode_batch(txs):
        out = struct.pack("<I", 0) + struct.pack("<Q", len(txs))
        for t in txs:
            out += struct.pack("<Q", len(t)) + t
        return out

    golden_layout = bincode_batch([bytes([1] * 5)] * 2).hex()
    assert golden_layout == "0000000002000000000000000500000000000000010101010105000000000000000101010101"
    batchv = []
    for ntx, size in [(0, 0), (1, 0), (2, 5), (3, 100), (100, 512), (977, 512)]:
        txs = []
        for j in range(ntx):
            # node/src/benchmark_client.rs:153-168: [tag u8][u64 BE counter][zero pad to size]
            t = (bytes([1]) + struct.pack(">Q", rnd.getrandbits(64))) if size >= 9 else rb(size)
            txs.append(t.ljust(size, b"\x00")[:size] if size else b"")
        digest = hashlib.blake2b(b"".join(txs), digest_size=32).hexdigest()
        rec = {"ntx": ntx, "tx_size": size, "digest": digest}
        if ntx <= 100:
            rec["serialized"] = bincode_batch(txs).hex()
        else:
            rec["gen"] = "node/src/benchmark_client.rs tx format, python random.Random(2025) stream"
            rec["serialized_sha256"] = hashlib.sha256(bincode_batch(txs)).hexdigest()
        batchv.append(rec)
    # malformed serialized batches -> InvalidArgumentError(offset) (offset of the failing u64 read)
    bad_ser = [
        {"hex": "00000000", "err_offset": 4},
        {"hex": "000000000100000000000000", "err_offset": 12},
        {"hex": "00000000010000000000000005000000000000000101", "err_offset": 12},
    ]

    # ---- Narwhal digests (types/src/primary.rs:209-227, 351-364, 594-607)
    def b2(*parts):
        h = hashlib.blake2b(digest_size=32)
        for x in parts:
            h.update(x)
        return h.digest()

    digests = []
    for i in range(8):
        author = rb(32)
        rnd_ = rnd.getrandbits(64)
        ep = rnd.getrandbits(64)
        payload = [(rb(32), rnd.getrandbits(32)) for _ in range(i % 3)]
        parents = sorted(rb(32) for _ in range(i * 3))
        hparts = [author, struct.pack("<Q", rnd_), struct.pack("<Q", ep)]
        for dg, wid in payload:
            hparts += [dg, struct.pack("<I", wid)]
        hparts += parents
        hid = b2(*hparts)
        origin = author
        vote_digest = b2(hid, struct.pack("<Q", rnd_), struct.pack("<Q", ep), origin)
        digests.append({"author": author.hex(), "round": rnd_, "epoch": ep,
                        "payload": [[dg.hex(), wid] for dg, wid in payload],
                        "parents": [x.hex() for x in parents],
                        "header_digest": hid.hex(), "vote_digest": vote_digest.hex(),
                        "certificate_digest": vote_digest.hex()})

    def dump(name, obj):
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(obj, f, indent=0, sort_keys=True)

    meta = {"generator": "oracle/gen_golden.py", "seed": 2025, "pins": pins,
            "semantics": "ed25519-consensus 2.0.1 / ZIP-215 (SURVEY.md Appendix A)"}
    dump("ed25519_vectors.json", {"meta": meta, "vectors": vectors, "batches": batches})
    dump("zip215_small_order.json", {"meta": meta, "vectors": zip215,
                                     "encodings": [e.hex() for e in small_set]})
    dump("keys.json", {"meta": meta, "keys": keys})
    dump("hash_vectors.json", {"meta": meta, **hashv})
    dump("worker_batches.json", {"meta": meta, "layout_golden": golden_layout, "batches": batchv,
                                 "malformed": bad_ser})
    dump("narwhal_digests.json", {"meta": meta, "digests": digests})
    cats = {}
    for v in vectors:
        cats.setdefault(v["category"], [0, 0])[0 if v["expect"] else 1] += 1
    print(json.dumps({"vectors": len(vectors), "zip215": len(zip215), "pins": pins, "categories": cats}, indent=1))


if __name__ == "__main__":
    sys.exit(main())
