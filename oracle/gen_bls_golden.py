#!/usr/bin/env python3
"""Golden vectors for the BLS12-381 path (the reference's default scheme,
crypto/src/lib.rs:29-33 -> fastcrypto 0.1.2 bls12381 -> blst 0.3.10 min_sig: public keys in G2
(96-byte compressed), signatures in G1 (48-byte compressed)).  Test infrastructure, run only in
this container (it reads /root/reference); writes tests/golden/bls12381_kats.json.

Pins, each from outside this repository:
  * keygen: the reference's own BLS12381KeyPair fixtures Docker/validators/validator-{0..3}/
    primary-key.json (base64 32-byte big-endian secret -> base64 96-byte compressed G2 public
    key): pin Fp / Fp2 arithmetic, G2 scalar multiplication and the ZCash compression format;
  * hash_to_curve: the known answers of RFC 9380 Appendix J.9.1 (suite
    BLS12381G1_XMD:SHA-256_SSWU_RO_, DST "QUUX-V01-CS02-with-BLS12381G1_XMD:SHA-256_SSWU_RO_",
    msg "" and "abc"): pin expand_message_xmd, hash_to_field, the SSWU map, the 11-isogeny
    (tools/gen_bls_iso.py) and cofactor clearing.
Derived (this restatement, big-integer Python, checked against the pins above before writing):
  * sign: sk * H(m) for the four Docker secrets under fastcrypto's DST
    "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_" (48-byte compressed G1).
The pairing has no published value here; it is pinned by algebra in the tests (bilinearity,
non-degeneracy, e(P, Q)^r = 1, the twisted/projective Miller loop equal to a plain affine one on
the untwisted curve)."""
import base64
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_bls_iso as iso  # noqa: E402

p = iso.p
r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
H_EFF = 0xd201000000010001
G2 = ((0x024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8,
       0x13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e),
      (0x0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801,
       0x0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be))
G1 = (0x17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb,
      0x08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1)
DST_NUL = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"
DST_RFC = b"QUUX-V01-CS02-with-BLS12381G1_XMD:SHA-256_SSWU_RO_"
# RFC 9380 Appendix J.9.1 (BLS12381G1_XMD:SHA-256_SSWU_RO_): msg -> P = (x, y)
RFC_J91 = [
    ("", "052926add2207b76ca4fa57a8734416c8dc95e24501772c814278700eed6d1e4e8cf62d9c09db0fac349612b759e79a1",
     "08ba738453bfed09cb546dbb0783dbb3a5f1f566ed67bb6be0e8c67e2e81a4cc68ee29813bb7994998f3eae0c9c6a265"),
    ("abc", "03567bc5ef9c690c2ab2ecdf6a96ef1c139cc0b2f284dca0a9a7943388a49a3aee664ba5379a7655d3c68900be2f6903",
     "0b9c15f3fe6e5cf4211f346271d7b01c8f3b28be689c8429c85b67af215533311f0b8dfaaa154fa6b88176c229f2885d"),
]
inv = iso.inv


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)


def f2add(a, b):
    return ((a[0] + b[0]) % p, (a[1] + b[1]) % p)


def f2sub(a, b):
    return ((a[0] - b[0]) % p, (a[1] - b[1]) % p)


def f2inv(a):
    n = inv((a[0] * a[0] + a[1] * a[1]) % p)
    return (a[0] * n % p, -a[1] * n % p)


class Fp:
    add = staticmethod(lambda a, b: (a + b) % p)
    sub = staticmethod(lambda a, b: (a - b) % p)
    mul = staticmethod(lambda a, b: a * b % p)
    inv = staticmethod(inv)
    zero, three = 0, 3


class Fp2:
    add, sub, mul, inv = staticmethod(f2add), staticmethod(f2sub), staticmethod(f2mul), staticmethod(f2inv)
    zero, three = (0, 0), (3, 0)


def ec_add(F, P, Q):
    if P is None:
        return Q
    if Q is None:
        return P
    if P[0] == Q[0]:
        if F.add(P[1], Q[1]) == F.zero:
            return None
        lam = F.mul(F.mul(F.three, F.mul(P[0], P[0])), F.inv(F.add(P[1], P[1])))
    else:
        lam = F.mul(F.sub(Q[1], P[1]), F.inv(F.sub(Q[0], P[0])))
    x = F.sub(F.sub(F.mul(lam, lam), P[0]), Q[0])
    return (x, F.sub(F.mul(lam, F.sub(P[0], x)), P[1]))


def ec_mul(F, k, P):
    R = None
    for bit in bin(k)[2:]:
        R = ec_add(F, R, R)
        if bit == "1":
            R = ec_add(F, R, P)
    return R


def compress_g1(P):
    x, y = P
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if y > (p - 1) // 2 else 0)
    return bytes(b)


def compress_g2(P):
    x, y = P
    big = y[1] > (p - 1) // 2 if y[1] else y[0] > (p - 1) // 2
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if big else 0)
    return bytes(b)


# ---- hash_to_curve (RFC 9380 §5.3.1, §6.6.2, §6.6.3, §7, §8.8.1) ----
def expand_xmd(msg, dst, n):
    h = lambda x: hashlib.sha256(x).digest()
    ell = (n + 31) // 32
    dp = dst + bytes([len(dst)])
    b0 = h(bytes(64) + msg + n.to_bytes(2, "big") + b"\0" + dp)
    bs = [h(b0 + b"\1" + dp)]
    for i in range(2, ell + 1):
        bs.append(h(bytes(x ^ y for x, y in zip(b0, bs[-1])) + bytes([i]) + dp))
    return b"".join(bs)[:n]


def hash_to_field(msg, dst):
    ub = expand_xmd(msg, dst, 128)
    return [int.from_bytes(ub[64 * i:64 * i + 64], "big") % p for i in range(2)]


def sqrt(a):
    s = pow(a, (p + 1) // 4, p)
    return s if s * s % p == a % p else None


def sswu(u):
    A, B, Z = iso.A_ISO, iso.B_ISO, 11
    tv1 = (Z * Z * pow(u, 4, p) + Z * u * u) % p
    x1 = (-B * inv(A) * (1 + inv(tv1))) % p if tv1 else B * inv(Z * A) % p
    gx1 = (x1 ** 3 + A * x1 + B) % p
    y = sqrt(gx1)
    x = x1
    if y is None:
        x = Z * u * u * x1 % p
        y = sqrt((x ** 3 + A * x + B) % p)
    if u % 2 != y % 2:
        y = -y % p
    return x, y


def iso_map(P, consts):
    xnum, xden, ynum, yden = consts
    ev = lambda f, x: sum(c * pow(x, i, p) for i, c in enumerate(f)) % p
    x, y = P
    return (ev(xnum, x) * inv(ev(xden, x)) % p, y * ev(ynum, x) * inv(ev(yden, x)) % p)


def hash_to_g1(msg, dst, consts):
    u = hash_to_field(msg, dst)
    Q = ec_add(Fp, iso_map(sswu(u[0]), consts), iso_map(sswu(u[1]), consts))
    return ec_mul(Fp, H_EFF, Q)


def main():
    consts = iso.derive()
    out = {"note": __doc__.split("\n\n")[0], "keygen": [], "hash_to_g1": [], "sign": [],
           "dst_nul": DST_NUL.decode(), "g1_gen": compress_g1(G1).hex(), "g2_gen": compress_g2(G2).hex()}
    assert ec_mul(Fp2, r, G2) is None and ec_mul(Fp, r, G1) is None
    for m, x, y in RFC_J91:
        P = hash_to_g1(m.encode(), DST_RFC, consts)
        assert P == (int(x, 16), int(y, 16)), f"RFC 9380 J.9.1 msg={m!r} not reproduced"
        out["hash_to_g1"].append({"dst": DST_RFC.decode(), "msg": m.encode().hex(), "x": x, "y": y,
                                  "source": "RFC 9380 Appendix J.9.1"})
    sks = []
    for i in range(4):
        f = os.path.join("/root/reference/Docker/validators", f"validator-{i}", "primary-key.json")
        with open(f) as fh:
            kp = json.load(fh)
        sk = base64.b64decode(kp["secret"])
        pk = base64.b64decode(kp["name"])
        assert compress_g2(ec_mul(Fp2, int.from_bytes(sk, "big"), G2)) == pk, f
        out["keygen"].append({"sk": sk.hex(), "pk": pk.hex(),
                              "source": f"reference Docker/validators/validator-{i}/primary-key.json"})
        sks.append(int.from_bytes(sk, "big"))
    for i, sk in enumerate(sks):
        for m in (b"", b"Hello, world!", bytes(range(32))):
            H = hash_to_g1(m, DST_NUL, consts)
            out["sign"].append({"sk_index": i, "msg": m.hex(), "sig": compress_g1(ec_mul(Fp, sk, H)).hex(),
                                "h": compress_g1(H).hex()})
    path = os.path.join(ROOT, "tests", "golden", "bls12381_kats.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", os.path.relpath(path, ROOT))


if __name__ == "__main__":
    main()
