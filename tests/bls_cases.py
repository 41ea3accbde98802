"""Adversarial BLS12-381 inputs shared by the oracle and GPU tests (test infrastructure): points
on the curves but outside the prime-order subgroups, bad encodings, identities."""
import bls_ffi as B

p = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab


def not_in_g1(start=5):
    """a compressed point on y^2 = x^3 + 4 outside G1 (the cofactor is not cleared)"""
    x = start
    while True:
        for sign in (0, 0x20):
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80 | sign
            rc, _ = B.g1_decompress(bytes(b))
            if rc == 0 and not B.lib().orb_g1_in_group(bytes(b)):
                return bytes(b)
        x += 1


def not_in_g2(start=3):
    x = start
    while True:
        b = bytearray(bytes(48) + x.to_bytes(48, "big"))
        b[0] |= 0x80
        rc, _ = B.g2_decompress(bytes(b))
        if rc == 0 and not B.lib().orb_g2_in_group(bytes(b)):
            return bytes(b)
        x += 1


def off_curve_g1():
    x = 1
    while True:
        b = bytearray(x.to_bytes(48, "big"))
        b[0] |= 0x80
        if B.g1_decompress(bytes(b))[0] == B.ORB_NOT_ON_CURVE:
            return bytes(b)
        x += 1


def bad_encodings_g1(sig):
    no_flag = bytearray(sig)
    no_flag[0] &= 0x7f
    big = bytearray(p.to_bytes(48, "big"))
    big[0] |= 0x80
    return [bytes(no_flag), bytes(big), bytes([0xc1]) + bytes(47), bytes([0xe0]) + bytes(47), off_curve_g1()]


IDENTITY_G1 = bytes([0xc0]) + bytes(47)
IDENTITY_G2 = bytes([0xc0]) + bytes(95)


def negate_g2(pk):
    b = bytearray(pk)
    b[0] ^= 0x20
    return bytes(b)
