// bls381.h -- BLS12-381 arithmetic for gfx950 VALU (the reference's default
// signature scheme, crypto/src/lib.rs:29-33 -> fastcrypto 0.1.2 bls12381 -> blst 0.3.10 min_sig).
//
// One pairing check per lane: like the Ed25519 field (fe25519.h) the natural multiply on CDNA4 is
// the 32x32->64 multiply-accumulate v_mad_u64_u32, so an Fp element is 14 limbs of 28 bits
// (392 bits) and a Montgomery product (R = 2^392) is 196 multiply-adds into 64-bit column sums
// followed by 14 reduction rows of 14 multiply-adds -- no carry handling inside the sums (a
// column holds at most 28 products of 2^56 < 2^61).  Every add / sub / mul returns normalised
// limbs (< 2^28) and a value in [0, 2p), so formulas need no magnitude bookkeeping; values are
// made canonical ([0, p)) only to compare, to test the sign or to serialise.
//
// Everything is __host__ __device__ so the CPU test build (tests/hostemu/bls_hostemu.cpp) runs
// the same code against the oracle (oracle/bls_oracle.c); the engine only runs it on the GPU.
// Algorithms (the same mathematical objects as the oracle, computed differently where it pays):
//   tower Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(1+u)), Fp12 = Fp6[w]/(w^2-v);
//   Miller loop over |x| = 0xd201000000010000 with Jacobian T on the M-type twist and sparse
//   line products (Costello-Lange-Naehrig, eprint 2010/354 Alg. 26/27), conjugated for x < 0;
//   final exponentiation f^(3(p^12-1)/r): easy part (p^6-1)(p^2+1), hard part through
//   3(p^4-p^2+1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3 with Granger-Scott cyclotomic squarings;
//   subgroup tests by endomorphism (Scott 2021): phi(P) = [-x^2] P on G1, psi(Q) = [x] Q on G2;
//   hash_to_curve G1 of RFC 9380 (SHA-256 expand_message_xmd, SSWU, 11-isogeny, h_eff).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls381_consts.h"

#ifndef NWV_HD
#define NWV_HD __host__ __device__ __forceinline__
#endif
#define BLS_HD __host__ __device__ inline
#ifndef BLS_NOINLINE
#define BLS_NOINLINE __host__ __device__ __attribute__((noinline))
#endif

namespace bls {

constexpr int NL = 14;
constexpr uint32_t LM = (1u << 28) - 1;

struct fp { uint32_t l[NL]; };
struct fp2 { fp c0, c1; };
struct fp6 { fp2 c0, c1, c2; };
struct fp12 { fp6 c0, c1; };
struct g1a { fp x, y; };            // affine
struct g1j { fp x, y, z; bool inf; };  // Jacobian (X/Z^2, Y/Z^3)
struct g2a { fp2 x, y; };
struct g2j { fp2 x, y, z; bool inf; };

#define BLS_CONST(name, ...) NWV_HD fp name() { fp r = {__VA_ARGS__}; return r; }
BLS_CONST(k_p, BLS_P)
BLS_CONST(k_p2, BLS_P2)
BLS_CONST(k_one, BLS_ONE)
BLS_CONST(k_r2, BLS_R2)
BLS_CONST(k_b1, BLS_B1)
BLS_CONST(k_beta, BLS_BETA)
BLS_CONST(k_sswu_a, BLS_SSWU_A)
BLS_CONST(k_sswu_b, BLS_SSWU_B)
BLS_CONST(k_sswu_z, BLS_SSWU_Z)
BLS_CONST(k_sswu_c2, BLS_SSWU_C2)
BLS_CONST(k_g1x, BLS_G1X)
BLS_CONST(k_g1y, BLS_G1Y)
BLS_CONST(k_two256, BLS_TWO256)
#define BLS_CONST2(name, A, B) NWV_HD fp2 name() { fp2 r = {{A}, {B}}; return r; }
BLS_CONST2(k_b2, BLS_B2_C0, BLS_B2_C1)
BLS_CONST2(k_g2x, BLS_G2X_C0, BLS_G2X_C1)
BLS_CONST2(k_g2y, BLS_G2Y_C0, BLS_G2Y_C1)
BLS_CONST2(k_psi_cx, BLS_PSI_CX_C0, BLS_PSI_CX_C1)
BLS_CONST2(k_psi_cy, BLS_PSI_CY_C0, BLS_PSI_CY_C1)

// ------------------------------------------------------------------------------------ Fp
NWV_HD fp fp_zero() { fp r; for (int i = 0; i < NL; i++) r.l[i] = 0; return r; }

// s (limbs < 2^28) minus c (< 2^28 each) with borrow; returns the final borrow (0 or -1)
NWV_HD int32_t limb_sub(fp& t, const fp& s, const fp& c) {
    int32_t br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const int32_t d = (int32_t)s.l[j] - (int32_t)c.l[j] + br;
        t.l[j] = (uint32_t)d & LM;
        br = d >> 28;
    }
    return br;
}
NWV_HD void limb_add(fp& t, const fp& a, const fp& b) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const uint32_t s = a.l[j] + b.l[j] + c;
        t.l[j] = s & LM;
        c = s >> 28;
    }
    t.l[NL - 1] += c << 28;
}
NWV_HD fp fp_sel(bool keep_a, const fp& a, const fp& b) {
    fp r;
#pragma unroll
    for (int j = 0; j < NL; j++) r.l[j] = keep_a ? a.l[j] : b.l[j];
    return r;
}
// [0, 4p) -> [0, 2p)
NWV_HD fp fp_red2(const fp& s) {
    fp t;
    const int32_t br = limb_sub(t, s, k_p2());
    return fp_sel(br != 0, s, t);
}
NWV_HD fp fp_add(const fp& a, const fp& b) {
    fp s;
    limb_add(s, a, b);
    return fp_red2(s);
}
NWV_HD fp fp_sub(const fp& a, const fp& b) {
    fp t, u;
    const int32_t br = limb_sub(t, a, b);  // on a borrow t = a - b + 2^392
    limb_add(u, t, k_p2());
    u.l[NL - 1] &= LM;                     // (a - b + 2p) mod 2^392, in [0, 2p)
    return fp_sel(br == 0, t, u);
}
NWV_HD fp fp_neg(const fp& a) { return fp_sub(fp_zero(), a); }
NWV_HD fp fp_dbl(const fp& a) { return fp_add(a, a); }
// canonical representative in [0, p)
NWV_HD fp fp_canon(const fp& a) {
    fp t;
    const int32_t br = limb_sub(t, a, k_p());
    return fp_sel(br != 0, a, t);
}
NWV_HD bool fp_is_zero(const fp& a) {
    const fp c = fp_canon(a);
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) o |= c.l[j];
    return o == 0;
}
NWV_HD bool fp_eq(const fp& a, const fp& b) { return fp_is_zero(fp_sub(a, b)); }

// Montgomery product a b / 2^392 mod p; a, b < 2p with limbs < 2^28 -> result < 2p, limbs < 2^28
BLS_HD fp fp_mul(const fp& a, const fp& b) {
    const fp P = k_p();
    uint64_t c[2 * NL];
#pragma unroll
    for (int k = 0; k < 2 * NL; k++) c[k] = 0;
#pragma unroll
    for (int i = 0; i < NL; i++)
#pragma unroll
        for (int j = 0; j < NL; j++) c[i + j] += (uint64_t)a.l[i] * b.l[j];
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const uint32_t m = ((uint32_t)c[i] * BLS_N0) & LM;
#pragma unroll
        for (int j = 0; j < NL; j++) c[i + j] += (uint64_t)m * P.l[j];
        c[i + 1] += c[i] >> 28;
    }
    fp r;
#pragma unroll
    for (int k = NL; k < 2 * NL - 1; k++) {
        c[k + 1] += c[k] >> 28;
        r.l[k - NL] = (uint32_t)c[k] & LM;
    }
    r.l[NL - 1] = (uint32_t)c[2 * NL - 1];
    return r;
}
BLS_HD fp fp_sqr(const fp& a) {
    const fp P = k_p();
    uint64_t c[2 * NL];
    uint32_t a2[NL];
#pragma unroll
    for (int k = 0; k < 2 * NL; k++) c[k] = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) a2[i] = a.l[i] << 1;
#pragma unroll
    for (int i = 0; i < NL; i++) {
        c[2 * i] += (uint64_t)a.l[i] * a.l[i];
#pragma unroll
        for (int j = i + 1; j < NL; j++) c[i + j] += (uint64_t)a2[i] * a.l[j];
    }
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const uint32_t m = ((uint32_t)c[i] * BLS_N0) & LM;
#pragma unroll
        for (int j = 0; j < NL; j++) c[i + j] += (uint64_t)m * P.l[j];
        c[i + 1] += c[i] >> 28;
    }
    fp r;
#pragma unroll
    for (int k = NL; k < 2 * NL - 1; k++) {
        c[k + 1] += c[k] >> 28;
        r.l[k - NL] = (uint32_t)c[k] & LM;
    }
    r.l[NL - 1] = (uint32_t)c[2 * NL - 1];
    return r;
}
NWV_HD fp fp_to_mont(const fp& plain) { return fp_mul(plain, k_r2()); }
NWV_HD fp fp_from_mont(const fp& a) {
    fp one = fp_zero();
    one.l[0] = 1;
    return fp_canon(fp_mul(a, one));
}
// a^e for a constant exponent given as 12 little-endian 32-bit words (wave-uniform control flow):
// sliding windows of up to 5 bits over the odd powers a, a^3, .., a^31 -- for the 379-bit square
// root / inversion exponents 379 squarings + 67 products + 16 for the table, against 228 products
// bit by bit
BLS_NOINLINE fp fp_pow(const fp& a, const uint32_t* e) {
    fp t[16];
    t[0] = a;
    const fp a2 = fp_sqr(a);
    for (int k = 1; k < 16; k++) t[k] = fp_mul(t[k - 1], a2);
    auto bit = [&](int i) -> uint32_t { return (e[i >> 5] >> (i & 31)) & 1u; };
    int i = 383;
    while (i >= 0 && !bit(i)) i--;
    fp acc = k_one();
    bool started = false;
    while (i >= 0) {
        if (!bit(i)) {
            acc = fp_sqr(acc);
            i--;
            continue;
        }
        int j = i - 4 < 0 ? 0 : i - 4;
        while (!bit(j)) j++;  // the window ends on a set bit (bit i is set)
        uint32_t v = 0;
        for (int k = i; k >= j; k--) v = (v << 1) | bit(k);
        if (started)
            for (int k = i; k >= j; k--) acc = fp_sqr(acc);
        acc = started ? fp_mul(acc, t[v >> 1]) : t[v >> 1];
        started = true;
        i = j - 1;
    }
    return acc;
}
NWV_HD fp fp_inv(const fp& a) {
    const uint32_t e[12] = BLS_E_INV;
    return fp_pow(a, e);
}
// ---- variable-time inversion: batched binary GCD (Pornin, eprint 2020/972) -------------------
// The inputs of a verification are public, so the inversion need not be constant time.  Binary
// extended Euclid with the invariants a = u y, b = v y (mod p), started at (a, b) = (y, p),
// (u, v) = (1, 0): while a != 0, an odd a below b swaps with b, then a -= b, and a, u halve.
// Thirty such steps run at a time on 62-bit approximations of a and b (each one's low 30 bits and
// its top 32 bits at the larger length) collecting a matrix [f0 g0; f1 g1], |entries| <= 2^30; the
// matrix then updates the 384-bit values once: (a, b) <- M (a, b) / 2^30 (exact; a negative
// result is negated with its row) and (u, v) <- M (u, v) / 2^30 mod p (Montgomery halving by
// 2^30).  About 26 batches for a 381-bit y (at most 2 len - 1 = 761 steps); when a reaches 0,
// b = 1 and v = y^-1.  On the device the values are wave-uniform, so the steps run on the scalar
// unit.
constexpr int BW = 12;
NWV_HD void w_from_fp(uint32_t* o, const fp& a) {  // a canonical, limbs < 2^28
#pragma unroll
    for (int k = 0; k < BW; k++) {
        const int bit = 32 * k, j = bit / 28, sh = bit % 28;
        uint32_t v = a.l[j] >> sh;
        if (j + 1 < NL) v |= a.l[j + 1] << (28 - sh);
        if (sh > 24 && j + 2 < NL) v |= a.l[j + 2] << (56 - sh);
        o[k] = v;
    }
}
NWV_HD fp fp_from_w(const uint32_t* w) {
    fp r;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const int bit = 28 * j, idx = bit >> 5, sh = bit & 31;
        uint32_t v = idx < BW ? w[idx] >> sh : 0;
        if (sh > 4 && idx + 1 < BW) v |= w[idx + 1] << (32 - sh);
        r.l[j] = v & LM;
    }
    return r;
}
NWV_HD uint32_t w_uni(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_readfirstlane(x);
#else
    return x;
#endif
}
NWV_HD int w_bitlen(const uint32_t* a) {
    for (int i = BW - 1; i >= 0; i--)
        if (a[i]) return 32 * i + 32 - __builtin_clz(a[i]);
    return 0;
}
// bits [lo, lo + 32) of a (lo >= 0)
NWV_HD uint32_t w_bits32(const uint32_t* a, int lo) {
    const int i = lo >> 5, sh = lo & 31;
    const uint32_t x = i < BW ? a[i] : 0u, y = i + 1 < BW ? a[i + 1] : 0u;
    return sh ? (x >> sh) | (y << (32 - sh)) : x;
}
// r = (f a + g b) as a 13-word two's complement number (|f|, |g| <= 2^30, a, b < 2^384)
NWV_HD void w_lin2(uint32_t* r, int64_t f, const uint32_t* a, int64_t g, const uint32_t* b) {
    int64_t c = 0;
    for (int i = 0; i < BW; i++) {
        c += f * (int64_t)a[i] + g * (int64_t)b[i];
        r[i] = (uint32_t)c;
        c >>= 32;  // arithmetic
    }
    r[BW] = (uint32_t)c;
}
// x (13 words, two's complement) >> 30 into 12 words; returns true if x was negative (then
// the result holds |x| >> 30: the caller negates first)
NWV_HD bool w_neg13(uint32_t* x) {
    if ((int32_t)x[BW] >= 0) return false;
    uint64_t c = 1;
    for (int i = 0; i <= BW; i++) {
        c += (uint32_t)~x[i];
        x[i] = (uint32_t)c;
        c >>= 32;
    }
    return true;
}
NWV_HD void w_shr30(uint32_t* o, const uint32_t* x) {
    for (int i = 0; i < BW; i++) o[i] = (x[i] >> 30) | (x[i + 1] << 2);
}
// o += s P (s = +1 or -1; 12 words, two's complement wrap)
NWV_HD void w_addp(uint32_t* o, const uint32_t* P, int64_t s) {
    int64_t c = 0;
    for (int i = 0; i < BW; i++) {
        c += (int64_t)o[i] + s * (int64_t)P[i];
        o[i] = (uint32_t)c;
        c >>= 32;
    }
}
NWV_HD bool w_lt(const uint32_t* a, const uint32_t* b) {
    for (int i = BW - 1; i >= 0; i--)
        if (a[i] != b[i]) return a[i] < b[i];
    return false;
}
// (f u + g v) / 2^30 mod p for u, v < p: the signed sum plus m p with m = sum (-p^-1) mod 2^30
// is divisible by 2^30; the quotient V has |V| < 3p (fits 12 words as two's complement) and is
// brought into [0, p)
NWV_HD void w_lin2_modp(uint32_t* o, int64_t f, const uint32_t* u, int64_t g, const uint32_t* v, const uint32_t* P) {
    uint32_t t[BW + 1];
    w_lin2(t, f, u, g, v);
    const uint32_t m = (t[0] * BLS_P_NINV32) & ((1u << 30) - 1u);
    int64_t c = 0;
    for (int i = 0; i < BW; i++) {
        c += (int64_t)t[i] + (int64_t)m * P[i];
        t[i] = (uint32_t)c;
        c >>= 32;
    }
    t[BW] = (uint32_t)((int64_t)(int32_t)t[BW] + c);
    w_shr30(o, t);
    while ((int32_t)o[BW - 1] < 0) w_addp(o, P, 1);
    while (!w_lt(o, P)) w_addp(o, P, -1);
}
NWV_HD bool w_is_zero(const uint32_t* a) {
    uint32_t o = 0;
    for (int i = 0; i < BW; i++) o |= a[i];
    return o == 0;
}
// UNI: x is the same on every lane of the wave (the final exponentiation's norm): the steps then
// run on the scalar unit.  Otherwise every lane inverts its own x.
template <bool UNI>
BLS_NOINLINE fp fp_inv_vt_t(const fp& x) {
    const fp xc = fp_canon(x);
    if (fp_is_zero(xc)) return fp_zero();
    uint32_t a[BW], b[BW], u[BW], v[BW], P[BW];
    w_from_fp(a, xc);
    w_from_fp(P, k_p());
    for (int i = 0; i < BW; i++) {
        a[i] = UNI ? w_uni(a[i]) : a[i];
        b[i] = P[i];
        u[i] = 0;
        v[i] = 0;
    }
    u[0] = 1;
    for (int it = 0; it < 64 && !w_is_zero(a); it++) {
        int n = w_bitlen(a);
        const int nb = w_bitlen(b);
        n = n > nb ? n : nb;
        n = n > 62 ? n : 62;
        uint64_t xa = ((uint64_t)w_bits32(a, n - 32) << 30) | (a[0] & ((1u << 30) - 1u));
        uint64_t xb = ((uint64_t)w_bits32(b, n - 32) << 30) | (b[0] & ((1u << 30) - 1u));
        int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
        for (int i = 0; i < 30; i++) {
            if (xa & 1) {
                if (xa < xb) {
                    const uint64_t t = xa;
                    xa = xb;
                    xb = t;
                    int64_t s = f0;
                    f0 = f1;
                    f1 = s;
                    s = g0;
                    g0 = g1;
                    g1 = s;
                }
                xa -= xb;
                f0 -= f1;
                g0 -= g1;
            }
            xa >>= 1;
            f1 *= 2;
            g1 *= 2;
        }
        uint32_t ta[BW + 1], tb[BW + 1];
        w_lin2(ta, f0, a, g0, b);
        w_lin2(tb, f1, a, g1, b);
        if (w_neg13(ta)) {
            f0 = -f0;
            g0 = -g0;
        }
        if (w_neg13(tb)) {
            f1 = -f1;
            g1 = -g1;
        }
        w_shr30(a, ta);
        w_shr30(b, tb);
        uint32_t nu[BW];
        w_lin2_modp(nu, f0, u, g0, v, P);
        w_lin2_modp(v, f1, u, g1, v, P);
        for (int i = 0; i < BW; i++) u[i] = nu[i];
    }
    fp r = fp_from_w(v);  // y^-1 (plain, canonical) for y = the Montgomery integer x R
    fp r3;
    {
        const uint32_t c[NL] = BLS_R3;
        for (int j = 0; j < NL; j++) r3.l[j] = c[j];
    }
    return fp_mul(r, r3);  // y^-1 R^3 / R = (x R)^-1 R^2 = x^-1 R: the Montgomery form of x^-1
}
NWV_HD fp fp_inv_vt(const fp& x) { return fp_inv_vt_t<false>(x); }
NWV_HD fp fp_inv_vt_uniform(const fp& x) { return fp_inv_vt_t<true>(x); }

// The same inversion with a batch's four 12-word updates as independent rows: row r (0..3) applies
// the matrix row r & 1 to (a, b) (r < 2: exact, / 2^30, made non-negative) or to (u, v) (r >= 2:
// / 2^30 mod p), each with the batch's own coefficients; a negative (a, b) row then negates its
// (u, v) row mod p (fp_inv_vt_t negates the coefficients first: the same value).  On the device the
// rows run on four lanes at once (fp_inv_wave); inv_rows is the host form, one row after another.
NWV_HD bool inv_row(int r, int64_t f0, int64_t g0, int64_t f1, int64_t g1, const uint32_t* a, const uint32_t* b,
                    const uint32_t* u, const uint32_t* v, const uint32_t* P, uint32_t* o) {
    const bool row1 = (r & 1) != 0, uv = (r & 2) != 0;
    const int64_t F = row1 ? f1 : f0, G = row1 ? g1 : g0;
    if (uv) {
        w_lin2_modp(o, F, u, G, v, P);
        return false;
    }
    uint32_t t[BW + 1];
    w_lin2(t, F, a, G, b);
    const bool neg = w_neg13(t);
    w_shr30(o, t);
    return neg;
}
// o <- p - o unless o = 0 (o in [0, p))
NWV_HD void w_negp(uint32_t* o, const uint32_t* P) {
    if (w_is_zero(o)) return;
    int64_t c = 0;
    for (int i = 0; i < BW; i++) {
        c += (int64_t)P[i] - (int64_t)o[i];
        o[i] = (uint32_t)c;
        c >>= 32;
    }
}
// the batch's 30 divsteps on the approximations of a and b -> the matrix [f0 g0; f1 g1]
NWV_HD void inv_divsteps(const uint32_t* a, const uint32_t* b, int64_t& f0o, int64_t& g0o, int64_t& f1o,
                         int64_t& g1o) {
    int n = w_bitlen(a);
    const int nb = w_bitlen(b);
    n = n > nb ? n : nb;
    n = n > 62 ? n : 62;
    uint64_t xa = ((uint64_t)w_bits32(a, n - 32) << 30) | (a[0] & ((1u << 30) - 1u));
    uint64_t xb = ((uint64_t)w_bits32(b, n - 32) << 30) | (b[0] & ((1u << 30) - 1u));
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll
    for (int i = 0; i < 30; i++) {
        const bool odd = (xa & 1) != 0;
        const bool sw = odd && xa < xb;
        const uint64_t ya = sw ? xb : xa, yb = sw ? xa : xb;
        const int32_t h0 = sw ? f1 : f0, h1 = sw ? f0 : f1, k0 = sw ? g1 : g0, k1 = sw ? g0 : g1;
        xa = odd ? ya - yb : ya;
        xb = yb;
        f0 = odd ? h0 - h1 : h0;
        g0 = odd ? k0 - k1 : k0;
        f1 = h1;
        g1 = k1;
        xa >>= 1;
        f1 *= 2;
        g1 *= 2;
    }
    f0o = f0;
    g0o = g0;
    f1o = f1;
    g1o = g1;
}
NWV_HD fp inv_finish(const uint32_t* v) {
    const fp r = fp_from_w(v);
    fp r3;
    {
        const uint32_t c[NL] = BLS_R3;
        for (int j = 0; j < NL; j++) r3.l[j] = c[j];
    }
    return fp_mul(r, r3);
}
inline fp inv_rows(const fp& x) {
    const fp xc = fp_canon(x);
    if (fp_is_zero(xc)) return fp_zero();
    uint32_t a[BW], b[BW], u[BW], v[BW], P[BW];
    w_from_fp(a, xc);
    w_from_fp(P, k_p());
    for (int i = 0; i < BW; i++) {
        b[i] = P[i];
        u[i] = v[i] = 0;
    }
    u[0] = 1;
    for (int it = 0; it < 64 && !w_is_zero(a); it++) {
        int64_t f0, g0, f1, g1;
        inv_divsteps(a, b, f0, g0, f1, g1);
        uint32_t o[4][BW];
        bool neg[4];
        for (int r = 0; r < 4; r++) neg[r] = inv_row(r, f0, g0, f1, g1, a, b, u, v, P, o[r]);
        for (int r = 2; r < 4; r++)
            if (neg[r - 2]) w_negp(o[r], P);
        for (int i = 0; i < BW; i++) {
            a[i] = o[0][i];
            b[i] = o[1][i];
            u[i] = o[2][i];
            v[i] = o[3][i];
        }
    }
    return inv_finish(v);
}
#if defined(__HIP_DEVICE_COMPILE__) || (defined(__HIPCC__) && !defined(BLS_GROUP_HOST_EMU))
// every lane of the wave calls it with the same x: each lane runs the divsteps (uniform), lanes
// 0..3 (and their copies r = lane & 3) compute the four rows at once, then read them back from
// lanes 0..3
__device__ __attribute__((noinline)) fp fp_inv_wave(const fp& x) {
    const int r = (int)(threadIdx.x & 3);
    fp xu;
    for (int j = 0; j < NL; j++) xu.l[j] = __builtin_amdgcn_readfirstlane(x.l[j]);
    const fp xc = fp_canon(xu);
    if (fp_is_zero(xc)) return fp_zero();
    uint32_t a[BW], b[BW], u[BW], v[BW], P[BW];
    w_from_fp(a, xc);
    w_from_fp(P, k_p());
    for (int i = 0; i < BW; i++) {
        b[i] = P[i];
        u[i] = v[i] = 0;
    }
    u[0] = 1;
    for (int it = 0; it < 64 && !w_is_zero(a); it++) {
        int64_t f0, g0, f1, g1;
        inv_divsteps(a, b, f0, g0, f1, g1);
        uint32_t o[BW];
        const bool neg = inv_row(r, f0, g0, f1, g1, a, b, u, v, P, o);
        const int negs = (int)__builtin_amdgcn_readfirstlane(__ballot(neg) & 3u);  // rows 0, 1
        if (r >= 2 && ((negs >> (r - 2)) & 1)) w_negp(o, P);
        for (int i = 0; i < BW; i++) {
            a[i] = __builtin_amdgcn_readlane(o[i], 0);
            b[i] = __builtin_amdgcn_readlane(o[i], 1);
            u[i] = __builtin_amdgcn_readlane(o[i], 2);
            v[i] = __builtin_amdgcn_readlane(o[i], 3);
        }
    }
    return inv_finish(v);
}
#endif

// sqrt for p = 3 mod 4; false if a is not a square
NWV_HD bool fp_sqrt(fp& r, const fp& a) {
    const uint32_t e[12] = BLS_E_SQRT;
    const fp s = fp_pow(a, e);
    r = s;
    return fp_eq(fp_sqr(s), a);
}
// plain (non-Montgomery) canonical limbs <-> 48 big-endian bytes, through twelve 32-bit words
// (w[0] least significant); every index is a compile-time constant after unrolling, so nothing is
// staged in private memory.  mask0 is applied to the first (most significant) byte -- the ZCash
// flag bits of a compressed point.
NWV_HD void plain_from_be(fp& r, const uint8_t* b, uint32_t mask0 = 0xff) {
    uint32_t w[13];
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const uint8_t* q = b + 44 - 4 * k;
        w[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
    w[11] &= (mask0 << 24) | 0xffffffu;
    w[12] = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const int bit = 28 * j, idx = bit >> 5, sh = bit & 31;
        uint32_t v = w[idx] >> sh;
        if (sh > 4) v |= w[idx + 1] << (32 - sh);
        r.l[j] = v & LM;
    }
}
// 32 big-endian bytes -> limbs (< 2^256)
NWV_HD void plain_from_be256(fp& r, const uint8_t* b) {
    uint32_t w[9];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint8_t* q = b + 28 - 4 * k;
        w[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
    w[8] = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const int bit = 28 * j, idx = bit >> 5, sh = bit & 31;
        uint32_t v = idx < 9 ? w[idx] >> sh : 0;
        if (sh > 4 && idx + 1 < 9) v |= w[idx + 1] << (32 - sh);
        r.l[j] = v & LM;
    }
}
NWV_HD void plain_to_be(uint8_t* b, const fp& a) {
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const int bit = 32 * k, j = bit / 28, sh = bit % 28;
        uint32_t v = a.l[j] >> sh;
        if (j + 1 < NL) v |= a.l[j + 1] << (28 - sh);
        if (sh > 24 && j + 2 < NL) v |= a.l[j + 2] << (56 - sh);
        uint8_t* q = b + 44 - 4 * k;
        q[0] = (uint8_t)(v >> 24);
        q[1] = (uint8_t)(v >> 16);
        q[2] = (uint8_t)(v >> 8);
        q[3] = (uint8_t)v;
    }
}
NWV_HD bool plain_lt_p(const fp& a) {
    fp t;
    return limb_sub(t, a, k_p()) != 0;
}
// canonical y > (p-1)/2  <=>  2y > p - 1  <=>  2y >= p + 1 > p (y canonical, y != (p-1)/2 ... )
NWV_HD bool fp_lex_large(const fp& a) {
    const fp c = fp_from_mont(a);
    fp d;
    limb_add(d, c, c);  // 2y < 2p, limbs normalised
    fp t;
    return limb_sub(t, d, k_p()) == 0;  // 2y >= p  <=>  y > (p-1)/2 (2y is even, p odd)
}
NWV_HD uint32_t fp_sgn0(const fp& a) { return fp_from_mont(a).l[0] & 1; }

// ----------------------------------------------------------------------------------- Fp2
NWV_HD fp2 f2_zero() { fp2 r = {fp_zero(), fp_zero()}; return r; }
NWV_HD fp2 f2_one() { fp2 r = {k_one(), fp_zero()}; return r; }
NWV_HD fp2 f2_add(const fp2& a, const fp2& b) { fp2 r = {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; return r; }
NWV_HD fp2 f2_sub(const fp2& a, const fp2& b) { fp2 r = {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; return r; }
NWV_HD fp2 f2_neg(const fp2& a) { fp2 r = {fp_neg(a.c0), fp_neg(a.c1)}; return r; }
NWV_HD fp2 f2_dbl(const fp2& a) { return f2_add(a, a); }
NWV_HD fp2 f2_conj(const fp2& a) { fp2 r = {a.c0, fp_neg(a.c1)}; return r; }
BLS_HD fp2 f2_mul(const fp2& a, const fp2& b) {
    const fp t0 = fp_mul(a.c0, b.c0), t1 = fp_mul(a.c1, b.c1);
    const fp m = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
    fp2 r = {fp_sub(t0, t1), fp_sub(fp_sub(m, t0), t1)};
    return r;
}
BLS_HD fp2 f2_sqr(const fp2& a) {
    const fp m = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
    const fp t = fp_mul(a.c0, a.c1);
    fp2 r = {m, fp_dbl(t)};
    return r;
}
NWV_HD fp2 f2_mul_fp(const fp2& a, const fp& b) { fp2 r = {fp_mul(a.c0, b), fp_mul(a.c1, b)}; return r; }
NWV_HD fp2 f2_mul_xi(const fp2& a) { fp2 r = {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; return r; }
NWV_HD bool f2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
NWV_HD bool f2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
NWV_HD fp2 f2_inv(const fp2& a) {
    const fp n = fp_inv(fp_add(fp_sqr(a.c0), fp_sqr(a.c1)));
    fp2 r = {fp_mul(a.c0, n), fp_neg(fp_mul(a.c1, n))};
    return r;
}
BLS_NOINLINE fp2 f2_pow(const fp2& a, const uint32_t* e) {
    fp2 acc = f2_one();
    bool started = false;
    for (int w = 11; w >= 0; w--)
        for (int b = 31; b >= 0; b--) {
            if (started) acc = f2_sqr(acc);
            if ((e[w] >> b) & 1) {
                acc = started ? f2_mul(acc, a) : a;
                started = true;
            }
        }
    return acc;
}
// square root in Fp2 for p = 3 mod 4 (Adj, Rodriguez-Henriquez, eprint 2012/685 Alg. 9)
NWV_HD bool f2_sqrt(fp2& r, const fp2& a) {
    const uint32_t eq[12] = BLS_E_QR, eh[12] = BLS_E_HALF;
    const fp2 a1 = f2_pow(a, eq);
    const fp2 alpha = f2_mul(f2_sqr(a1), a);
    const fp2 x0 = f2_mul(a1, a);
    const fp2 a0 = f2_mul(f2_conj(alpha), alpha);
    const fp2 m1 = f2_neg(f2_one());
    fp2 x;
    if (f2_eq(alpha, m1)) {
        x.c0 = fp_neg(x0.c1);
        x.c1 = x0.c0;
    } else {
        x = f2_mul(f2_pow(f2_add(alpha, f2_one()), eh), x0);
    }
    r = x;
    return !f2_eq(a0, m1) && f2_eq(f2_sqr(x), a);
}
NWV_HD bool f2_lex_large(const fp2& a) { return fp_is_zero(a.c1) ? fp_lex_large(a.c0) : fp_lex_large(a.c1); }

// ----------------------------------------------------------------------------- Fp6, Fp12
NWV_HD fp6 f6_add(const fp6& a, const fp6& b) { fp6 r = {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; return r; }
NWV_HD fp6 f6_sub(const fp6& a, const fp6& b) { fp6 r = {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; return r; }
NWV_HD fp6 f6_neg(const fp6& a) { fp6 r = {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; return r; }
NWV_HD fp6 f6_mul_v(const fp6& a) { fp6 r = {f2_mul_xi(a.c2), a.c0, a.c1}; return r; }
BLS_HD fp6 f6_mul(const fp6& a, const fp6& b) {
    const fp2 t0 = f2_mul(a.c0, b.c0), t1 = f2_mul(a.c1, b.c1), t2 = f2_mul(a.c2, b.c2);
    fp6 r;
    r.c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), t1), t2)));
    r.c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), t0), t1), f2_mul_xi(t2));
    r.c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), t0), t2), t1);
    return r;
}
// a * (b0 + b1 v)
BLS_HD fp6 f6_mul_01(const fp6& a, const fp2& b0, const fp2& b1) {
    const fp2 aa = f2_mul(a.c0, b0), bb = f2_mul(a.c1, b1);
    fp6 r;
    r.c0 = f2_add(f2_mul_xi(f2_mul(a.c2, b1)), aa);
    r.c1 = f2_sub(f2_sub(f2_mul(f2_add(b0, b1), f2_add(a.c0, a.c1)), aa), bb);
    r.c2 = f2_add(f2_mul(a.c2, b0), bb);
    return r;
}
// a * (b1 v)
NWV_HD fp6 f6_mul_1(const fp6& a, const fp2& b1) {
    fp6 r = {f2_mul_xi(f2_mul(a.c2, b1)), f2_mul(a.c0, b1), f2_mul(a.c1, b1)};
    return r;
}
NWV_HD fp6 f6_inv(const fp6& a) {
    const fp2 A = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
    const fp2 B = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
    const fp2 C = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
    const fp2 F = f2_inv(f2_add(f2_mul(a.c0, A), f2_mul_xi(f2_add(f2_mul(a.c2, B), f2_mul(a.c1, C)))));
    fp6 r = {f2_mul(A, F), f2_mul(B, F), f2_mul(C, F)};
    return r;
}
NWV_HD fp12 f12_one() { fp12 r; r.c0.c0 = f2_one(); r.c0.c1 = r.c0.c2 = r.c1.c0 = r.c1.c1 = r.c1.c2 = f2_zero(); return r; }
BLS_HD fp12 f12_mul(const fp12& a, const fp12& b) {
    const fp6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
    fp12 r;
    r.c1 = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
    r.c0 = f6_add(t0, f6_mul_v(t1));
    return r;
}
// (a0 + a1 w)^2 = (a0 + a1)(a0 + v a1) - t - v t + 2 t w, t = a0 a1
BLS_HD fp12 f12_sqr(const fp12& a) {
    const fp6 t = f6_mul(a.c0, a.c1);
    const fp6 m = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
    fp12 r;
    r.c0 = f6_sub(f6_sub(m, t), f6_mul_v(t));
    r.c1 = f6_add(t, t);
    return r;
}
NWV_HD fp12 f12_conj(const fp12& a) { fp12 r = {a.c0, f6_neg(a.c1)}; return r; }
NWV_HD fp12 f12_inv(const fp12& a) {
    const fp6 t = f6_inv(f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1))));
    fp12 r = {f6_mul(a.c0, t), f6_neg(f6_mul(a.c1, t))};
    return r;
}
// sparse product by the line c0 + c1 v + c4 v w (slots c0.c0, c0.c1, c1.c1)
BLS_HD fp12 f12_mul_014(const fp12& a, const fp2& c0, const fp2& c1, const fp2& c4) {
    const fp6 aa = f6_mul_01(a.c0, c0, c1);
    const fp6 bb = f6_mul_1(a.c1, c4);
    fp12 r;
    r.c1 = f6_sub(f6_sub(f6_mul_01(f6_add(a.c1, a.c0), c0, f2_add(c1, c4)), aa), bb);
    r.c0 = f6_add(f6_mul_v(bb), aa);
    return r;
}
// Frobenius a^p: w-basis coefficient k (w^(2i) -> c0.ci, w^(2i+1) -> c1.ci) -> conj(a_k) GAMMA[k]
NWV_HD fp2 gamma_k(int k) {
    const uint32_t g[6][2][NL] = BLS_GAMMA;
    fp2 r;
    for (int j = 0; j < NL; j++) {
        r.c0.l[j] = g[k][0][j];
        r.c1.l[j] = g[k][1][j];
    }
    return r;
}
NWV_HD fp12 f12_frob(const fp12& a) {
    fp12 r;
    r.c0.c0 = f2_conj(a.c0.c0);
    r.c1.c0 = f2_mul(f2_conj(a.c1.c0), gamma_k(1));
    r.c0.c1 = f2_mul(f2_conj(a.c0.c1), gamma_k(2));
    r.c1.c1 = f2_mul(f2_conj(a.c1.c1), gamma_k(3));
    r.c0.c2 = f2_mul(f2_conj(a.c0.c2), gamma_k(4));
    r.c1.c2 = f2_mul(f2_conj(a.c1.c2), gamma_k(5));
    return r;
}
NWV_HD bool f12_is_one(const fp12& a) {
    return f2_eq(a.c0.c0, f2_one()) && f2_is_zero(a.c0.c1) && f2_is_zero(a.c0.c2) && f2_is_zero(a.c1.c0) &&
           f2_is_zero(a.c1.c1) && f2_is_zero(a.c1.c2);
}
// Granger-Scott squaring in the cyclotomic subgroup (eprint 2009/565 §3.2): Fp12 as Fp4^3 over
// (z0, z4, z3, z2, z1, z5) = (c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2)
NWV_HD void fp4_sqr(fp2& o0, fp2& o1, const fp2& a, const fp2& b) {
    const fp2 t0 = f2_sqr(a), t1 = f2_sqr(b);
    o0 = f2_add(f2_mul_xi(t1), t0);
    o1 = f2_sub(f2_sub(f2_sqr(f2_add(a, b)), t0), t1);
}
BLS_HD fp12 f12_cyc_sqr(const fp12& f) {
    fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
    fp2 t0, t1, t2, t3;
    fp4_sqr(t0, t1, z0, z1);
    z0 = f2_add(f2_dbl(f2_sub(t0, z0)), t0);
    z1 = f2_add(f2_dbl(f2_add(t1, z1)), t1);
    fp4_sqr(t0, t1, z2, z3);
    fp4_sqr(t2, t3, z4, z5);
    z4 = f2_add(f2_dbl(f2_sub(t0, z4)), t0);
    z5 = f2_add(f2_dbl(f2_add(t1, z5)), t1);
    t0 = f2_mul_xi(t3);
    z2 = f2_add(f2_dbl(f2_add(t0, z2)), t0);
    z3 = f2_add(f2_dbl(f2_sub(t2, z3)), t2);
    fp12 r;
    r.c0.c0 = z0; r.c0.c1 = z4; r.c0.c2 = z3;
    r.c1.c0 = z2; r.c1.c1 = z1; r.c1.c2 = z5;
    return r;
}
// f^x (x = -BLS_X_ABS) for f in the cyclotomic subgroup
BLS_NOINLINE fp12 f12_cyc_exp_x(const fp12& f) {
    fp12 acc = f;
    for (int b = 62; b >= 0; b--) {
        acc = f12_cyc_sqr(acc);
        if ((BLS_X_ABS >> b) & 1) acc = f12_mul(acc, f);
    }
    return f12_conj(acc);
}
// f^(3 (p^12 - 1) / r)
BLS_NOINLINE fp12 final_exp(const fp12& f) {
    fp12 m = f12_mul(f12_conj(f), f12_inv(f));  // f^(p^6 - 1)
    m = f12_mul(f12_frob(f12_frob(m)), m);       // ^(p^2 + 1)
    fp12 a = f12_mul(f12_cyc_exp_x(m), f12_conj(m));  // m^(x-1)
    a = f12_mul(f12_cyc_exp_x(a), f12_conj(a));       // m^((x-1)^2)
    const fp12 b = f12_mul(f12_cyc_exp_x(a), f12_frob(a));  // a^(x+p)
    fp12 c = f12_cyc_exp_x(f12_cyc_exp_x(b));
    c = f12_mul(f12_mul(c, f12_frob(f12_frob(b))), f12_conj(b));  // b^(x^2+p^2-1)
    return f12_mul(c, f12_mul(f12_cyc_sqr(m), m));
}

// --------------------------------------------------------------------------------- G1 / G2
template <class F> struct ops;
template <> struct ops<fp> {
    NWV_HD static fp add(const fp& a, const fp& b) { return fp_add(a, b); }
    NWV_HD static fp sub(const fp& a, const fp& b) { return fp_sub(a, b); }
    NWV_HD static fp mul(const fp& a, const fp& b) { return fp_mul(a, b); }
    NWV_HD static fp sqr(const fp& a) { return fp_sqr(a); }
    NWV_HD static bool is_zero(const fp& a) { return fp_is_zero(a); }
    NWV_HD static bool eq(const fp& a, const fp& b) { return fp_eq(a, b); }
    NWV_HD static fp one() { return k_one(); }
};
template <> struct ops<fp2> {
    NWV_HD static fp2 add(const fp2& a, const fp2& b) { return f2_add(a, b); }
    NWV_HD static fp2 sub(const fp2& a, const fp2& b) { return f2_sub(a, b); }
    NWV_HD static fp2 mul(const fp2& a, const fp2& b) { return f2_mul(a, b); }
    NWV_HD static fp2 sqr(const fp2& a) { return f2_sqr(a); }
    NWV_HD static bool is_zero(const fp2& a) { return f2_is_zero(a); }
    NWV_HD static bool eq(const fp2& a, const fp2& b) { return f2_eq(a, b); }
    NWV_HD static fp2 one() { return f2_one(); }
};
template <class F> struct jac { F x, y, z; bool inf; };

// doubling (dbl-2009-l, a = 0)
template <class F> BLS_HD jac<F> jac_dbl(const jac<F>& a) {
    using O = ops<F>;
    jac<F> o;
    o.inf = a.inf || O::is_zero(a.y);
    const F A = O::sqr(a.x), B = O::sqr(a.y), C = O::sqr(B);
    const F t = O::sub(O::sub(O::sqr(O::add(a.x, B)), A), C);
    const F D = O::add(t, t);
    const F E = O::add(O::add(A, A), A);
    const F Fv = O::sqr(E);
    o.x = O::sub(O::sub(Fv, D), D);
    const F yz = O::mul(a.y, a.z);
    o.z = O::add(yz, yz);
    F c8 = O::add(C, C);
    c8 = O::add(c8, c8);
    c8 = O::add(c8, c8);
    o.y = O::sub(O::mul(E, O::sub(D, o.x)), c8);
    return o;
}
// general addition (add-2007-bl) with the exceptional cases
template <class F> BLS_NOINLINE jac<F> jac_add(const jac<F>& a, const jac<F>& b) {
    using O = ops<F>;
    if (a.inf) return b;
    if (b.inf) return a;
    const F z1z1 = O::sqr(a.z), z2z2 = O::sqr(b.z);
    const F u1 = O::mul(a.x, z2z2), u2 = O::mul(b.x, z1z1);
    const F s1 = O::mul(O::mul(a.y, b.z), z2z2), s2 = O::mul(O::mul(b.y, a.z), z1z1);
    if (O::eq(u1, u2)) {
        if (O::eq(s1, s2)) return jac_dbl(a);
        jac<F> o = a;
        o.inf = true;
        return o;
    }
    const F h = O::sub(u2, u1);
    F i = O::add(h, h);
    i = O::sqr(i);
    const F j = O::mul(h, i);
    F rr = O::sub(s2, s1);
    rr = O::add(rr, rr);
    const F v = O::mul(u1, i);
    jac<F> o;
    o.inf = false;
    o.x = O::sub(O::sub(O::sub(O::sqr(rr), j), v), v);
    const F sj = O::mul(s1, j);
    o.y = O::sub(O::mul(rr, O::sub(v, o.x)), O::add(sj, sj));
    o.z = O::mul(O::sub(O::sub(O::sqr(O::add(a.z, b.z)), z1z1), z2z2), h);
    return o;
}
template <class F> NWV_HD jac<F> jac_from_affine(const F& x, const F& y) {
    jac<F> o;
    o.x = x;
    o.y = y;
    o.z = ops<F>::one();
    o.inf = false;
    return o;
}
// [k] a for a 64-bit scalar (double-and-add, MSB first)
template <class F> BLS_NOINLINE jac<F> jac_mul64(const jac<F>& a, uint64_t k) {
    jac<F> acc = a;
    acc.inf = true;
    for (int b = 63; b >= 0; b--) {
        if (!acc.inf) acc = jac_dbl(acc);
        if ((k >> b) & 1) acc = jac_add(acc, a);
    }
    return acc;
}
// [k] a for a big-endian scalar of nb bytes (key generation and signing of synthetic workloads)
template <class F> BLS_NOINLINE jac<F> jac_mul_be(const jac<F>& a, const uint8_t* k, int nb) {
    jac<F> acc = a;
    acc.inf = true;
    for (int i = 0; i < nb; i++)
        for (int b = 7; b >= 0; b--) {
            if (!acc.inf) acc = jac_dbl(acc);
            if ((k[i] >> b) & 1) acc = jac_add(acc, a);
        }
    return acc;
}
// Jacobian (X, Y, Z) == affine (x, y)?
template <class F> NWV_HD bool jac_eq_affine(const jac<F>& a, const F& x, const F& y) {
    using O = ops<F>;
    if (a.inf) return false;
    const F z2 = O::sqr(a.z);
    return O::eq(a.x, O::mul(x, z2)) && O::eq(a.y, O::mul(y, O::mul(z2, a.z)));
}
NWV_HD void g1_to_affine(fp& x, fp& y, const jac<fp>& a) {
    const fp zi = fp_inv(a.z), zi2 = fp_sqr(zi);
    x = fp_mul(a.x, zi2);
    y = fp_mul(a.y, fp_mul(zi2, zi));
}
NWV_HD void g2_to_affine(fp2& x, fp2& y, const jac<fp2>& a) {
    const fp2 zi = f2_inv(a.z), zi2 = f2_sqr(zi);
    x = f2_mul(a.x, zi2);
    y = f2_mul(a.y, f2_mul(zi2, zi));
}
// the same for public points (verification, aggregation, keys): the variable-time inversion
NWV_HD void g1_to_affine_vt(fp& x, fp& y, const jac<fp>& a) {
    const fp zi = fp_inv_vt(a.z), zi2 = fp_sqr(zi);
    x = fp_mul(a.x, zi2);
    y = fp_mul(a.y, fp_mul(zi2, zi));
}
NWV_HD void g2_to_affine_vt(fp2& x, fp2& y, const jac<fp2>& a) {
    const fp n = fp_inv_vt(fp_add(fp_sqr(a.z.c0), fp_sqr(a.z.c1)));
    const fp2 zi = {fp_mul(a.z.c0, n), fp_neg(fp_mul(a.z.c1, n))}, zi2 = f2_sqr(zi);
    x = f2_mul(a.x, zi2);
    y = f2_mul(a.y, f2_mul(zi2, zi));
}
// P (affine, on the curve) in G1  <=>  phi(P) = (beta x, y) = [-x^2] P
NWV_HD bool g1_in_group(const fp& x, const fp& y) {
    const jac<fp> P = jac_from_affine(x, y);
    const jac<fp> t = jac_mul64(jac_mul64(P, BLS_X_ABS), BLS_X_ABS);  // [x^2] P
    return jac_eq_affine(t, fp_mul(x, k_beta()), fp_neg(y));          // [x^2] P = -phi(P)
}
// Q (affine, on the twist) in G2  <=>  psi(Q) = [x] Q = -[|x|] Q
NWV_HD bool g2_in_group(const fp2& x, const fp2& y) {
    const jac<fp2> Q = jac_from_affine(x, y);
    const jac<fp2> t = jac_mul64(Q, BLS_X_ABS);
    const fp2 px = f2_mul(f2_conj(x), k_psi_cx()), py = f2_mul(f2_conj(y), k_psi_cy());
    return jac_eq_affine(t, px, f2_neg(py));
}

// status codes (= blst BLST_ERROR subset, the oracle's ORB_* codes)
enum : int32_t { ST_OK = 0, ST_BAD_ENCODING = 1, ST_NOT_ON_CURVE = 2, ST_NOT_IN_GROUP = 3, ST_AGGR_MISMATCH = 4,
                 ST_VERIFY_FAIL = 5, ST_PK_INFINITY = 6 };

// ZCash compressed G1 (48 bytes) -> affine; *inf for the identity
NWV_HD int32_t g1_decompress(fp& x, fp& y, bool& inf, const uint8_t* in) {
    const uint8_t f = in[0];
    inf = false;
    if (!(f & 0x80)) return ST_BAD_ENCODING;
    if (f & 0x40) {
        uint32_t o = f & 0x3f;
        for (int i = 1; i < 48; i++) o |= in[i];
        inf = true;
        return o ? ST_BAD_ENCODING : ST_OK;
    }
    fp px;
    plain_from_be(px, in, 0x1f);
    if (!plain_lt_p(px)) return ST_BAD_ENCODING;
    x = fp_to_mont(px);
    const fp rhs = fp_add(fp_mul(fp_sqr(x), x), k_b1());
    if (!fp_sqrt(y, rhs)) return ST_NOT_ON_CURVE;
    if (fp_lex_large(y) != ((f & 0x20) != 0)) y = fp_neg(y);
    return ST_OK;
}
NWV_HD int32_t g2_decompress(fp2& x, fp2& y, bool& inf, const uint8_t* in) {
    const uint8_t f = in[0];
    inf = false;
    if (!(f & 0x80)) return ST_BAD_ENCODING;
    if (f & 0x40) {
        uint32_t o = f & 0x3f;
        for (int i = 1; i < 96; i++) o |= in[i];
        inf = true;
        return o ? ST_BAD_ENCODING : ST_OK;
    }
    fp p1, p0;
    plain_from_be(p1, in, 0x1f);
    plain_from_be(p0, in + 48);
    if (!plain_lt_p(p1) || !plain_lt_p(p0)) return ST_BAD_ENCODING;
    x.c0 = fp_to_mont(p0);
    x.c1 = fp_to_mont(p1);
    const fp2 rhs = f2_add(f2_mul(f2_sqr(x), x), k_b2());
    if (!f2_sqrt(y, rhs)) return ST_NOT_ON_CURVE;
    if (f2_lex_large(y) != ((f & 0x20) != 0)) y = f2_neg(y);
    return ST_OK;
}
NWV_HD void g1_compress(uint8_t* out, const fp& x, const fp& y, bool inf) {
    if (inf) {
        for (int i = 0; i < 48; i++) out[i] = 0;
        out[0] = 0xc0;
        return;
    }
    plain_to_be(out, fp_from_mont(x));
    out[0] |= 0x80 | (fp_lex_large(y) ? 0x20 : 0);
}
NWV_HD void g2_compress(uint8_t* out, const fp2& x, const fp2& y, bool inf) {
    if (inf) {
        for (int i = 0; i < 96; i++) out[i] = 0;
        out[0] = 0xc0;
        return;
    }
    plain_to_be(out, fp_from_mont(x.c1));
    plain_to_be(out + 48, fp_from_mont(x.c0));
    out[0] |= 0x80 | (f2_lex_large(y) ? 0x20 : 0);
}

// --------------------------------------------------------------------------------- SHA-256
struct sha256_state { uint32_t h[8]; };
NWV_HD uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
BLS_NOINLINE void sha256_block(uint32_t* h, const uint32_t* blk) {
    const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = blk[i];
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    // fully unrolled: the message schedule's indices and the round constants are compile-time
    // (a rolled loop indexes w[] dynamically, which puts it in scratch memory)
#pragma unroll
    for (int i = 0; i < 64; i++) {
        if (i >= 16) {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            w[i & 15] += (ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3)) + w[(i + 9) & 15] +
                         (ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10));
        }
        const uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i & 15];
        const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
// SHA-256 of (`prefix` bytes already absorbed into h) || a byte stream of `total` bytes given by
// byte(pos): words are assembled in registers (no byte arrays, whose dynamic indices would go to
// scratch memory); out8 = the digest as eight big-endian words
template <class B>
NWV_HD void sha256_stream(uint32_t* h, uint32_t prefix, uint32_t total, B byte, uint32_t* out8) {
    const uint64_t bits = (uint64_t)(prefix + total) * 8;
    const uint32_t nb = (total + 9 + 63) / 64;
    for (uint32_t blk = 0; blk < nb; blk++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t pos = 64 * blk + 4 * j + k;
                uint32_t b = 0;
                if (pos < total) b = byte(pos);
                else if (pos == total) b = 0x80u;
                else if (blk == nb - 1 && 4 * j + k >= 56) b = (uint32_t)(bits >> (8 * (63 - (4 * j + k)))) & 0xffu;
                v = (v << 8) | b;
            }
            w[j] = v;
        }
        sha256_block(h, w);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out8[i] = h[i];
}
NWV_HD void sha256_iv(uint32_t* h) {
    const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    for (int i = 0; i < 8; i++) h[i] = iv[i];
}
// byte k (< 32) of eight big-endian words, by selects (no dynamic register indexing)
NWV_HD uint32_t words_byte(const uint32_t* x, uint32_t k) {
    const uint32_t q = k >> 2;
    uint32_t v = x[0];
#pragma unroll
    for (int t = 1; t < 8; t++) v = q == (uint32_t)t ? x[t] : v;
    return (v >> (24 - 8 * (k & 3))) & 0xffu;
}

// ------------------------------------------------------------------- hash_to_curve (G1)
// expand_message_xmd (RFC 9380 §5.3.1), 128 output bytes as 32 big-endian words; the 64-byte zero
// block Z_pad is the first block of b_0's input: its compression is absorbed once per lane
NWV_HD void expand_xmd_128w(uint32_t* out, const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl) {
    uint32_t h[8];
    sha256_iv(h);
    const uint32_t zero[16] = {0};
    sha256_block(h, zero);
    uint32_t b0[8], bi[8];
    // b_0 = H(Z_pad || msg || I2OSP(128, 2) || I2OSP(0, 1) || DST || I2OSP(len(DST), 1))
    sha256_stream(h, 64, n + 3 + dl + 1,
                  [&](uint32_t k) -> uint32_t {
                      if (k < n) return msg[k];
                      k -= n;
                      if (k < 3) return k == 1 ? 128u : 0u;
                      k -= 3;
                      return k < dl ? (uint32_t)dst[k] : dl;
                  },
                  b0);
    for (int i = 1; i <= 4; i++) {
        // b_i = H((b_0 xor b_{i-1}) || I2OSP(i, 1) || DST || I2OSP(len(DST), 1))
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = i == 1 ? b0[k] : (b0[k] ^ bi[k]);
        sha256_iv(h);
        sha256_stream(h, 0, 33 + dl + 1,
                      [&](uint32_t k) -> uint32_t {
                          if (k < 32) return words_byte(x, k);
                          if (k == 32) return (uint32_t)i;
                          k -= 33;
                          return k < dl ? (uint32_t)dst[k] : dl;
                      },
                      bi);
#pragma unroll
        for (int k = 0; k < 8; k++) out[8 * (i - 1) + k] = bi[k];
    }
}
NWV_HD void expand_xmd_128(uint8_t* out, const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl) {
    uint32_t w[32];
    expand_xmd_128w(w, msg, n, dst, dl);
    for (int i = 0; i < 32; i++)
        for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(w[i] >> (24 - 8 * k));
}
// 256 bits from eight big-endian words, as plain limbs
NWV_HD fp plain_from_be256w(const uint32_t* w) {
    uint32_t le[8];
#pragma unroll
    for (int i = 0; i < 8; i++) le[i] = w[7 - i];
    fp r;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const int bit = 28 * j, idx = bit >> 5, sh = bit & 31;
        uint32_t v = idx < 8 ? le[idx] >> sh : 0u;
        if (sh > 4 && idx + 1 < 8) v |= le[idx + 1] << (32 - sh);
        r.l[j] = v & LM;
    }
    return r;
}
// 16 big-endian words (64 bytes) mod p, Montgomery form: hi * 2^256 + lo
NWV_HD fp fp_from_be64w(const uint32_t* w) {
    return fp_add(fp_mul(fp_to_mont(plain_from_be256w(w)), k_two256()), fp_to_mont(plain_from_be256w(w + 8)));
}
// 64 big-endian bytes mod p, Montgomery form: hi * 2^256 + lo
NWV_HD fp fp_from_be64(const uint8_t* b) {
    fp h, l;
    plain_from_be256(h, b);
    plain_from_be256(l, b + 32);
    return fp_add(fp_mul(fp_to_mont(h), k_two256()), fp_to_mont(l));
}
// simplified SWU on y^2 = x^3 + A'x + B' (RFC 9380 §6.6.2, Z = 11), the straight-line form of
// Appendix F.2 with sqrt_ratio for q = 3 mod 4 (F.2.1.2): one exponentiation and one inversion
// per call (the textbook form's inversions of A and tv1 and its second square root are gone)
// the same map with x left as the fraction xn / xd (no inversion: the wave engine takes the
// isogeny map in homogeneous coordinates)
NWV_HD void map_sswu_frac(fp& xn_o, fp& xd_o, fp& yo, const fp& u);
NWV_HD void map_sswu(fp& xo, fp& yo, const fp& u) {
    fp xn, xd;
    map_sswu_frac(xn, xd, yo, u);
    xo = fp_mul(xn, fp_inv(xd));
}
NWV_HD void map_sswu_frac(fp& xn_o, fp& xd_o, fp& yo, const fp& u) {
    const fp A = k_sswu_a(), B = k_sswu_b(), Z = k_sswu_z();
    const fp tv1 = fp_mul(Z, fp_sqr(u));
    fp tv2 = fp_add(fp_sqr(tv1), tv1);
    const fp tv3 = fp_mul(B, fp_add(tv2, k_one()));
    const fp tv4 = fp_mul(A, fp_is_zero(tv2) ? Z : fp_neg(tv2));
    fp tv6 = fp_sqr(tv4);
    tv2 = fp_mul(fp_add(fp_sqr(tv3), fp_mul(A, tv6)), tv3);
    tv6 = fp_mul(tv6, tv4);
    tv2 = fp_add(tv2, fp_mul(B, tv6));  // gx1 = tv2 / tv6
    const fp xn = fp_mul(tv1, tv3);
    // sqrt_ratio(tv2, tv6)
    const uint32_t c1[12] = BLS_E_QR;  // (p - 3) / 4
    const fp s1 = fp_mul(fp_sqr(tv6), fp_mul(tv2, tv6));
    fp y1 = fp_mul(fp_pow(s1, c1), fp_mul(tv2, tv6));
    const fp y2 = fp_mul(y1, k_sswu_c2());
    const bool qr = fp_eq(fp_mul(fp_sqr(y1), tv6), tv2);
    y1 = qr ? y1 : y2;
    fp y = qr ? y1 : fp_mul(fp_mul(tv1, u), y1);
    const fp x = qr ? tv3 : xn;
    if (fp_sgn0(u) != fp_sgn0(y)) y = fp_neg(y);
    xn_o = x;
    xd_o = tv4;
    yo = y;
}
// the 11-isogeny (RFC 9380 Appendix E.2), constants from tools/gen_bls_iso.py
NWV_HD fp iso_poly(const uint32_t (*c)[NL], int n, bool monic, const fp& x) {
    fp acc;
    int top;
    if (monic) {
        acc = k_one();
        top = n - 1;
    } else {
        for (int j = 0; j < NL; j++) acc.l[j] = c[n - 1][j];
        top = n - 2;
    }
    for (int i = top; i >= 0; i--) {
        fp ci;
        for (int j = 0; j < NL; j++) ci.l[j] = c[i][j];
        acc = fp_add(fp_mul(acc, x), ci);
    }
    return acc;
}
NWV_HD jac<fp> iso_map(const fp& x, const fp& y) {
    const uint32_t xn[BLS_ISO_XNUM_LEN][NL] = BLS_ISO_XNUM, xd[BLS_ISO_XDEN_LEN][NL] = BLS_ISO_XDEN;
    const uint32_t yn[BLS_ISO_YNUM_LEN][NL] = BLS_ISO_YNUM, yd[BLS_ISO_YDEN_LEN][NL] = BLS_ISO_YDEN;
    const fp Xn = iso_poly(xn, BLS_ISO_XNUM_LEN, false, x), Xd = iso_poly(xd, BLS_ISO_XDEN_LEN, true, x);
    const fp Yn = fp_mul(iso_poly(yn, BLS_ISO_YNUM_LEN, false, x), y), Yd = iso_poly(yd, BLS_ISO_YDEN_LEN, true, x);
    // affine (Xn/Xd, Yn/Yd) as Jacobian with Z = Xd Yd: X = Xn Xd Yd^2, Y = Yn Yd^2 Xd^3
    jac<fp> o;
    o.inf = false;
    o.z = fp_mul(Xd, Yd);
    o.x = fp_mul(Xn, fp_mul(o.z, Yd));                   // Xn/Xd * Z^2 = Xn Xd Yd^2
    o.y = fp_mul(fp_mul(Yn, o.z), fp_mul(o.z, Xd));      // Yn/Yd * Z^3 = Yn Xd^3 Yd^2
    return o;
}
// one of the two field elements of hash_to_field (j = 0, 1) mapped to E: iso(SSWU(u_j))
BLS_NOINLINE jac<fp> h2c_map(const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl, int j) {
    uint32_t uw[32];
    expand_xmd_128w(uw, msg, n, dst, dl);
    const fp u0 = fp_from_be64w(uw), u1 = fp_from_be64w(uw + 16);  // constant offsets, then a select
    fp x, y;
    map_sswu(x, y, fp_sel(j == 0, u0, u1));
    return iso_map(x, y);
}
// H(m) in Jacobian form
BLS_NOINLINE jac<fp> hash_to_g1(const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl) {
    const jac<fp> q0 = h2c_map(msg, n, dst, dl, 0), q1 = h2c_map(msg, n, dst, dl, 1);
    return jac_mul64(jac_add(q0, q1), BLS_H_EFF);
}

// --------------------------------------------------------------------------------- pairing
// Miller-loop steps on the M-type twist; lines l0 + l1 x_P v + l4 y_P v w (eprint 2010/354)
BLS_HD void ml_dbl(jac<fp2>& T, fp2& l0, fp2& l1, fp2& l4) {
    const fp2 t0 = f2_sqr(T.x), t1 = f2_sqr(T.y), t2 = f2_sqr(t1);
    fp2 t3 = f2_sub(f2_sub(f2_sqr(f2_add(t1, T.x)), t0), t2);
    t3 = f2_dbl(t3);
    const fp2 t4 = f2_add(f2_dbl(t0), t0);
    const fp2 t6 = f2_add(T.x, t4);
    const fp2 t5 = f2_sqr(t4);
    const fp2 zz = f2_sqr(T.z);
    T.x = f2_sub(f2_sub(t5, t3), t3);
    T.z = f2_sub(f2_sub(f2_sqr(f2_add(T.z, T.y)), t1), zz);
    fp2 t2x8 = f2_dbl(f2_dbl(f2_dbl(t2)));
    T.y = f2_sub(f2_mul(f2_sub(t3, T.x), t4), t2x8);
    l1 = f2_neg(f2_dbl(f2_mul(t4, zz)));
    l0 = f2_sub(f2_sub(f2_sub(f2_sqr(t6), t0), t5), f2_dbl(f2_dbl(t1)));
    l4 = f2_dbl(f2_mul(T.z, zz));
}
BLS_HD void ml_add(jac<fp2>& T, const fp2& qx, const fp2& qy, fp2& l0, fp2& l1, fp2& l4) {
    const fp2 zz = f2_sqr(T.z), yy = f2_sqr(qy);
    const fp2 t0 = f2_mul(zz, qx);
    const fp2 t1 = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(qy, T.z)), yy), zz), zz);
    const fp2 t2 = f2_sub(t0, T.x);
    const fp2 t3 = f2_sqr(t2);
    const fp2 t4 = f2_dbl(f2_dbl(t3));
    const fp2 t5 = f2_mul(t4, t2);
    const fp2 t6 = f2_sub(f2_sub(t1, T.y), T.y);
    fp2 t9 = f2_mul(t6, qx);
    const fp2 t7 = f2_mul(t4, T.x);
    T.x = f2_sub(f2_sub(f2_sub(f2_sqr(t6), t5), t7), t7);
    T.z = f2_sub(f2_sub(f2_sqr(f2_add(T.z, t2)), zz), t3);
    fp2 t10 = f2_add(qy, T.z);
    const fp2 t8 = f2_mul(f2_sub(t7, T.x), t6);
    T.y = f2_sub(t8, f2_dbl(f2_mul(T.y, t5)));
    t10 = f2_sub(f2_sub(f2_sqr(t10), yy), f2_sqr(T.z));
    t9 = f2_sub(f2_dbl(t9), t10);
    l4 = f2_dbl(T.z);
    l1 = f2_dbl(f2_neg(t6));
    l0 = t9;
}
BLS_HD fp12 ml_line(const fp12& f, const fp2& l0, const fp2& l1, const fp2& l4, const fp& px, const fp& py) {
    return f12_mul_014(f, l0, f2_mul_fp(l1, px), f2_mul_fp(l4, py));
}
// prod_{i < n} f_{|x|, Q_i}(P_i), conjugated (x < 0); n <= 2
BLS_NOINLINE fp12 miller_loop2(int n, const fp* px, const fp* py, const fp2* qx, const fp2* qy) {
    jac<fp2> T[2];
    for (int i = 0; i < n; i++) T[i] = jac_from_affine(qx[i], qy[i]);
    fp12 f = f12_one();
    fp2 l0, l1, l4;
    for (int b = 62; b >= 0; b--) {
        if (b != 62) f = f12_sqr(f);
        for (int i = 0; i < n; i++) {
            ml_dbl(T[i], l0, l1, l4);
            f = ml_line(f, l0, l1, l4, px[i], py[i]);
        }
        if ((BLS_X_ABS >> b) & 1)
            for (int i = 0; i < n; i++) {
                ml_add(T[i], qx[i], qy[i], l0, l1, l4);
                f = ml_line(f, l0, l1, l4, px[i], py[i]);
            }
    }
    return f12_conj(f);
}

}  // namespace bls
