/*
 * bls_oracle.c -- TEST INFRASTRUCTURE ONLY (see bls_oracle.h): a plain-C restatement of the
 * BLS12-381 min_sig signature scheme as fastcrypto 0.1.2 / blst 0.3.10 run it behind the
 * reference's crypto aliases (crypto/src/lib.rs:29-33).  Written for clarity, not speed: 6 x
 * 64-bit Montgomery limbs with unsigned __int128 products, the textbook tower
 * Fp2 = Fp[u]/(u^2+1), Fp6 = Fp2[v]/(v^3-(1+u)), Fp12 = Fp6[w]/(w^2-v).
 *
 * Verdict semantics restated (blst 0.3.10 + fastcrypto 0.1.2 wrappers; draft-irtf-cfrg-bls-signature):
 *   decode (ZCash format): compression flag set; infinity flag => every other bit zero; each
 *     coordinate < p; the point on the curve (G1: y^2 = x^3 + 4, G2: y^2 = x^3 + 4(1+u)); the sort
 *     flag picks the lexicographically larger y (Fp2: c1 first, then c0).
 *   public key: decodes, is not the identity, lies in G2 (KeyValidate).
 *   Verifier::verify(pk, m, sig): sig decodes and lies in G1 (the identity passes the group
 *     check); pk validates; e(sig, -g2) * e(H(m), pk) == 1.
 *   AggregateSignature::aggregate(sigs): every sig decodes and lies in G1, sum; empty => error.
 *   AggregateAuthenticator::verify / fast_aggregate_verify(sig, pks, m): pks non-empty, apk =
 *     sum of the (already validated) pks, apk != identity, then as verify with pk = apk.
 * H(m) = hash_to_curve G1 (RFC 9380 §3, §5.3.1 expand_message_xmd SHA-256, §6.6.2 simplified SWU
 * with Z = 11 on the 11-isogenous curve, §6.6.3 isogeny map (oracle/bls_iso.h), §7 cofactor
 * clearing by h_eff = 0xd201000000010001).
 */
#include "bls_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "bls_iso.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t v[6]; } fp;
typedef struct { fp c0, c1; } fp2;
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
typedef struct { fp x, y, z; int inf; } g1j;    /* Jacobian: (X/Z^2, Y/Z^3) */
typedef struct { fp2 x, y, z; int inf; } g2j;

/* p = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab */
static const uint64_t P_[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                               0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
/* r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001 */
static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                 0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                 0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};
static const uint64_t BLS_X_ABS = 0xd201000000010000ull; /* the curve parameter x = -BLS_X_ABS */
static const uint64_t H_EFF = 0xd201000000010001ull;
/* (p^4 - p^2 + 1) / r, big-endian (computed with Python integers; tests/test_bls_oracle.py
 * recomputes it and compares) */
static const char* HARD_EXP_HEX =
    "000f686b3d807d01c0bd38c3195c899ed3cde88eeb996ca394506632528d6a9a"
    "2f230063cf081517f68f7764c28b6f8ae5a72bce8d63cb9f827eca0ba621315b"
    "2076995003fc77a17988f8761bdc51dc2378b9039096d1b767f17fcbde783765"
    "915c97f36c6f18212ed0b283ed237db421d160aeb6a1e79983774940996754c8"
    "c71a2629b0dea236905ce937335d5b68fa9912aae208ccf1e516c3f438e3ba79";

static uint64_t N0;          /* -p^-1 mod 2^64 */
static fp R2, ONE, FP_ZERO;  /* R^2 mod p, R mod p (Montgomery 1) */
static fp2 GAMMA[6];         /* xi^(k(p-1)/6): w^(kp) = w^k * GAMMA[k] */
static fp2 B2;               /* 4(1+u) */
static fp B1, SSWU_A, SSWU_B, SSWU_Z;
static fp ISO[4][16];
static int ISO_LEN[4];
static uint8_t HARD_EXP[160];
static pthread_once_t once = PTHREAD_ONCE_INIT;

/* ------------------------------------------------------------------------------------ Fp */
static int fp_geq_p(const uint64_t* t) {
    for (int i = 5; i >= 0; i--) {
        if (t[i] > P_[i]) return 1;
        if (t[i] < P_[i]) return 0;
    }
    return 1;
}
static void sub_p(uint64_t* t) {
    u128 br = 0;
    for (int i = 0; i < 6; i++) {
        u128 d = (u128)t[i] - P_[i] - br;
        t[i] = (uint64_t)d;
        br = (d >> 64) & 1;
    }
}
static void fp_add(fp* r, const fp* a, const fp* b) {
    u128 c = 0;
    uint64_t t[6];
    for (int i = 0; i < 6; i++) {
        c += (u128)a->v[i] + b->v[i];
        t[i] = (uint64_t)c;
        c >>= 64;
    }
    if (c || fp_geq_p(t)) sub_p(t);
    memcpy(r->v, t, 48);
}
static void fp_sub(fp* r, const fp* a, const fp* b) {
    u128 br = 0;
    uint64_t t[6];
    for (int i = 0; i < 6; i++) {
        u128 d = (u128)a->v[i] - b->v[i] - br;
        t[i] = (uint64_t)d;
        br = (d >> 64) & 1;
    }
    if (br) {
        u128 c = 0;
        for (int i = 0; i < 6; i++) {
            c += (u128)t[i] + P_[i];
            t[i] = (uint64_t)c;
            c >>= 64;
        }
    }
    memcpy(r->v, t, 48);
}
static void fp_neg(fp* r, const fp* a) { fp_sub(r, &FP_ZERO, a); }
/* Montgomery product a b R^-1 mod p (CIOS) */
static void fp_mul(fp* r, const fp* a, const fp* b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 6; i++) {
        u128 c = 0;
        for (int j = 0; j < 6; j++) {
            c += (u128)a->v[j] * b->v[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[6];
        t[6] = (uint64_t)c;
        t[7] = (uint64_t)(c >> 64);
        const uint64_t m = t[0] * N0;
        c = (u128)m * P_[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 6; j++) {
            c += (u128)m * P_[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[6];
        t[5] = (uint64_t)c;
        t[6] = t[7] + (uint64_t)(c >> 64);
    }
    if (t[6] || fp_geq_p(t)) sub_p(t);
    memcpy(r->v, t, 48);
}
static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static int fp_is_zero(const fp* a) {
    uint64_t o = 0;
    for (int i = 0; i < 6; i++) o |= a->v[i];
    return o == 0;
}
static int fp_eq(const fp* a, const fp* b) { return memcmp(a->v, b->v, 48) == 0; }
static void fp_from_u64(fp* r, uint64_t x) {
    fp t = {{x, 0, 0, 0, 0, 0}};
    fp_mul(r, &t, &R2);
}
static void fp_from_limbs(fp* r, const uint64_t l[6]) {
    fp t;
    memcpy(t.v, l, 48);
    fp_mul(r, &t, &R2);
}
static void fp_to_plain(uint64_t l[6], const fp* a) {
    fp one = {{1, 0, 0, 0, 0, 0}}, t;
    fp_mul(&t, a, &one);
    memcpy(l, t.v, 48);
}
/* big-endian 48 bytes -> Fp; 0 if the value is >= p */
static int fp_from_be(fp* r, const uint8_t b[48]) {
    uint64_t l[6];
    for (int i = 0; i < 6; i++) {
        uint64_t w = 0;
        for (int k = 0; k < 8; k++) w = (w << 8) | b[48 - 8 * (i + 1) + k];
        l[i] = w;
    }
    if (fp_geq_p(l)) return 0;
    fp_from_limbs(r, l);
    return 1;
}
static void fp_to_be(uint8_t b[48], const fp* a) {
    uint64_t l[6];
    fp_to_plain(l, a);
    for (int i = 0; i < 6; i++)
        for (int k = 0; k < 8; k++) b[48 - 8 * (i + 1) + k] = (uint8_t)(l[i] >> (56 - 8 * k));
}
/* a^e, e given as little-endian 64-bit limbs */
static void fp_pow(fp* r, const fp* a, const uint64_t* e, int nl) {
    fp acc = ONE, base = *a;
    for (int i = nl - 1; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            fp_sqr(&acc, &acc);
            if ((e[i] >> b) & 1) fp_mul(&acc, &acc, &base);
        }
    *r = acc;
}
static void p_minus(uint64_t out[6], uint64_t k) { /* p - k */
    memcpy(out, P_, 48);
    u128 br = k;
    for (int i = 0; i < 6 && br; i++) {
        u128 d = (u128)out[i] - br;
        out[i] = (uint64_t)d;
        br = (d >> 64) & 1;
    }
}
static void shr(uint64_t out[6], const uint64_t in[6], int s) {
    for (int i = 0; i < 6; i++) out[i] = (in[i] >> s) | (i < 5 ? in[i + 1] << (64 - s) : 0);
}
static void fp_inv(fp* r, const fp* a) {
    uint64_t e[6];
    p_minus(e, 2);
    fp_pow(r, a, e, 6);
}
static int fp_sqrt(fp* r, const fp* a) { /* p = 3 mod 4: a^((p+1)/4) */
    uint64_t e[6], t[6];
    memcpy(t, P_, 48);
    shr(e, t, 2);
    e[0] += 1; /* (p+1)/4 = floor(p/4) + 1 since p = 3 mod 4 */
    fp s, c;
    fp_pow(&s, a, e, 6);
    fp_sqr(&c, &s);
    if (!fp_eq(&c, a)) return 0;
    *r = s;
    return 1;
}
/* lexicographic sign of the ZCash format: y > (p-1)/2 */
static int fp_lex_large(const fp* a) {
    uint64_t l[6], h[6], t[6];
    fp_to_plain(l, a);
    memcpy(t, P_, 48);
    shr(h, t, 1); /* (p-1)/2 = floor(p/2) */
    for (int i = 5; i >= 0; i--) {
        if (l[i] > h[i]) return 1;
        if (l[i] < h[i]) return 0;
    }
    return 0;
}
static int fp_sgn0(const fp* a) {
    uint64_t l[6];
    fp_to_plain(l, a);
    return (int)(l[0] & 1);
}

/* ----------------------------------------------------------------------------------- Fp2 */
static void f2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void f2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void f2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void f2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static void f2_mul(fp2* r, const fp2* a, const fp2* b) {
    fp t0, t1, s0, s1, m;
    fp_mul(&t0, &a->c0, &b->c0);
    fp_mul(&t1, &a->c1, &b->c1);
    fp_add(&s0, &a->c0, &a->c1);
    fp_add(&s1, &b->c0, &b->c1);
    fp_mul(&m, &s0, &s1);
    fp_sub(&r->c0, &t0, &t1);
    fp_sub(&m, &m, &t0);
    fp_sub(&r->c1, &m, &t1);
}
static void f2_sqr(fp2* r, const fp2* a) { f2_mul(r, a, a); }
static void f2_mul_fp(fp2* r, const fp2* a, const fp* b) { fp_mul(&r->c0, &a->c0, b); fp_mul(&r->c1, &a->c1, b); }
static void f2_mul_xi(fp2* r, const fp2* a) { /* (1+u) a */
    fp t0, t1;
    fp_sub(&t0, &a->c0, &a->c1);
    fp_add(&t1, &a->c0, &a->c1);
    r->c0 = t0;
    r->c1 = t1;
}
static int f2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int f2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void f2_inv(fp2* r, const fp2* a) {
    fp n, t;
    fp_sqr(&n, &a->c0);
    fp_sqr(&t, &a->c1);
    fp_add(&n, &n, &t);
    fp_inv(&n, &n);
    fp_mul(&r->c0, &a->c0, &n);
    fp_mul(&t, &a->c1, &n);
    fp_neg(&r->c1, &t);
}
/* a^e, e as little-endian 64-bit limbs */
static void f2_pow(fp2* r, const fp2* a, const uint64_t* e, int nl) {
    fp2 acc = {ONE, FP_ZERO}, base = *a;
    for (int i = nl - 1; i >= 0; i--)
        for (int b = 63; b >= 0; b--) {
            f2_sqr(&acc, &acc);
            if ((e[i] >> b) & 1) f2_mul(&acc, &acc, &base);
        }
    *r = acc;
}
/* square root in Fp2 for p = 3 mod 4 (Adj, Rodriguez-Henriquez 2012, Algorithm 9) */
static int f2_sqrt(fp2* r, const fp2* a) {
    if (f2_is_zero(a)) {
        *r = *a;
        return 1;
    }
    uint64_t e[6], t[6];
    memcpy(t, P_, 48);
    shr(e, t, 2); /* (p-3)/4 */
    fp2 a1, alpha, x0, a0, c;
    f2_pow(&a1, a, e, 6);
    f2_sqr(&alpha, &a1);
    f2_mul(&alpha, &alpha, a);
    f2_mul(&x0, &a1, a);
    f2_conj(&a0, &alpha);
    f2_mul(&a0, &a0, &alpha);
    fp2 m1 = {ONE, FP_ZERO};
    f2_neg(&m1, &m1);
    if (f2_eq(&a0, &m1)) return 0;
    fp2 x;
    if (f2_eq(&alpha, &m1)) {
        x.c0 = x0.c1;
        fp_neg(&x.c0, &x.c0); /* u * (c0 + c1 u) = -c1 + c0 u */
        x.c1 = x0.c0;
    } else {
        fp2 one = {ONE, FP_ZERO}, b;
        f2_add(&b, &alpha, &one);
        shr(e, t, 1); /* (p-1)/2 */
        f2_pow(&b, &b, e, 6);
        f2_mul(&x, &b, &x0);
    }
    f2_sqr(&c, &x);
    if (!f2_eq(&c, a)) return 0;
    *r = x;
    return 1;
}
static int f2_lex_large(const fp2* a) {
    if (!fp_is_zero(&a->c1)) return fp_lex_large(&a->c1);
    return fp_lex_large(&a->c0);
}

/* ----------------------------------------------------------------------------- Fp6, Fp12 */
static void f6_add(fp6* r, const fp6* a, const fp6* b) { f2_add(&r->c0, &a->c0, &b->c0); f2_add(&r->c1, &a->c1, &b->c1); f2_add(&r->c2, &a->c2, &b->c2); }
static void f6_sub(fp6* r, const fp6* a, const fp6* b) { f2_sub(&r->c0, &a->c0, &b->c0); f2_sub(&r->c1, &a->c1, &b->c1); f2_sub(&r->c2, &a->c2, &b->c2); }
static void f6_neg(fp6* r, const fp6* a) { f2_neg(&r->c0, &a->c0); f2_neg(&r->c1, &a->c1); f2_neg(&r->c2, &a->c2); }
static void f6_mul(fp6* r, const fp6* a, const fp6* b) {
    fp2 t0, t1, t2, s0, s1, m, c0, c1, c2;
    f2_mul(&t0, &a->c0, &b->c0);
    f2_mul(&t1, &a->c1, &b->c1);
    f2_mul(&t2, &a->c2, &b->c2);
    f2_add(&s0, &a->c1, &a->c2);
    f2_add(&s1, &b->c1, &b->c2);
    f2_mul(&m, &s0, &s1);
    f2_sub(&m, &m, &t1);
    f2_sub(&m, &m, &t2);
    f2_mul_xi(&m, &m);
    f2_add(&c0, &t0, &m);
    f2_add(&s0, &a->c0, &a->c1);
    f2_add(&s1, &b->c0, &b->c1);
    f2_mul(&m, &s0, &s1);
    f2_sub(&m, &m, &t0);
    f2_sub(&m, &m, &t1);
    f2_mul_xi(&c1, &t2);
    f2_add(&c1, &c1, &m);
    f2_add(&s0, &a->c0, &a->c2);
    f2_add(&s1, &b->c0, &b->c2);
    f2_mul(&m, &s0, &s1);
    f2_sub(&m, &m, &t0);
    f2_sub(&m, &m, &t2);
    f2_add(&c2, &m, &t1);
    r->c0 = c0;
    r->c1 = c1;
    r->c2 = c2;
}
static void f6_mul_v(fp6* r, const fp6* a) {
    fp2 t;
    f2_mul_xi(&t, &a->c2);
    r->c2 = a->c1;
    r->c1 = a->c0;
    r->c0 = t;
}
static void f6_inv(fp6* r, const fp6* a) {
    fp2 A, B, C, t, F;
    f2_sqr(&A, &a->c0);
    f2_mul(&t, &a->c1, &a->c2);
    f2_mul_xi(&t, &t);
    f2_sub(&A, &A, &t);
    f2_sqr(&B, &a->c2);
    f2_mul_xi(&B, &B);
    f2_mul(&t, &a->c0, &a->c1);
    f2_sub(&B, &B, &t);
    f2_sqr(&C, &a->c1);
    f2_mul(&t, &a->c0, &a->c2);
    f2_sub(&C, &C, &t);
    f2_mul(&F, &a->c2, &B);
    f2_mul(&t, &a->c1, &C);
    f2_add(&F, &F, &t);
    f2_mul_xi(&F, &F);
    f2_mul(&t, &a->c0, &A);
    f2_add(&F, &F, &t);
    f2_inv(&F, &F);
    f2_mul(&r->c0, &A, &F);
    f2_mul(&r->c1, &B, &F);
    f2_mul(&r->c2, &C, &F);
}
static void f12_one(fp12* r) {
    memset(r, 0, sizeof(*r));
    r->c0.c0.c0 = ONE;
}
static void f12_mul(fp12* r, const fp12* a, const fp12* b) {
    fp6 t0, t1, s0, s1, m;
    f6_mul(&t0, &a->c0, &b->c0);
    f6_mul(&t1, &a->c1, &b->c1);
    f6_add(&s0, &a->c0, &a->c1);
    f6_add(&s1, &b->c0, &b->c1);
    f6_mul(&m, &s0, &s1);
    f6_sub(&m, &m, &t0);
    f6_sub(&r->c1, &m, &t1);
    f6_mul_v(&t1, &t1);
    f6_add(&r->c0, &t0, &t1);
}
static void f12_sqr(fp12* r, const fp12* a) { f12_mul(r, a, a); }
static void f12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; f6_neg(&r->c1, &a->c1); }
static void f12_inv(fp12* r, const fp12* a) {
    fp6 t0, t1;
    f6_mul(&t0, &a->c0, &a->c0);
    f6_mul(&t1, &a->c1, &a->c1);
    f6_mul_v(&t1, &t1);
    f6_sub(&t0, &t0, &t1);
    f6_inv(&t0, &t0);
    f6_mul(&r->c0, &a->c0, &t0);
    f6_mul(&t1, &a->c1, &t0);
    f6_neg(&r->c1, &t1);
}
/* coefficient k of the w-basis: w^(2i) -> c0.ci, w^(2i+1) -> c1.ci */
static fp2* f12_coef(fp12* a, int k) {
    fp6* h = (k & 1) ? &a->c1 : &a->c0;
    return k / 2 == 0 ? &h->c0 : k / 2 == 1 ? &h->c1 : &h->c2;
}
static void f12_frob(fp12* r, const fp12* a) {
    fp12 t = *a;
    for (int k = 0; k < 6; k++) {
        fp2* c = f12_coef(&t, k);
        f2_conj(c, c);
        f2_mul(c, c, &GAMMA[k]);
    }
    *r = t;
}
static int f12_eq(const fp12* a, const fp12* b) {
    fp12 x = *a, y = *b;
    for (int k = 0; k < 6; k++)
        if (!f2_eq(f12_coef(&x, k), f12_coef(&y, k))) return 0;
    return 1;
}
static int f12_is_one(const fp12* a) {
    fp12 o;
    f12_one(&o);
    return f12_eq(a, &o);
}
/* a^e, e big-endian bytes */
static void f12_pow_be(fp12* r, const fp12* a, const uint8_t* e, size_t n) {
    fp12 acc, base = *a;
    f12_one(&acc);
    for (size_t i = 0; i < n; i++)
        for (int b = 7; b >= 0; b--) {
            f12_sqr(&acc, &acc);
            if ((e[i] >> b) & 1) f12_mul(&acc, &acc, &base);
        }
    *r = acc;
}
/* sparse product by the line l = c0 + c1 v + c4 v w (tower slots c0.c0, c0.c1, c1.c1, i.e. the
 * w-basis powers 0, 2, 3: "014" in the Fp6-major numbering c0.c0..c0.c2, c1.c0..c1.c2) */
static void f12_mul_014(fp12* r, const fp12* a, const fp2* c0, const fp2* c1, const fp2* c4) {
    fp12 l;
    memset(&l, 0, sizeof(l));
    l.c0.c0 = *c0;
    l.c0.c1 = *c1;
    l.c1.c1 = *c4;
    f12_mul(r, a, &l);
}

/* ------------------------------------------------------------------------------ G1 / G2 */
static void g1_dbl(g1j* r, const g1j* a) {
    if (a->inf || fp_is_zero(&a->y)) {
        r->inf = 1;
        return;
    }
    fp A, B, C, D, E, F, t;
    fp_sqr(&A, &a->x);
    fp_sqr(&B, &a->y);
    fp_sqr(&C, &B);
    fp_add(&t, &a->x, &B);
    fp_sqr(&t, &t);
    fp_sub(&t, &t, &A);
    fp_sub(&t, &t, &C);
    fp_add(&D, &t, &t);
    fp_add(&E, &A, &A);
    fp_add(&E, &E, &A);
    fp_sqr(&F, &E);
    g1j o;
    fp_sub(&o.x, &F, &D);
    fp_sub(&o.x, &o.x, &D);
    fp_mul(&o.z, &a->y, &a->z);
    fp_add(&o.z, &o.z, &o.z);
    fp_sub(&t, &D, &o.x);
    fp_mul(&o.y, &E, &t);
    fp_add(&C, &C, &C);
    fp_add(&C, &C, &C);
    fp_add(&C, &C, &C);
    fp_sub(&o.y, &o.y, &C);
    o.inf = 0;
    *r = o;
}
static void g1_add(g1j* r, const g1j* a, const g1j* b) {
    if (a->inf) {
        *r = *b;
        return;
    }
    if (b->inf) {
        *r = *a;
        return;
    }
    fp z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
    fp_sqr(&z1z1, &a->z);
    fp_sqr(&z2z2, &b->z);
    fp_mul(&u1, &a->x, &z2z2);
    fp_mul(&u2, &b->x, &z1z1);
    fp_mul(&s1, &a->y, &b->z);
    fp_mul(&s1, &s1, &z2z2);
    fp_mul(&s2, &b->y, &a->z);
    fp_mul(&s2, &s2, &z1z1);
    if (fp_eq(&u1, &u2)) {
        if (fp_eq(&s1, &s2)) {
            g1_dbl(r, a);
            return;
        }
        r->inf = 1;
        return;
    }
    fp_sub(&h, &u2, &u1);
    fp_add(&i, &h, &h);
    fp_sqr(&i, &i);
    fp_mul(&j, &h, &i);
    fp_sub(&rr, &s2, &s1);
    fp_add(&rr, &rr, &rr);
    fp_mul(&v, &u1, &i);
    g1j o;
    fp_sqr(&o.x, &rr);
    fp_sub(&o.x, &o.x, &j);
    fp_sub(&o.x, &o.x, &v);
    fp_sub(&o.x, &o.x, &v);
    fp_sub(&t, &v, &o.x);
    fp_mul(&o.y, &rr, &t);
    fp_mul(&t, &s1, &j);
    fp_add(&t, &t, &t);
    fp_sub(&o.y, &o.y, &t);
    fp_add(&t, &a->z, &b->z);
    fp_sqr(&t, &t);
    fp_sub(&t, &t, &z1z1);
    fp_sub(&t, &t, &z2z2);
    fp_mul(&o.z, &t, &h);
    o.inf = 0;
    *r = o;
}
static void g1_mul_be(g1j* r, const g1j* a, const uint8_t* k, size_t n) {
    g1j acc;
    acc.inf = 1;
    for (size_t i = 0; i < n; i++)
        for (int b = 7; b >= 0; b--) {
            g1_dbl(&acc, &acc);
            if ((k[i] >> b) & 1) g1_add(&acc, &acc, a);
        }
    *r = acc;
}
static void g1_affine(fp* x, fp* y, const g1j* a) {
    fp zi, zi2;
    fp_inv(&zi, &a->z);
    fp_sqr(&zi2, &zi);
    fp_mul(x, &a->x, &zi2);
    fp_mul(&zi2, &zi2, &zi);
    fp_mul(y, &a->y, &zi2);
}
static void g2_dbl(g2j* r, const g2j* a) {
    if (a->inf || f2_is_zero(&a->y)) {
        r->inf = 1;
        return;
    }
    fp2 A, B, C, D, E, F, t;
    f2_sqr(&A, &a->x);
    f2_sqr(&B, &a->y);
    f2_sqr(&C, &B);
    f2_add(&t, &a->x, &B);
    f2_sqr(&t, &t);
    f2_sub(&t, &t, &A);
    f2_sub(&t, &t, &C);
    f2_add(&D, &t, &t);
    f2_add(&E, &A, &A);
    f2_add(&E, &E, &A);
    f2_sqr(&F, &E);
    g2j o;
    f2_sub(&o.x, &F, &D);
    f2_sub(&o.x, &o.x, &D);
    f2_mul(&o.z, &a->y, &a->z);
    f2_add(&o.z, &o.z, &o.z);
    f2_sub(&t, &D, &o.x);
    f2_mul(&o.y, &E, &t);
    f2_add(&C, &C, &C);
    f2_add(&C, &C, &C);
    f2_add(&C, &C, &C);
    f2_sub(&o.y, &o.y, &C);
    o.inf = 0;
    *r = o;
}
static void g2_add(g2j* r, const g2j* a, const g2j* b) {
    if (a->inf) {
        *r = *b;
        return;
    }
    if (b->inf) {
        *r = *a;
        return;
    }
    fp2 z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
    f2_sqr(&z1z1, &a->z);
    f2_sqr(&z2z2, &b->z);
    f2_mul(&u1, &a->x, &z2z2);
    f2_mul(&u2, &b->x, &z1z1);
    f2_mul(&s1, &a->y, &b->z);
    f2_mul(&s1, &s1, &z2z2);
    f2_mul(&s2, &b->y, &a->z);
    f2_mul(&s2, &s2, &z1z1);
    if (f2_eq(&u1, &u2)) {
        if (f2_eq(&s1, &s2)) {
            g2_dbl(r, a);
            return;
        }
        r->inf = 1;
        return;
    }
    f2_sub(&h, &u2, &u1);
    f2_add(&i, &h, &h);
    f2_sqr(&i, &i);
    f2_mul(&j, &h, &i);
    f2_sub(&rr, &s2, &s1);
    f2_add(&rr, &rr, &rr);
    f2_mul(&v, &u1, &i);
    g2j o;
    f2_sqr(&o.x, &rr);
    f2_sub(&o.x, &o.x, &j);
    f2_sub(&o.x, &o.x, &v);
    f2_sub(&o.x, &o.x, &v);
    f2_sub(&t, &v, &o.x);
    f2_mul(&o.y, &rr, &t);
    f2_mul(&t, &s1, &j);
    f2_add(&t, &t, &t);
    f2_sub(&o.y, &o.y, &t);
    f2_add(&t, &a->z, &b->z);
    f2_sqr(&t, &t);
    f2_sub(&t, &t, &z1z1);
    f2_sub(&t, &t, &z2z2);
    f2_mul(&o.z, &t, &h);
    o.inf = 0;
    *r = o;
}
static void g2_mul_be(g2j* r, const g2j* a, const uint8_t* k, size_t n) {
    g2j acc;
    acc.inf = 1;
    for (size_t i = 0; i < n; i++)
        for (int b = 7; b >= 0; b--) {
            g2_dbl(&acc, &acc);
            if ((k[i] >> b) & 1) g2_add(&acc, &acc, a);
        }
    *r = acc;
}
static void g2_affine(fp2* x, fp2* y, const g2j* a) {
    fp2 zi, zi2;
    f2_inv(&zi, &a->z);
    f2_sqr(&zi2, &zi);
    f2_mul(x, &a->x, &zi2);
    f2_mul(&zi2, &zi2, &zi);
    f2_mul(y, &a->y, &zi2);
}

/* -------------------------------------------------------------------------------- init */
static void hex_to_bytes(const char* h, uint8_t* out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        unsigned v;
        char b[3] = {h[2 * i], h[2 * i + 1], 0};
        v = (unsigned)strtoul(b, NULL, 16);
        out[i] = (uint8_t)v;
    }
}
static void init(void) {
    uint64_t inv = 1; /* Newton: p^-1 mod 2^64 */
    for (int i = 0; i < 7; i++) inv *= 2 - P_[0] * inv;
    N0 = (uint64_t)0 - inv;
    memset(&FP_ZERO, 0, sizeof(FP_ZERO));
    /* R mod p and R^2 mod p by doubling 1 (plain residues) */
    fp t = {{1, 0, 0, 0, 0, 0}};
    for (int i = 0; i < 768; i++) {
        if (i == 384) ONE = t;
        fp_add(&t, &t, &t);
    }
    R2 = t;
    fp_from_u64(&B1, 4);
    fp2 xi = {ONE, ONE};
    B2.c0 = B1;
    B2.c1 = B1;
    /* GAMMA[k] = xi^(k (p-1)/6) */
    uint64_t e[6], pm1[6];
    p_minus(pm1, 1);
    {  /* (p-1)/6: divide the 384-bit number by 6 */
        u128 rem = 0;
        for (int i = 5; i >= 0; i--) {
            u128 cur = (rem << 64) | pm1[i];
            e[i] = (uint64_t)(cur / 6);
            rem = cur % 6;
        }
    }
    fp2 g;
    f2_pow(&g, &xi, e, 6);
    GAMMA[0].c0 = ONE;
    GAMMA[0].c1 = FP_ZERO;
    for (int k = 1; k < 6; k++) f2_mul(&GAMMA[k], &GAMMA[k - 1], &g);
    const uint64_t(*tabs[4])[6] = {ISO_XNUM, ISO_XDEN, ISO_YNUM, ISO_YDEN};
    const int lens[4] = {ISO_XNUM_LEN, ISO_XDEN_LEN, ISO_YNUM_LEN, ISO_YDEN_LEN};
    for (int k = 0; k < 4; k++) {
        ISO_LEN[k] = lens[k];
        for (int i = 0; i < lens[k]; i++) fp_from_limbs(&ISO[k][i], tabs[k][i]);
    }
    static const uint8_t A_BE[48] = {0x00, 0x14, 0x46, 0x98, 0xa3, 0xb8, 0xe9, 0x43, 0x3d, 0x69, 0x3a, 0x02,
                                     0xc9, 0x6d, 0x49, 0x82, 0xb0, 0xea, 0x98, 0x53, 0x83, 0xee, 0x66, 0xa8,
                                     0xd8, 0xe8, 0x98, 0x1a, 0xef, 0xd8, 0x81, 0xac, 0x98, 0x93, 0x6f, 0x8d,
                                     0xa0, 0xe0, 0xf9, 0x7f, 0x5c, 0xf4, 0x28, 0x08, 0x2d, 0x58, 0x4c, 0x1d};
    static const uint8_t B_BE[48] = {0x12, 0xe2, 0x90, 0x8d, 0x11, 0x68, 0x80, 0x30, 0x01, 0x8b, 0x12, 0xe8,
                                     0x75, 0x3e, 0xee, 0x3b, 0x20, 0x16, 0xc1, 0xf0, 0xf2, 0x4f, 0x40, 0x70,
                                     0xa0, 0xb9, 0xc1, 0x4f, 0xce, 0xf3, 0x5e, 0xf5, 0x5a, 0x23, 0x21, 0x5a,
                                     0x31, 0x6c, 0xea, 0xa5, 0xd1, 0xcc, 0x48, 0xe9, 0x8e, 0x17, 0x2b, 0xe0};
    fp_from_be(&SSWU_A, A_BE);
    fp_from_be(&SSWU_B, B_BE);
    fp_from_u64(&SSWU_Z, 11);
    hex_to_bytes(HARD_EXP_HEX, HARD_EXP, 160);
}
#define INIT() pthread_once(&once, init)

static void g1_gen(g1j* g) {
    static const uint8_t X[48] = {0x17, 0xf1, 0xd3, 0xa7, 0x31, 0x97, 0xd7, 0x94, 0x26, 0x95, 0x63, 0x8c,
                                  0x4f, 0xa9, 0xac, 0x0f, 0xc3, 0x68, 0x8c, 0x4f, 0x97, 0x74, 0xb9, 0x05,
                                  0xa1, 0x4e, 0x3a, 0x3f, 0x17, 0x1b, 0xac, 0x58, 0x6c, 0x55, 0xe8, 0x3f,
                                  0xf9, 0x7a, 0x1a, 0xef, 0xfb, 0x3a, 0xf0, 0x0a, 0xdb, 0x22, 0xc6, 0xbb};
    static const uint8_t Y[48] = {0x08, 0xb3, 0xf4, 0x81, 0xe3, 0xaa, 0xa0, 0xf1, 0xa0, 0x9e, 0x30, 0xed,
                                  0x74, 0x1d, 0x8a, 0xe4, 0xfc, 0xf5, 0xe0, 0x95, 0xd5, 0xd0, 0x0a, 0xf6,
                                  0x00, 0xdb, 0x18, 0xcb, 0x2c, 0x04, 0xb3, 0xed, 0xd0, 0x3c, 0xc7, 0x44,
                                  0xa2, 0x88, 0x8a, 0xe4, 0x0c, 0xaa, 0x23, 0x29, 0x46, 0xc5, 0xe7, 0xe1};
    fp_from_be(&g->x, X);
    fp_from_be(&g->y, Y);
    g->z = ONE;
    g->inf = 0;
}
static void g2_gen(g2j* g) {
    static const char* H[4] = {
        "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8",
        "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e",
        "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801",
        "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"};
    uint8_t b[48];
    fp* c[4] = {&g->x.c0, &g->x.c1, &g->y.c0, &g->y.c1};
    for (int i = 0; i < 4; i++) {
        hex_to_bytes(H[i], b, 48);
        fp_from_be(c[i], b);
    }
    g->z.c0 = ONE;
    g->z.c1 = FP_ZERO;
    g->inf = 0;
}

/* ---------------------------------------------------------- (de)serialisation, ZCash format */
static void g1_load(g1j* P, const uint8_t in[96]) {
    int zero = 1;
    for (int i = 0; i < 96; i++) zero &= in[i] == 0;
    P->inf = zero;
    if (zero) return;
    fp_from_be(&P->x, in);
    fp_from_be(&P->y, in + 48);
    P->z = ONE;
}
static void g1_store(uint8_t out[96], const g1j* P) {
    if (P->inf) {
        memset(out, 0, 96);
        return;
    }
    fp x, y;
    g1_affine(&x, &y, P);
    fp_to_be(out, &x);
    fp_to_be(out + 48, &y);
}
static void g2_load(g2j* Q, const uint8_t in[192]) {
    int zero = 1;
    for (int i = 0; i < 192; i++) zero &= in[i] == 0;
    Q->inf = zero;
    if (zero) return;
    /* uncompressed G2 layout: x.c1 || x.c0 || y.c1 || y.c0 (ZCash order) */
    fp_from_be(&Q->x.c1, in);
    fp_from_be(&Q->x.c0, in + 48);
    fp_from_be(&Q->y.c1, in + 96);
    fp_from_be(&Q->y.c0, in + 144);
    Q->z.c0 = ONE;
    Q->z.c1 = FP_ZERO;
}
static void g2_store(uint8_t out[192], const g2j* Q) {
    if (Q->inf) {
        memset(out, 0, 192);
        return;
    }
    fp2 x, y;
    g2_affine(&x, &y, Q);
    fp_to_be(out, &x.c1);
    fp_to_be(out + 48, &x.c0);
    fp_to_be(out + 96, &y.c1);
    fp_to_be(out + 144, &y.c0);
}
static void g1_compress_j(uint8_t out[48], const g1j* P) {
    if (P->inf) {
        memset(out, 0, 48);
        out[0] = 0xc0;
        return;
    }
    fp x, y;
    g1_affine(&x, &y, P);
    fp_to_be(out, &x);
    out[0] |= 0x80 | (fp_lex_large(&y) ? 0x20 : 0);
}
static void g2_compress_j(uint8_t out[96], const g2j* Q) {
    if (Q->inf) {
        memset(out, 0, 96);
        out[0] = 0xc0;
        return;
    }
    fp2 x, y;
    g2_affine(&x, &y, Q);
    fp_to_be(out, &x.c1);
    fp_to_be(out + 48, &x.c0);
    out[0] |= 0x80 | (f2_lex_large(&y) ? 0x20 : 0);
}
static int g1_decompress_j(g1j* P, const uint8_t in[48]) {
    const uint8_t f = in[0];
    if (!(f & 0x80)) return ORB_BAD_ENCODING;
    if (f & 0x40) {
        if (f & 0x3f) return ORB_BAD_ENCODING;
        for (int i = 1; i < 48; i++)
            if (in[i]) return ORB_BAD_ENCODING;
        P->inf = 1;
        return ORB_OK;
    }
    uint8_t b[48];
    memcpy(b, in, 48);
    b[0] &= 0x1f;
    fp x, y2, y;
    if (!fp_from_be(&x, b)) return ORB_BAD_ENCODING;
    fp_sqr(&y2, &x);
    fp_mul(&y2, &y2, &x);
    fp_add(&y2, &y2, &B1);
    if (!fp_sqrt(&y, &y2)) return ORB_NOT_ON_CURVE;
    if (fp_lex_large(&y) != !!(f & 0x20)) fp_neg(&y, &y);
    P->x = x;
    P->y = y;
    P->z = ONE;
    P->inf = 0;
    return ORB_OK;
}
static int g2_decompress_j(g2j* Q, const uint8_t in[96]) {
    const uint8_t f = in[0];
    if (!(f & 0x80)) return ORB_BAD_ENCODING;
    if (f & 0x40) {
        if (f & 0x3f) return ORB_BAD_ENCODING;
        for (int i = 1; i < 96; i++)
            if (in[i]) return ORB_BAD_ENCODING;
        Q->inf = 1;
        return ORB_OK;
    }
    uint8_t b[48];
    memcpy(b, in, 48);
    b[0] &= 0x1f;
    fp2 x, y2, y;
    if (!fp_from_be(&x.c1, b) || !fp_from_be(&x.c0, in + 48)) return ORB_BAD_ENCODING;
    f2_sqr(&y2, &x);
    f2_mul(&y2, &y2, &x);
    f2_add(&y2, &y2, &B2);
    if (!f2_sqrt(&y, &y2)) return ORB_NOT_ON_CURVE;
    if (f2_lex_large(&y) != !!(f & 0x20)) f2_neg(&y, &y);
    Q->x = x;
    Q->y = y;
    Q->z.c0 = ONE;
    Q->z.c1 = FP_ZERO;
    Q->inf = 0;
    return ORB_OK;
}
/* subgroup membership by definition: [r] P = O */
static int g1_in_group_j(const g1j* P) {
    g1j t;
    g1_mul_be(&t, P, R_BE, 32);
    return t.inf;
}
static int g2_in_group_j(const g2j* Q) {
    g2j t;
    g2_mul_be(&t, Q, R_BE, 32);
    return t.inf;
}

/* --------------------------------------------------------------------------------- SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(uint32_t h[8], const uint8_t* b) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b_ = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b_) ^ (a & c) ^ (b_ & c));
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b_;
        b_ = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b_;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
}
typedef struct {
    uint32_t h[8];
    uint8_t buf[64];
    size_t n, total;
} sha256_ctx;
static void sha256_init(sha256_ctx* c) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(c->h, iv, 32);
    c->n = c->total = 0;
}
static void sha256_update(sha256_ctx* c, const uint8_t* m, size_t n) {
    c->total += n;
    while (n) {
        size_t k = 64 - c->n < n ? 64 - c->n : n;
        memcpy(c->buf + c->n, m, k);
        c->n += k;
        m += k;
        n -= k;
        if (c->n == 64) {
            sha256_block(c->h, c->buf);
            c->n = 0;
        }
    }
}
static void sha256_final(sha256_ctx* c, uint8_t out[32]) {
    const uint64_t bits = (uint64_t)c->total * 8;
    uint8_t pad = 0x80;
    sha256_update(c, &pad, 1);
    pad = 0;
    while (c->n != 56) sha256_update(c, &pad, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha256_update(c, l, 8);
    for (int i = 0; i < 8; i++)
        for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(c->h[i] >> (24 - 8 * k));
}
void orb_sha256(const uint8_t* m, size_t n, uint8_t out[32]) {
    sha256_ctx c;
    sha256_init(&c);
    sha256_update(&c, m, n);
    sha256_final(&c, out);
}

/* ------------------------------------------------------------------- hash_to_curve (G1) */
/* RFC 9380 §5.3.1 with SHA-256 (b_in_bytes 32, s_in_bytes 64); out_len <= 255 * 32 */
void orb_expand_message_xmd(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len, uint8_t* out,
                            size_t out_len) {
    const size_t ell = (out_len + 31) / 32;
    const uint8_t dl = (uint8_t)dst_len;
    uint8_t b0[32], bi[32], z[64] = {0};
    sha256_ctx c;
    sha256_init(&c);
    sha256_update(&c, z, 64);
    sha256_update(&c, msg, n);
    uint8_t lib[3] = {(uint8_t)(out_len >> 8), (uint8_t)out_len, 0};
    sha256_update(&c, lib, 3);
    sha256_update(&c, dst, dst_len);
    sha256_update(&c, &dl, 1);
    sha256_final(&c, b0);
    uint8_t prev[32];
    for (size_t i = 1; i <= ell; i++) {
        uint8_t x[32], idx = (uint8_t)i;
        for (int k = 0; k < 32; k++) x[k] = i == 1 ? b0[k] : (uint8_t)(b0[k] ^ prev[k]);
        sha256_init(&c);
        sha256_update(&c, x, 32);
        sha256_update(&c, &idx, 1);
        sha256_update(&c, dst, dst_len);
        sha256_update(&c, &dl, 1);
        sha256_final(&c, bi);
        const size_t off = 32 * (i - 1), k = out_len - off < 32 ? out_len - off : 32;
        memcpy(out + off, bi, k);
        memcpy(prev, bi, 32);
    }
}
/* 64 big-endian bytes mod p */
static void fp_from_be64(fp* r, const uint8_t b[64]) {
    /* hi * 2^256 + lo with hi, lo < 2^256 < p: (hi * R * 2^256 / R) via Montgomery */
    uint8_t hi[48] = {0}, lo[48] = {0};
    memcpy(hi + 16, b, 32);
    memcpy(lo + 16, b + 32, 32);
    fp h, l, s;
    fp_from_be(&h, hi);
    fp_from_be(&l, lo);
    /* 2^256 mod p as a field element */
    fp two = {{2, 0, 0, 0, 0, 0}}, t;
    fp_mul(&t, &two, &R2); /* Montgomery 2 */
    s = ONE;
    for (int i = 0; i < 256; i++) fp_mul(&s, &s, &t);
    fp_mul(&h, &h, &s);
    fp_add(r, &h, &l);
}
static void map_sswu(fp* xo, fp* yo, const fp* u) {
    fp u2, tv1, t, x1, gx1, x2, gx2, y;
    fp_sqr(&u2, u);
    fp_mul(&t, &SSWU_Z, &u2);      /* Z u^2 */
    fp_sqr(&tv1, &t);              /* Z^2 u^4 */
    fp_add(&tv1, &tv1, &t);        /* Z^2 u^4 + Z u^2 */
    if (fp_is_zero(&tv1)) {
        fp za;
        fp_mul(&za, &SSWU_Z, &SSWU_A);
        fp_inv(&za, &za);
        fp_mul(&x1, &SSWU_B, &za);
    } else {
        fp_inv(&tv1, &tv1);
        fp_add(&tv1, &tv1, &ONE);
        fp ia, nb;
        fp_inv(&ia, &SSWU_A);
        fp_neg(&nb, &SSWU_B);
        fp_mul(&x1, &nb, &ia);
        fp_mul(&x1, &x1, &tv1);
    }
    fp_sqr(&gx1, &x1);
    fp_add(&gx1, &gx1, &SSWU_A);
    fp_mul(&gx1, &gx1, &x1);
    fp_add(&gx1, &gx1, &SSWU_B);
    fp_mul(&x2, &t, &x1);
    fp_sqr(&gx2, &x2);
    fp_add(&gx2, &gx2, &SSWU_A);
    fp_mul(&gx2, &gx2, &x2);
    fp_add(&gx2, &gx2, &SSWU_B);
    if (fp_sqrt(&y, &gx1)) {
        *xo = x1;
    } else {
        fp_sqrt(&y, &gx2);
        *xo = x2;
    }
    if (fp_sgn0(u) != fp_sgn0(&y)) fp_neg(&y, &y);
    *yo = y;
}
static void poly_eval(fp* r, const fp* c, int n, int monic, const fp* x) {
    fp acc = monic ? ONE : c[n - 1];
    for (int i = (monic ? n : n - 1) - 1; i >= 0; i--) {
        fp_mul(&acc, &acc, x);
        fp_add(&acc, &acc, &c[i]);
    }
    *r = acc;
}
static void iso_map(g1j* P, const fp* x, const fp* y) {
    fp xn, xd, yn, yd;
    poly_eval(&xn, ISO[0], ISO_LEN[0], 0, x);
    poly_eval(&xd, ISO[1], ISO_LEN[1], 1, x);
    poly_eval(&yn, ISO[2], ISO_LEN[2], 0, x);
    poly_eval(&yd, ISO[3], ISO_LEN[3], 1, x);
    fp_inv(&xd, &xd);
    fp_inv(&yd, &yd);
    fp_mul(&P->x, &xn, &xd);
    fp_mul(&P->y, &yn, &yd);
    fp_mul(&P->y, &P->y, y);
    P->z = ONE;
    P->inf = 0;
}
static void hash_to_g1_j(g1j* out, const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len) {
    uint8_t ub[128];
    orb_expand_message_xmd(msg, n, dst, dst_len, ub, 128);
    fp u0, u1, x, y;
    fp_from_be64(&u0, ub);
    fp_from_be64(&u1, ub + 64);
    g1j Q0, Q1, R;
    map_sswu(&x, &y, &u0);
    iso_map(&Q0, &x, &y);
    map_sswu(&x, &y, &u1);
    iso_map(&Q1, &x, &y);
    g1_add(&R, &Q0, &Q1);
    uint8_t h[8];
    for (int i = 0; i < 8; i++) h[i] = (uint8_t)(H_EFF >> (56 - 8 * i));
    g1_mul_be(out, &R, h, 8);
}
void orb_hash_to_g1(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len, uint8_t out[96]) {
    INIT();
    g1j P;
    hash_to_g1_j(&P, msg, n, dst, dst_len);
    g1_store(out, &P);
}

/* ------------------------------------------------------------------------------- pairing */
/* fast Miller loop: Jacobian T on the twist, lines l = c0 + c1 w + c4 w^4 scaled by Fp2
 * factors (killed by the final exponentiation); doubling / addition steps after Costello,
 * Lange, Naehrig (eprint 2010/354, Algorithms 26 and 27) for the M-type twist y^2 = x^3 + 4(1+u) */
static void ml_dbl(g2j* T, fp2* l0, fp2* l1, fp2* l4) {
    fp2 t0, t1, t2, t3, t4, t5, t6, zz, t;
    f2_sqr(&t0, &T->x);
    f2_sqr(&t1, &T->y);
    f2_sqr(&t2, &t1);
    f2_add(&t3, &t1, &T->x);
    f2_sqr(&t3, &t3);
    f2_sub(&t3, &t3, &t0);
    f2_sub(&t3, &t3, &t2);
    f2_add(&t3, &t3, &t3);
    f2_add(&t4, &t0, &t0);
    f2_add(&t4, &t4, &t0);
    f2_add(&t6, &T->x, &t4);
    f2_sqr(&t5, &t4);
    f2_sqr(&zz, &T->z);
    f2_sub(&T->x, &t5, &t3);
    f2_sub(&T->x, &T->x, &t3);
    f2_add(&t, &T->z, &T->y);
    f2_sqr(&t, &t);
    f2_sub(&t, &t, &t1);
    f2_sub(&T->z, &t, &zz);
    f2_sub(&t, &t3, &T->x);
    f2_mul(&T->y, &t, &t4);
    f2_add(&t2, &t2, &t2);
    f2_add(&t2, &t2, &t2);
    f2_add(&t2, &t2, &t2);
    f2_sub(&T->y, &T->y, &t2);
    f2_mul(&t3, &t4, &zz);
    f2_add(&t3, &t3, &t3);
    f2_neg(&t3, &t3);
    f2_sqr(&t6, &t6);
    f2_sub(&t6, &t6, &t0);
    f2_sub(&t6, &t6, &t5);
    f2_add(&t1, &t1, &t1);
    f2_add(&t1, &t1, &t1);
    f2_sub(&t6, &t6, &t1);
    f2_mul(&t0, &T->z, &zz);
    f2_add(&t0, &t0, &t0);
    *l4 = t0;  /* times y_P */
    *l1 = t3;  /* times x_P */
    *l0 = t6;
}
static void ml_add(g2j* T, const fp2* qx, const fp2* qy, fp2* l0, fp2* l1, fp2* l4) {
    fp2 zz, yy, t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t;
    f2_sqr(&zz, &T->z);
    f2_sqr(&yy, qy);
    f2_mul(&t0, &zz, qx);
    f2_add(&t, qy, &T->z);
    f2_sqr(&t, &t);
    f2_sub(&t, &t, &yy);
    f2_sub(&t, &t, &zz);
    f2_mul(&t1, &t, &zz);
    f2_sub(&t2, &t0, &T->x);
    f2_sqr(&t3, &t2);
    f2_add(&t4, &t3, &t3);
    f2_add(&t4, &t4, &t4);
    f2_mul(&t5, &t4, &t2);
    f2_sub(&t6, &t1, &T->y);
    f2_sub(&t6, &t6, &T->y);
    f2_mul(&t9, &t6, qx);
    f2_mul(&t7, &t4, &T->x);
    f2_sqr(&T->x, &t6);
    f2_sub(&T->x, &T->x, &t5);
    f2_sub(&T->x, &T->x, &t7);
    f2_sub(&T->x, &T->x, &t7);
    f2_add(&t, &T->z, &t2);
    f2_sqr(&t, &t);
    f2_sub(&t, &t, &zz);
    f2_sub(&T->z, &t, &t3);
    f2_add(&t10, qy, &T->z);
    f2_sub(&t8, &t7, &T->x);
    f2_mul(&t8, &t8, &t6);
    f2_mul(&t0, &T->y, &t5);
    f2_add(&t0, &t0, &t0);
    f2_sub(&T->y, &t8, &t0);
    f2_sqr(&t10, &t10);
    f2_sub(&t10, &t10, &yy);
    f2_sqr(&t, &T->z);
    f2_sub(&t10, &t10, &t);
    f2_add(&t9, &t9, &t9);
    f2_sub(&t9, &t9, &t10);
    f2_add(&t10, &T->z, &T->z);
    f2_neg(&t6, &t6);
    f2_add(&t1, &t6, &t6);
    *l4 = t10; /* times y_P */
    *l1 = t1;  /* times x_P */
    *l0 = t9;
}
static void ml_line(fp12* f, const fp2* l0, const fp2* l1, const fp2* l4, const fp* px, const fp* py) {
    fp2 a, b;
    f2_mul_fp(&a, l1, px);
    f2_mul_fp(&b, l4, py);
    f12_mul_014(f, f, l0, &a, &b);
}
/* prod_i f_{|x|, Q_i}(P_i), conjugated (x < 0) */
static void miller_loop(fp12* f, int n, const fp* px, const fp* py, const fp2* qx, const fp2* qy) {
    g2j T[4];
    fp2 l0, l1, l4;
    for (int i = 0; i < n; i++) {
        T[i].x = qx[i];
        T[i].y = qy[i];
        T[i].z.c0 = ONE;
        T[i].z.c1 = FP_ZERO;
        T[i].inf = 0;
    }
    f12_one(f);
    for (int b = 62; b >= 0; b--) {
        f12_sqr(f, f);
        for (int i = 0; i < n; i++) {
            ml_dbl(&T[i], &l0, &l1, &l4);
            ml_line(f, &l0, &l1, &l4, &px[i], &py[i]);
        }
        if ((BLS_X_ABS >> b) & 1)
            for (int i = 0; i < n; i++) {
                ml_add(&T[i], &qx[i], &qy[i], &l0, &l1, &l4);
                ml_line(f, &l0, &l1, &l4, &px[i], &py[i]);
            }
    }
    f12_conj(f, f);
}
/* f^|x| then conjugate: f^x in the cyclotomic subgroup */
static void cyc_exp_x(fp12* r, const fp12* a) {
    fp12 acc = *a;
    for (int b = 62; b >= 0; b--) {
        f12_sqr(&acc, &acc);
        if ((BLS_X_ABS >> b) & 1) f12_mul(&acc, &acc, a);
    }
    f12_conj(r, &acc);
}
/* f^(3 (p^12 - 1) / r): easy part (p^6 - 1)(p^2 + 1), then the hard part through
 * 3 (p^4 - p^2 + 1) / r = (x - 1)^2 (x + p) (x^2 + p^2 - 1) + 3 */
static void final_exp(fp12* r, const fp12* f) {
    fp12 m, t, a, b, c, d;
    f12_inv(&t, f);
    f12_conj(&m, f);
    f12_mul(&m, &m, &t);  /* f^(p^6 - 1) */
    f12_frob(&t, &m);
    f12_frob(&t, &t);
    f12_mul(&m, &t, &m);  /* ^(p^2 + 1) */
    cyc_exp_x(&a, &m);
    f12_conj(&t, &m);
    f12_mul(&a, &a, &t);  /* m^(x-1) */
    cyc_exp_x(&t, &a);
    f12_conj(&d, &a);
    f12_mul(&a, &t, &d);  /* m^((x-1)^2) */
    cyc_exp_x(&b, &a);
    f12_frob(&t, &a);
    f12_mul(&b, &b, &t);  /* a^(x+p) */
    cyc_exp_x(&c, &b);
    cyc_exp_x(&c, &c);
    f12_frob(&t, &b);
    f12_frob(&t, &t);
    f12_mul(&c, &c, &t);
    f12_conj(&t, &b);
    f12_mul(&c, &c, &t);  /* b^(x^2 + p^2 - 1) */
    f12_sqr(&t, &m);
    f12_mul(&t, &t, &m);
    f12_mul(r, &c, &t);   /* * m^3 */
}
/* reference pairing: Q untwisted onto E(Fp12) by (x, y) -> (x / w^2, y / w^3), a plain affine
 * Miller loop there, then f^((p^12-1)/r) by square-and-multiply on the hard exponent */
static void fp12_from_fp(fp12* r, const fp* a) {
    memset(r, 0, sizeof(*r));
    r->c0.c0.c0 = *a;
}
static void untwist(fp12* X, fp12* Y, const fp2* qx, const fp2* qy) {
    fp12 w, w2, w3, t;
    memset(&w, 0, sizeof(w));
    w.c1.c0.c0 = ONE; /* w */
    f12_mul(&w2, &w, &w);
    f12_mul(&w3, &w2, &w);
    memset(&t, 0, sizeof(t));
    t.c0.c0 = *qx;
    f12_inv(&w2, &w2);
    f12_mul(X, &t, &w2);
    memset(&t, 0, sizeof(t));
    t.c0.c0 = *qy;
    f12_inv(&w3, &w3);
    f12_mul(Y, &t, &w3);
}
static void f12_sub(fp12* r, const fp12* a, const fp12* b) { f6_sub(&r->c0, &a->c0, &b->c0); f6_sub(&r->c1, &a->c1, &b->c1); }
static void f12_add(fp12* r, const fp12* a, const fp12* b) { f6_add(&r->c0, &a->c0, &b->c0); f6_add(&r->c1, &a->c1, &b->c1); }
static void pairing_ref(fp12* out, const fp* px, const fp* py, const fp2* qx, const fp2* qy) {
    fp12 Qx, Qy, Tx, Ty, Px, Py, f, lam, t, u, l;
    untwist(&Qx, &Qy, qx, qy);
    fp12_from_fp(&Px, px);
    fp12_from_fp(&Py, py);
    Tx = Qx;
    Ty = Qy;
    f12_one(&f);
    for (int b = 62; b >= 0; b--) {
        /* tangent at T: lambda = 3 x^2 / 2 y */
        f12_mul(&t, &Tx, &Tx);
        f12_add(&u, &t, &t);
        f12_add(&t, &u, &t);
        f12_add(&u, &Ty, &Ty);
        f12_inv(&u, &u);
        f12_mul(&lam, &t, &u);
        f12_sub(&t, &Py, &Ty);
        f12_sub(&u, &Px, &Tx);
        f12_mul(&u, &lam, &u);
        f12_sub(&l, &t, &u);
        f12_sqr(&f, &f);
        f12_mul(&f, &f, &l);
        fp12 x3;
        f12_mul(&x3, &lam, &lam);
        f12_sub(&x3, &x3, &Tx);
        f12_sub(&x3, &x3, &Tx);
        f12_sub(&t, &Tx, &x3);
        f12_mul(&t, &lam, &t);
        f12_sub(&Ty, &t, &Ty);
        Tx = x3;
        if ((BLS_X_ABS >> b) & 1) {
            f12_sub(&t, &Qy, &Ty);
            f12_sub(&u, &Qx, &Tx);
            f12_inv(&u, &u);
            f12_mul(&lam, &t, &u);
            f12_sub(&t, &Py, &Ty);
            f12_sub(&u, &Px, &Tx);
            f12_mul(&u, &lam, &u);
            f12_sub(&l, &t, &u);
            f12_mul(&f, &f, &l);
            f12_mul(&x3, &lam, &lam);
            f12_sub(&x3, &x3, &Tx);
            f12_sub(&x3, &x3, &Qx);
            f12_sub(&t, &Tx, &x3);
            f12_mul(&t, &lam, &t);
            f12_sub(&Ty, &t, &Ty);
            Tx = x3;
        }
    }
    f12_inv(&f, &f); /* f_{x,Q} = 1 / f_{|x|,Q} up to a vertical line */
    fp12 m;
    f12_inv(&t, &f);
    f12_conj(&m, &f);
    f12_mul(&m, &m, &t);
    f12_frob(&t, &m);
    f12_frob(&t, &t);
    f12_mul(&m, &t, &m);
    f12_pow_be(out, &m, HARD_EXP, 160);
}
static void f12_store(uint8_t out[576], const fp12* a) {
    const fp* c[12] = {&a->c0.c0.c0, &a->c0.c0.c1, &a->c0.c1.c0, &a->c0.c1.c1, &a->c0.c2.c0, &a->c0.c2.c1,
                       &a->c1.c0.c0, &a->c1.c0.c1, &a->c1.c1.c0, &a->c1.c1.c1, &a->c1.c2.c0, &a->c1.c2.c1};
    for (int i = 0; i < 12; i++) fp_to_be(out + 48 * i, c[i]);
}
static void f12_load(fp12* a, const uint8_t in[576]) {
    fp* c[12] = {&a->c0.c0.c0, &a->c0.c0.c1, &a->c0.c1.c0, &a->c0.c1.c1, &a->c0.c2.c0, &a->c0.c2.c1,
                 &a->c1.c0.c0, &a->c1.c0.c1, &a->c1.c1.c0, &a->c1.c1.c1, &a->c1.c2.c0, &a->c1.c2.c1};
    for (int i = 0; i < 12; i++) fp_from_be(c[i], in + 48 * i);
}

/* e(P0, Q0) * e(P1, Q1) == 1 with one shared Miller loop and final exponentiation */
static int pairing_check2(const g1j* P0, const g2j* Q0, const g1j* P1, const g2j* Q1) {
    fp px[2], py[2];
    fp2 qx[2], qy[2];
    int n = 0;
    const g1j* Ps[2] = {P0, P1};
    const g2j* Qs[2] = {Q0, Q1};
    for (int i = 0; i < 2; i++) {
        if (Ps[i]->inf || Qs[i]->inf) continue; /* e(O, Q) = e(P, O) = 1 */
        g1_affine(&px[n], &py[n], Ps[i]);
        g2_affine(&qx[n], &qy[n], Qs[i]);
        n++;
    }
    fp12 f, r;
    miller_loop(&f, n, px, py, qx, qy);
    final_exp(&r, &f);
    return f12_is_one(&r);
}

/* ------------------------------------------------------------------------------ public API */
void orb_pairing(const uint8_t P[96], const uint8_t Q[192], uint8_t out[576]) {
    INIT();
    g1j p1;
    g2j q2;
    g1_load(&p1, P);
    g2_load(&q2, Q);
    fp12 f, r;
    if (p1.inf || q2.inf) {
        f12_one(&r);
    } else {
        fp px, py;
        fp2 qx, qy;
        g1_affine(&px, &py, &p1);
        g2_affine(&qx, &qy, &q2);
        miller_loop(&f, 1, &px, &py, &qx, &qy);
        final_exp(&r, &f);
    }
    f12_store(out, &r);
}
void orb_pairing_ref(const uint8_t P[96], const uint8_t Q[192], uint8_t out[576]) {
    INIT();
    g1j p1;
    g2j q2;
    g1_load(&p1, P);
    g2_load(&q2, Q);
    fp12 r;
    if (p1.inf || q2.inf) {
        f12_one(&r);
    } else {
        fp px, py;
        fp2 qx, qy;
        g1_affine(&px, &py, &p1);
        g2_affine(&qx, &qy, &q2);
        pairing_ref(&r, &px, &py, &qx, &qy);
    }
    f12_store(out, &r);
}
void orb_gt_pow(const uint8_t in[576], const uint8_t* e, size_t e_len, uint8_t out[576]) {
    INIT();
    fp12 a, r;
    f12_load(&a, in);
    f12_pow_be(&r, &a, e, e_len);
    f12_store(out, &r);
}
void orb_gt_mul(const uint8_t a[576], const uint8_t b[576], uint8_t out[576]) {
    INIT();
    fp12 x, y, r;
    f12_load(&x, a);
    f12_load(&y, b);
    f12_mul(&r, &x, &y);
    f12_store(out, &r);
}
void orb_g1_mul(const uint8_t P[96], const uint8_t* k, size_t k_len, uint8_t out[96]) {
    INIT();
    g1j a, r;
    g1_load(&a, P);
    g1_mul_be(&r, &a, k, k_len);
    g1_store(out, &r);
}
void orb_g2_mul(const uint8_t Q[192], const uint8_t* k, size_t k_len, uint8_t out[192]) {
    INIT();
    g2j a, r;
    g2_load(&a, Q);
    g2_mul_be(&r, &a, k, k_len);
    g2_store(out, &r);
}
void orb_g1_add(const uint8_t A[96], const uint8_t B[96], uint8_t out[96]) {
    INIT();
    g1j a, b, r;
    g1_load(&a, A);
    g1_load(&b, B);
    g1_add(&r, &a, &b);
    g1_store(out, &r);
}
void orb_g2_add(const uint8_t A[192], const uint8_t B[192], uint8_t out[192]) {
    INIT();
    g2j a, b, r;
    g2_load(&a, A);
    g2_load(&b, B);
    g2_add(&r, &a, &b);
    g2_store(out, &r);
}
void orb_g1_compress(const uint8_t P[96], uint8_t out[48]) {
    INIT();
    g1j a;
    g1_load(&a, P);
    g1_compress_j(out, &a);
}
void orb_g2_compress(const uint8_t Q[192], uint8_t out[96]) {
    INIT();
    g2j a;
    g2_load(&a, Q);
    g2_compress_j(out, &a);
}
void orb_g1_generator(uint8_t out[96]) {
    INIT();
    g1j g;
    g1_gen(&g);
    g1_store(out, &g);
}
void orb_g2_generator(uint8_t out[192]) {
    INIT();
    g2j g;
    g2_gen(&g);
    g2_store(out, &g);
}
void orb_hard_exponent(uint8_t out[160]) {
    INIT();
    memcpy(out, HARD_EXP, 160);
}
int orb_g1_decompress(const uint8_t in[48], uint8_t out_xy[96], int* infinity) {
    INIT();
    g1j P;
    int rc = g1_decompress_j(&P, in);
    if (rc) return rc;
    if (infinity) *infinity = P.inf;
    if (out_xy) g1_store(out_xy, &P);
    return ORB_OK;
}
int orb_g2_decompress(const uint8_t in[96], uint8_t out_xy[192], int* infinity) {
    INIT();
    g2j Q;
    int rc = g2_decompress_j(&Q, in);
    if (rc) return rc;
    if (infinity) *infinity = Q.inf;
    if (out_xy) g2_store(out_xy, &Q);
    return ORB_OK;
}
int orb_g1_in_group(const uint8_t in[48]) {
    INIT();
    g1j P;
    return g1_decompress_j(&P, in) == ORB_OK && g1_in_group_j(&P);
}
int orb_g2_in_group(const uint8_t in[96]) {
    INIT();
    g2j Q;
    return g2_decompress_j(&Q, in) == ORB_OK && g2_in_group_j(&Q);
}
static int pk_load(g2j* Q, const uint8_t pk[96]) {
    int rc = g2_decompress_j(Q, pk);
    if (rc) return rc;
    if (Q->inf) return ORB_PK_INFINITY;
    if (!g2_in_group_j(Q)) return ORB_NOT_IN_GROUP;
    return ORB_OK;
}
static int sig_load(g1j* S, const uint8_t sig[48]) {
    int rc = g1_decompress_j(S, sig);
    if (rc) return rc;
    if (!S->inf && !g1_in_group_j(S)) return ORB_NOT_IN_GROUP;
    return ORB_OK;
}
int orb_pubkey_validate(const uint8_t pk[96]) {
    INIT();
    g2j Q;
    return pk_load(&Q, pk);
}
int orb_keygen(const uint8_t sk[32], uint8_t pk[96]) {
    INIT();
    g2j g, Q;
    g2_gen(&g);
    g2_mul_be(&Q, &g, sk, 32);
    g2_compress_j(pk, &Q);
    return Q.inf ? ORB_PK_INFINITY : ORB_OK;
}
int orb_sign(const uint8_t sk[32], const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len,
             uint8_t sig[48]) {
    INIT();
    g1j H, S;
    hash_to_g1_j(&H, msg, n, dst, dst_len);
    g1_mul_be(&S, &H, sk, 32);
    g1_compress_j(sig, &S);
    return ORB_OK;
}
static int verify_core(const g2j* pk, const uint8_t* msg, size_t n, const g1j* S, const uint8_t* dst,
                       size_t dst_len) {
    if (pk->inf) return ORB_PK_INFINITY;
    g1j H, negS = *S;
    hash_to_g1_j(&H, msg, n, dst, dst_len);
    if (!negS.inf) fp_neg(&negS.y, &negS.y);
    g2j g;
    g2_gen(&g);
    /* e(-sig, g2) * e(H(m), pk) == 1 */
    return pairing_check2(&negS, &g, &H, pk) ? ORB_OK : ORB_VERIFY_FAIL;
}
int orb_verify(const uint8_t pk[96], const uint8_t* msg, size_t n, const uint8_t sig[48], const uint8_t* dst,
               size_t dst_len) {
    INIT();
    g1j S;
    g2j Q;
    int rc = sig_load(&S, sig);
    if (rc) return rc;
    if ((rc = pk_load(&Q, pk))) return rc;
    return verify_core(&Q, msg, n, &S, dst, dst_len);
}
int orb_aggregate(size_t n, const uint8_t* sigs48, uint8_t out[48]) {
    INIT();
    if (n == 0) return ORB_AGGR_MISMATCH;
    g1j acc, S;
    acc.inf = 1;
    for (size_t i = 0; i < n; i++) {
        int rc = sig_load(&S, sigs48 + 48 * i);
        if (rc) return rc;
        g1_add(&acc, &acc, &S);
    }
    g1_compress_j(out, &acc);
    return ORB_OK;
}
int orb_aggregate_pubkeys(size_t n, const uint8_t* pks96, uint8_t out[96]) {
    INIT();
    if (n == 0) return ORB_AGGR_MISMATCH;
    g2j acc, Q;
    acc.inf = 1;
    for (size_t i = 0; i < n; i++) {
        int rc = pk_load(&Q, pks96 + 96 * i);
        if (rc) return rc;
        g2_add(&acc, &acc, &Q);
    }
    g2_compress_j(out, &acc);
    return ORB_OK;
}
int orb_fast_aggregate_verify(const uint8_t sig[48], size_t n_pks, const uint8_t* pks96, const uint8_t* msg,
                              size_t n, const uint8_t* dst, size_t dst_len) {
    INIT();
    g1j S;
    int rc = sig_load(&S, sig);
    if (rc) return rc;
    if (n_pks == 0) return ORB_AGGR_MISMATCH;
    g2j acc, Q;
    acc.inf = 1;
    for (size_t i = 0; i < n_pks; i++) {
        if ((rc = pk_load(&Q, pks96 + 96 * i))) return rc;
        g2_add(&acc, &acc, &Q);
    }
    return verify_core(&acc, msg, n, &S, dst, dst_len);
}

typedef struct {
    size_t lo, hi;
    const uint8_t *sigs, *pks, *msg, *dst;
    const uint32_t *pk_off, *pk_cnt, *msg_len;
    const uint64_t* msg_off;
    size_t dst_len;
    uint8_t* verdict;
} mt_job;
static void* mt_run(void* arg) {
    mt_job* j = (mt_job*)arg;
    for (size_t i = j->lo; i < j->hi; i++)
        j->verdict[i] = orb_fast_aggregate_verify(j->sigs + 48 * i, j->pk_cnt[i], j->pks + 96 * (size_t)j->pk_off[i],
                                                  j->msg + j->msg_off[i], j->msg_len[i], j->dst, j->dst_len) == ORB_OK;
    return NULL;
}
void orb_fast_aggregate_verify_mt(size_t n_items, const uint8_t* sigs48, const uint32_t* pk_off,
                                  const uint32_t* pk_cnt, const uint8_t* pks96, const uint8_t* msg_base,
                                  const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* dst,
                                  size_t dst_len, uint8_t* verdict, int threads) {
    INIT();
    if (threads < 1) threads = 1;
    pthread_t th[256];
    mt_job jobs[256];
    if (threads > 256) threads = 256;
    const size_t per = (n_items + (size_t)threads - 1) / (size_t)threads;
    int k = 0;
    for (int t = 0; t < threads; t++) {
        const size_t lo = (size_t)t * per, hi = lo + per < n_items ? lo + per : n_items;
        if (lo >= hi) break;
        jobs[k] = (mt_job){lo, hi, sigs48, pks96, msg_base, dst, pk_off, pk_cnt, msg_len, msg_off, dst_len, verdict};
        pthread_create(&th[k], NULL, mt_run, &jobs[k]);
        k++;
    }
    for (int t = 0; t < k; t++) pthread_join(th[t], NULL);
}

/* The same statuses as orb_fast_aggregate_verify item by item, with each key of the table decoded
 * and validated ONCE (as fastcrypto deserializes a public key once, crypto/src/lib.rs:29-33 ->
 * BLS12381PublicKey::from_bytes) instead of once per item: item i names keys[pk_idx[pk_off[i] + j]],
 * j < pk_cnt[i].  Items are split over `threads` host threads.  The CPU baseline of the BLS leg and
 * the checker of large GPU batches (100-node committees). */
typedef struct {
    size_t lo, hi;
    const uint8_t *sigs, *msg, *dst;
    const uint32_t *pk_off, *pk_cnt, *pk_idx, *msg_len;
    const uint64_t* msg_off;
    size_t dst_len;
    const g2j* keys;
    const int* key_st;
    int32_t* status;
} tab_job;
static void* tab_keys_run(void* arg) {
    tab_job* j = (tab_job*)arg;
    for (size_t k = j->lo; k < j->hi; k++) ((int*)j->key_st)[k] = pk_load((g2j*)&j->keys[k], j->sigs + 96 * k);
    return NULL;
}
static void* tab_items_run(void* arg) {
    tab_job* j = (tab_job*)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        g1j S;
        int rc = sig_load(&S, j->sigs + 48 * i);
        if (!rc && j->pk_cnt[i] == 0) rc = ORB_AGGR_MISMATCH;
        g2j acc;
        acc.inf = 1;
        for (uint32_t t = 0; !rc && t < j->pk_cnt[i]; t++) {
            const uint32_t k = j->pk_idx[j->pk_off[i] + t];
            if (j->key_st[k]) rc = j->key_st[k];
            else g2_add(&acc, &acc, &j->keys[k]);
        }
        if (!rc) rc = verify_core(&acc, j->msg + j->msg_off[i], j->msg_len[i], &S, j->dst, j->dst_len);
        j->status[i] = rc;
    }
    return NULL;
}
static void tab_parallel(void* (*fn)(void*), tab_job base, size_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    tab_job jobs[256];
    const size_t per = (n + (size_t)threads - 1) / (size_t)threads;
    int k = 0;
    for (int t = 0; t < threads; t++) {
        const size_t lo = (size_t)t * per, hi = lo + per < n ? lo + per : n;
        if (lo >= hi) break;
        jobs[k] = base;
        jobs[k].lo = lo;
        jobs[k].hi = hi;
        pthread_create(&th[k], NULL, fn, &jobs[k]);
        k++;
    }
    for (int t = 0; t < k; t++) pthread_join(th[t], NULL);
}
void orb_verify_items_keytab_mt(size_t n_keys, const uint8_t* keys96, size_t n_items, const uint8_t* sigs48,
                                const uint32_t* pk_off, const uint32_t* pk_cnt, const uint32_t* pk_idx,
                                const uint8_t* msg_base, const uint64_t* msg_off, const uint32_t* msg_len,
                                const uint8_t* dst, size_t dst_len, int32_t* status, int threads) {
    INIT();
    g2j* keys = (g2j*)calloc(n_keys ? n_keys : 1, sizeof(g2j));
    int* kst = (int*)calloc(n_keys ? n_keys : 1, sizeof(int));
    tab_job b = {0, 0, keys96, msg_base, dst, pk_off, pk_cnt, pk_idx, msg_len, msg_off, dst_len, keys, kst, status};
    tab_parallel(tab_keys_run, b, n_keys, threads);  /* .sigs carries the key bytes for this pass */
    b.sigs = sigs48;
    tab_parallel(tab_items_run, b, n_items, threads);
    free(keys);
    free(kst);
}
