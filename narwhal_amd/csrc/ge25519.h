// ge25519.h -- twisted Edwards (a = -1) group operations on GF(2^255-19), gfx950 layout.
//
// Restates the point layer of curve25519-dalek-ng 4.1.1 (extended coordinates, the
// Hisil-Wong-Carter-Dawson formulas dalek uses; /root/reference/Cargo.lock:1166-1177) over
// the radix-2^25.5 field of fe25519.h.  Representations:
//   ge_p3      extended (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z
//   ge_p2      projective (X:Y:Z)
//   ge_p1p1    completed ((X:Z),(Y:T)), x = X/Z, y = Y/T
//   ge_cached  projective Niels (Y+X, Y-X, 2Z, 2dT)   -- per-signature tables
//   ge_precomp affine Niels (y+x, y-x, 2dxy)          -- basepoint table
// Every output limb magnitude is tracked against the bounds documented in fe25519.h.
#pragma once
#include "fe25519.h"

namespace nwv {

struct ge_p3 { fe X, Y, Z, T; };
struct ge_p2 { fe X, Y, Z; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z2, T2d; };
struct ge_precomp { fe ypx, ymx, xy2d; };

NWV_HD ge_p2 ge_p2_identity() { return ge_p2{fe_zero(), fe_one(), fe_one()}; }
NWV_HD ge_p3 ge_p3_identity() { return ge_p3{fe_zero(), fe_one(), fe_one(), fe_zero()}; }
NWV_HD ge_cached ge_cached_identity() {
    return ge_cached{fe_one(), fe_one(), fe_small(2), fe_zero()};
}

NWV_HD ge_p3 ge_p1p1_to_p3(const ge_p1p1& c) {
    return ge_p3{fe_mul(c.X, c.T), fe_mul(c.Y, c.Z), fe_mul(c.Z, c.T), fe_mul(c.X, c.Y)};
}
NWV_HD ge_p2 ge_p1p1_to_p2(const ge_p1p1& c) {
    return ge_p2{fe_mul(c.X, c.T), fe_mul(c.Y, c.Z), fe_mul(c.Z, c.T)};
}
NWV_HD ge_p2 ge_p3_to_p2(const ge_p3& p) { return ge_p2{p.X, p.Y, p.Z}; }

// ProjectivePoint::double -> CompletedPoint (4 squarings); input limbs must be carried
NWV_HD ge_p1p1 ge_p2_dbl(const ge_p2& p) {
    fe XX = fe_sq(p.X);
    fe YY = fe_sq(p.Y);
    fe ZZ = fe_sq(p.Z);
    fe ZZ2 = fe_carry(fe_add(ZZ, ZZ));
    fe XpY2 = fe_sq(fe_add(p.X, p.Y));
    ge_p1p1 r;
    r.Y = fe_carry(fe_add(YY, XX));   // YY + XX
    r.Z = fe_carry(fe_sub(YY, XX));   // YY - XX
    r.X = fe_sub(XpY2, r.Y);          // (X+Y)^2 - YY - XX
    r.T = fe_sub(ZZ2, r.Z);           // 2Z^2 - (YY - XX)
    return r;
}

// EdwardsPoint + ProjectiveNielsPoint
NWV_HD ge_p1p1 ge_add(const ge_p3& p, const ge_cached& q) {
    fe PP = fe_mul(fe_add(p.Y, p.X), q.YpX);
    fe MM = fe_mul(fe_sub(p.Y, p.X), q.YmX);
    fe TT2d = fe_mul(p.T, q.T2d);
    fe ZZ2 = fe_mul(p.Z, q.Z2);
    return ge_p1p1{fe_sub(PP, MM), fe_add(PP, MM), fe_add(ZZ2, TT2d), fe_sub(ZZ2, TT2d)};
}
NWV_HD ge_p1p1 ge_sub(const ge_p3& p, const ge_cached& q) {
    fe PM = fe_mul(fe_add(p.Y, p.X), q.YmX);
    fe MP = fe_mul(fe_sub(p.Y, p.X), q.YpX);
    fe TT2d = fe_mul(p.T, q.T2d);
    fe ZZ2 = fe_mul(p.Z, q.Z2);
    return ge_p1p1{fe_sub(PM, MP), fe_add(PM, MP), fe_sub(ZZ2, TT2d), fe_add(ZZ2, TT2d)};
}
// EdwardsPoint + AffineNielsPoint (mixed addition, Z2 = 1)
NWV_HD ge_p1p1 ge_madd(const ge_p3& p, const ge_precomp& q) {
    fe PP = fe_mul(fe_add(p.Y, p.X), q.ypx);
    fe MM = fe_mul(fe_sub(p.Y, p.X), q.ymx);
    fe Txy2d = fe_mul(p.T, q.xy2d);
    fe Z2 = fe_carry(fe_add(p.Z, p.Z));
    return ge_p1p1{fe_sub(PP, MM), fe_add(PP, MM), fe_add(Z2, Txy2d), fe_sub(Z2, Txy2d)};
}
NWV_HD ge_p1p1 ge_msub(const ge_p3& p, const ge_precomp& q) {
    fe PM = fe_mul(fe_add(p.Y, p.X), q.ymx);
    fe MP = fe_mul(fe_sub(p.Y, p.X), q.ypx);
    fe Txy2d = fe_mul(p.T, q.xy2d);
    fe Z2 = fe_carry(fe_add(p.Z, p.Z));
    return ge_p1p1{fe_sub(PM, MP), fe_add(PM, MP), fe_sub(Z2, Txy2d), fe_add(Z2, Txy2d)};
}

// Table-driven additions with lazily loaded operands.  A table entry holds the point and
// the negation of its last coordinate, so a signed digit only changes which words are read
// (Y+X <-> Y-X swap, 2dT -> -2dT) and no selects are executed:
//   cached entry  (50 words): Y+X | Y-X | 2Z | 2dT | -2dT
//   precomp entry (40 words): y+x | y-x | 2dxy | -2dxy
static constexpr int CACHED_ENTRY_WORDS = 50;
static constexpr int PRECOMP_ENTRY_WORDS = 40;

NWV_HD fe load_fe(const uint32_t* src) {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = src[i];
    return r;
}
NWV_HD void store_fe(uint32_t* dst, const fe& a) {
#pragma unroll
    for (int i = 0; i < 10; i++) dst[i] = a.v[i];
}

// p + (neg ? -Q : Q), Q a cached entry
NWV_HD ge_p1p1 ge_add_entry(const ge_p3& p, const uint32_t* e, bool neg) {
    fe TT2d = fe_mul(p.T, load_fe(e + (neg ? 40 : 30)));
    fe ZZ2 = fe_mul(p.Z, load_fe(e + 20));
    fe PP = fe_mul(fe_add(p.Y, p.X), load_fe(e + (neg ? 10 : 0)));
    fe MM = fe_mul(fe_sub(p.Y, p.X), load_fe(e + (neg ? 0 : 10)));
    return ge_p1p1{fe_sub(PP, MM), fe_add(PP, MM), fe_add(ZZ2, TT2d), fe_sub(ZZ2, TT2d)};
}
// the 40 words of a cached entry that p + (neg ? -Q : Q) reads (Y+X, Y-X swapped and -2dT for -Q)
NWV_HD void load_cached_entry(const uint32_t* e, bool neg, uint32_t out[40]) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        out[i] = e[(neg ? 10 : 0) + i];
        out[10 + i] = e[(neg ? 0 : 10) + i];
        out[20 + i] = e[20 + i];
        out[30 + i] = e[(neg ? 40 : 30) + i];
    }
}
// p + Q', Q' the words load_cached_entry fetched
NWV_HD ge_p1p1 ge_add_loaded(const ge_p3& p, const uint32_t q[40]) {
    fe TT2d = fe_mul(p.T, load_fe(q + 30));
    fe ZZ2 = fe_mul(p.Z, load_fe(q + 20));
    fe PP = fe_mul(fe_add(p.Y, p.X), load_fe(q));
    fe MM = fe_mul(fe_sub(p.Y, p.X), load_fe(q + 10));
    return ge_p1p1{fe_sub(PP, MM), fe_add(PP, MM), fe_add(ZZ2, TT2d), fe_sub(ZZ2, TT2d)};
}
// p + (neg ? -Q : Q), Q a precomp entry (mixed addition)
NWV_HD ge_p1p1 ge_madd_entry(const ge_p3& p, const uint32_t* e, bool neg) {
    fe Txy2d = fe_mul(p.T, load_fe(e + (neg ? 30 : 20)));
    fe Z2 = fe_carry(fe_add(p.Z, p.Z));
    fe PP = fe_mul(fe_add(p.Y, p.X), load_fe(e + (neg ? 10 : 0)));
    fe MM = fe_mul(fe_sub(p.Y, p.X), load_fe(e + (neg ? 0 : 10)));
    return ge_p1p1{fe_sub(PP, MM), fe_add(PP, MM), fe_add(Z2, Txy2d), fe_sub(Z2, Txy2d)};
}
NWV_HD void store_cached_entry(uint32_t* e, const ge_cached& c) {
    store_fe(e, c.YpX);
    store_fe(e + 10, c.YmX);
    store_fe(e + 20, c.Z2);
    store_fe(e + 30, c.T2d);
    store_fe(e + 40, fe_carry(fe_neg(c.T2d)));
}
NWV_HD void store_precomp_entry(uint32_t* e, const ge_precomp& c) {
    store_fe(e, c.ypx);
    store_fe(e + 10, c.ymx);
    store_fe(e + 20, c.xy2d);
    store_fe(e + 30, fe_carry(fe_neg(c.xy2d)));
}

NWV_HD ge_cached ge_p3_to_cached(const ge_p3& p) {
    return ge_cached{fe_carry(fe_add(p.Y, p.X)), fe_carry(fe_sub(p.Y, p.X)),
                     fe_carry(fe_add(p.Z, p.Z)), fe_mul(p.T, fe_d2())};
}
// conditional negation of a cached point: -(x, y) = (-x, y): swap Y+X / Y-X, negate 2dT
NWV_HD ge_cached ge_cached_cneg(const ge_cached& q, bool neg) {
    ge_cached r;
    r.YpX = fe_select(q.YpX, q.YmX, neg);
    r.YmX = fe_select(q.YmX, q.YpX, neg);
    r.Z2 = q.Z2;
    r.T2d = fe_select(q.T2d, fe_carry(fe_neg(q.T2d)), neg);
    return r;
}
NWV_HD ge_precomp ge_precomp_cneg(const ge_precomp& q, bool neg) {
    ge_precomp r;
    r.ypx = fe_select(q.ypx, q.ymx, neg);
    r.ymx = fe_select(q.ymx, q.ypx, neg);
    r.xy2d = fe_select(q.xy2d, fe_carry(fe_neg(q.xy2d)), neg);
    return r;
}

NWV_HD ge_p3 ge_p3_dbl(const ge_p3& p) { return ge_p1p1_to_p3(ge_p2_dbl(ge_p3_to_p2(p))); }

// CompressedEdwardsY::decompress (dalek), SURVEY.md Appendix A "Decode":
// y taken from the 255 low bits (values >= p accepted), x = sqrt_ratio_i(y^2-1, dy^2+1),
// reject on non-square, negate on the sign bit ("negative zero" is accepted as x = 0).
NWV_HD void ge_uv_from_words(const uint32_t w[8], fe& y, fe& u, fe& v) {
    y = fe_from_words(w);
    fe yy = fe_sq(y);
    u = fe_carry(fe_sub(yy, fe_one()));
    v = fe_carry(fe_add(fe_mul(yy, fe_d()), fe_one()));
}
NWV_HD void words_pin(uint32_t w[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("" : "+v"(w[i]));
#else
    (void)w;
#endif
}
// sqrt_ratio_i(u, v) with u = y^2 - 1, v = d y^2 + 1 inlined.  Only the 8 input words and the
// exponentiation state are live across the 250-squaring chain: y, u, v and u v^3 are
// recomputed after it (5 multiplies) instead of occupying 40 VGPRs through it.
// The decompression in three pieces, so that the exponentiation can run elsewhere (on 16-lane
// rows for small batches, k_msm_prep): the prelude u v^7, the power (u v^7)^((p-5)/8), the rest.
NWV_HD fe ge_decompress_pre(const uint32_t w[8]) {
    fe y, u, v;
    ge_uv_from_words(w, y, u, v);
    fe v3 = fe_mul(fe_sq(v), v);
    return fe_mul(u, fe_mul(fe_sq(v3), v));
}
NWV_HD bool ge_decompress_post(const uint32_t w_in[8], fe pw, ge_p3& out);
NWV_HD bool ge_decompress(const uint32_t w_in[8], ge_p3& out) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = w_in[i];
    const fe pw = fe_pow_p58(ge_decompress_pre(w));
    return ge_decompress_post(w, pw, out);
}
NWV_HD bool ge_decompress_post(const uint32_t w_in[8], fe pw, ge_p3& out) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = w_in[i];
    fe_pin(pw);
    words_pin(w);
    fe y, u, v;
    ge_uv_from_words(w, y, u, v);
    fe r = fe_mul(fe_mul(u, fe_mul(fe_sq(v), v)), pw);  // (u v^3)(u v^7)^((p-5)/8)
    fe check = fe_carry(fe_mul(v, fe_sq(r)));
    const bool correct = fe_is_zero(fe_sub(check, u));
    const bool flipped = fe_is_zero(fe_add(check, u));
    fe_pin(u);
    const bool flipped_i = fe_is_zero(fe_add(check, fe_mul(u, fe_sqrtm1())));
    fe_pin(r);
    r = fe_select(r, fe_mul(r, fe_sqrtm1()), flipped || flipped_i);
    r = fe_select(r, fe_carry(fe_neg(r)), fe_is_negative(r) != 0);
    // sign bit of the encoding; x = 0 with sign 1 ("negative zero") stays x = 0
    fe x = fe_select(r, fe_carry(fe_neg(r)), (w[7] >> 31) != 0);
    out.X = x;
    out.Y = y;
    out.Z = fe_one();
    out.T = fe_mul(x, y);
    return correct || flipped;
}

// affine (x, y) -> compressed words (y with the sign of x in bit 255)
NWV_HD void ge_compress(const ge_p3& p, uint32_t w[8]) {
    fe zi = fe_invert(p.Z);
    fe x = fe_mul(p.X, zi);
    fe y = fe_mul(p.Y, zi);
    fe_freeze(y, w);
    w[7] |= fe_is_negative(x) << 31;
}

NWV_HD ge_precomp ge_p3_to_precomp(const ge_p3& p) {
    fe zi = fe_invert(p.Z);
    fe x = fe_mul(p.X, zi);
    fe y = fe_mul(p.Y, zi);
    return ge_precomp{fe_carry(fe_add(y, x)), fe_carry(fe_sub(y, x)),
                      fe_mul(fe_mul(x, y), fe_d2())};
}

// identity test of a completed point: x = X/Z = 0 and y = Y/T = 1
NWV_HD bool ge_p1p1_is_identity(const ge_p1p1& c) {
    return fe_is_zero(c.X) && fe_eq(c.Y, c.T);
}

// Ed25519 basepoint B, compressed (y = 4/5, sign 0)
NWV_HD void ge_basepoint_words(uint32_t w[8]) {
    w[0] = 0x66666658u;
    for (int i = 1; i < 8; i++) w[i] = 0x66666666u;
}

}  // namespace nwv
