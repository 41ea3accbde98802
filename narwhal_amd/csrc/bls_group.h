// bls_group.h -- BLS12-381 Fp12 arithmetic spread over a GROUP of 8 lanes (gfx950), for the Miller
// loops and final exponentiations of the pairing check.
//
// One lane holding a whole Fp12 (12 x 14 limbs = 168 VGPRs per operand) spills to scratch on every
// tower product, and the product's 54 Fp multiplications run one after another.  Here an Fp12 is
// read as Fp2[W] / (W^6 - xi) (W = w, so v = W^2): lane k of a group holds the coefficient of W^k
// (k = 0..5; lanes 6, 7 shadow lanes 0, 1), so an Fp12 product is a length-6 cyclic convolution
// with the xi wrap -- every lane computes its own output coefficient from six Fp2 products of
// operands exchanged through LDS: 18 Fp multiplications deep instead of 54, with everything in
// registers.  The sparse line product is 3 Fp2 products deep, the Granger-Scott cyclotomic square
// 3 Fp2 squarings deep (lane k computes one of the six Fp4 half-products), the Frobenius map one
// Fp2 product.  The Miller loop's G2 doubling and its line run as rounds of independent Fp
// products over the lanes (g_ml_dbl); its G2 additions are computed redundantly by every lane.
//
// Tower slot <-> W power: k 0 c0.c0, 1 c1.c0, 2 c0.c1, 3 c1.c1, 4 c0.c2, 5 c1.c2 (bls381.h).
//
// The same algorithms compile for the host (tests/hostemu): there a G12 holds all six coefficients
// and each group operation loops over k with the same per-coefficient code, so the host build
// checks the group arithmetic against bls381.h's single-lane tower bit for bit.
#pragma once
#include "bls381.h"

// the lane-group form everywhere except in the CPU test build, which defines BLS_GROUP_HOST_EMU
// (nwv_bls.hip's host compilation pass only analyses the kernels, it never runs them)
#if !defined(BLS_GROUP_HOST_EMU)
#define BLS_GDEV 1
#endif

namespace bls {

constexpr int GRP = 8;                   // lanes per group
constexpr int F2W = 2 * NL;              // u32 words of an Fp2
// one group's LDS exchange area: operand A slots [GRP][F2W], B slots, and room for the 18 Fp
// products of g_cyc_sqr behind the A slots (GRP F2W + 18 NL = 476 words)
constexpr int GX_WORDS = 480;
static_assert(GX_WORDS >= 2 * GRP * F2W && GX_WORDS >= GRP * F2W + 18 * NL, "group LDS area");

NWV_HD void st_fp(uint32_t* o, const fp& a) { for (int j = 0; j < NL; j++) o[j] = a.l[j]; }
NWV_HD fp ld_fp(const uint32_t* o) { fp a; for (int j = 0; j < NL; j++) a.l[j] = o[j]; return a; }
NWV_HD void st_f2(uint32_t* o, const fp2& a) {
    st_fp(o, a.c0);
    st_fp(o + NL, a.c1);
}
NWV_HD fp2 ld_f2(const uint32_t* o) {
    fp2 a;
    a.c0 = ld_fp(o);
    a.c1 = ld_fp(o + NL);
    return a;
}

#ifdef BLS_GDEV
__constant__ uint32_t c_gamma[6][2][NL] = BLS_GAMMA;
#endif
// Frobenius coefficient of W^k (gamma_k of bls381.h; k = 0: 1)
NWV_HD fp2 w_gamma(int k) {
#ifdef BLS_GDEV
    fp2 r;
    for (int j = 0; j < NL; j++) {
        r.c0.l[j] = c_gamma[k][0][j];
        r.c1.l[j] = c_gamma[k][1][j];
    }
    return k == 0 ? f2_one() : r;
#else
    return k == 0 ? f2_one() : gamma_k(k);
#endif
}

// ---- per-coefficient arithmetic (shared by the device and host forms) ----------------------
// c_k of a * b: sum_r a_{k-r} b_r, the wrapped terms (k < r) times xi
template <class A, class B>
NWV_HD fp2 coef_mul(int k, const A& a, const B& b) {
    fp2 acc = f2_zero();
#pragma unroll 1
    for (int r = 0; r < 6; r++) {
        const int i = k >= r ? k - r : k - r + 6;
        fp2 t = f2_mul(a(i), b(r));
        if (k < r) t = f2_mul_xi(t);
        acc = f2_add(acc, t);
    }
    return acc;
}
// c_k of a^2 in four Fp2 products instead of six: the terms a_r a_s and a_s a_r of coef_mul are
// equal (and wrap together: r + s = k or k + 6), so c_k is the squares a_h^2 + a_{h+3}^2 plus twice
// the pairs (h+1, h+5), (h+2, h+4) for k = 2h, and twice the pairs (h, h+1), (h+2, h+5),
// (h+3, h+4) for k = 2h+1 (indices mod 6).  Every lane runs the same four products (the odd
// lanes' fourth has weight 0), so the lanes of a group do not diverge.
template <class A>
NWV_HD fp2 coef_sqr(int k, const A& a) {
    const int h = k >> 1;
    const bool odd = (k & 1) != 0;
    auto m6 = [](int x) { return x >= 6 ? x - 6 : x; };
    fp2 acc = f2_zero();
#pragma unroll 1
    for (int m = 0; m < 4; m++) {
        int i, j;
        if (odd) {
            i = m6(h + (m == 0 ? 0 : m == 1 ? 2 : 3));
            j = m6(h + (m == 0 ? 1 : m == 1 ? 5 : 4));
        } else {
            i = m6(h + (m == 0 ? 0 : m == 1 ? 3 : m == 2 ? 1 : 2));
            j = m6(h + (m == 0 ? 0 : m == 1 ? 3 : m == 2 ? 5 : 4));
        }
        fp2 t = f2_mul(a(i), a(j));
        if (i + j >= 6) t = f2_mul_xi(t);
        const int w = odd ? (m < 3 ? 2 : 0) : (m < 2 ? 1 : 2);
        if (w != 0) acc = f2_add(acc, t);
        if (w == 2) acc = f2_add(acc, t);
    }
    return acc;
}
// c_k of a * (L0 + L2 W^2 + L3 W^3): the Miller loop's sparse line product
template <class A>
NWV_HD fp2 coef_line(int k, const A& a, const fp2& L0, const fp2& L2, const fp2& L3) {
    const int i2 = k >= 2 ? k - 2 : k + 4, i3 = k >= 3 ? k - 3 : k + 3;
    fp2 t2 = f2_mul(a(i2), L2);
    if (k < 2) t2 = f2_mul_xi(t2);
    fp2 t3 = f2_mul(a(i3), L3);
    if (k < 3) t3 = f2_mul_xi(t3);
    return f2_add(f2_add(f2_mul(a(k), L0), t2), t3);
}
// c_k of the Granger-Scott cyclotomic square (f12_cyc_sqr): the Fp4 pairs are (W^0, W^3),
// (W^1, W^4), (W^2, W^5); lane k takes one output of one pair's square
//   fp4_sqr(a, b) = (xi b^2 + a^2, (a + b)^2 - a^2 - b^2)
// k -> (pair, output): 0 (0,3).0, 1 (2,5).1 * xi, 2 (1,4).0, 3 (0,3).1, 4 (2,5).0, 5 (1,4).1;
// then z_k' = 2 (o - z_k) + o (even k) or 2 (o + z_k) + o (odd k)
template <class A>
NWV_HD fp2 coef_cyc_sqr(int k, const A& a) {
    const int p = (k == 0 || k == 3) ? 0 : (k == 2 || k == 5) ? 1 : 2;
    const bool second = (k & 1) != 0;
    const fp2 x = a(p), y = a(p + 3);
    const fp2 t0 = f2_sqr(x), t1 = f2_sqr(y), s = f2_sqr(f2_add(x, y));
    fp2 o = second ? f2_sub(f2_sub(s, t0), t1) : f2_add(f2_mul_xi(t1), t0);
    if (k == 1) o = f2_mul_xi(o);
    const fp2 z = a(k);
    return second ? f2_add(f2_dbl(f2_add(o, z)), o) : f2_add(f2_dbl(f2_sub(o, z)), o);
}
// tower slot of W^k in an fp12
NWV_HD fp2& w_slot(fp12& f, int k) {
    switch (k) {
        case 0: return f.c0.c0;
        case 1: return f.c1.c0;
        case 2: return f.c0.c1;
        case 3: return f.c1.c1;
        case 4: return f.c0.c2;
        default: return f.c1.c2;
    }
}

// ---- the group element and its operations ----------------------------------------------------
#ifdef BLS_GDEV

struct GCtx {
    uint32_t* xa;  // this group's LDS exchange area (GX_WORDS): A slots [GRP][F2W], then B slots
    int slot;      // this lane's slot in the group (0..7)
    int k;         // its coefficient (slot mod 6)
};
struct G12 {
    fp2 v;  // this lane's coefficient of W^k
};
__device__ inline GCtx g_ctx(uint32_t* lds_base) {
    GCtx g;
    const int lane = (int)(threadIdx.x & 63);
    g.slot = lane & (GRP - 1);
    g.k = g.slot < 6 ? g.slot : g.slot - 6;
    g.xa = lds_base + (size_t)(threadIdx.x / GRP) * GX_WORDS;
    return g;
}
// LDS writes of the group visible to its reads (one wave: in-order LDS; fence the compiler)
__device__ inline void g_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
struct GRead {
    const uint32_t* base;
    __device__ fp2 operator()(int i) const { return ld_f2(base + i * F2W); }
};
__device__ inline void g_put(const GCtx& g, int which, const fp2& x) { st_f2(g.xa + which * GRP * F2W + g.slot * F2W, x); }
__device__ inline GRead g_reader(const GCtx& g, int which) { return GRead{g.xa + which * GRP * F2W}; }

__device__ inline G12 g_mul(const GCtx& g, const G12& a, const G12& b) {
    g_sync();
    g_put(g, 0, a.v);
    g_put(g, 1, b.v);
    g_sync();
    return G12{coef_mul(g.k, g_reader(g, 0), g_reader(g, 1))};
}
__device__ inline G12 g_sqr(const GCtx& g, const G12& a) {
    g_sync();
    g_put(g, 0, a.v);
    g_sync();
    return G12{coef_sqr(g.k, g_reader(g, 0))};
}
__device__ inline G12 g_mul_line(const GCtx& g, const G12& a, const fp2& L0, const fp2& L2, const fp2& L3) {
    g_sync();
    g_put(g, 0, a.v);
    g_sync();
    return G12{coef_line(g.k, g_reader(g, 0), L0, L2, L3)};
}
// The Granger-Scott square's 18 Fp products -- three Fp2 squarings x^2, y^2, (x + y)^2 of each
// Fp4 pair (W^p, W^(p+3)), two products each -- spread over the group in three rounds instead of
// six products on every lane; then lane k combines its pair's squares exactly as coef_cyc_sqr.
__device__ inline G12 g_cyc_sqr(const GCtx& g, const G12& a) {
    g_sync();
    g_put(g, 0, a.v);
    g_sync();
    const GRead rd = g_reader(g, 0);
    uint32_t* R = g.xa + GRP * F2W;  // product q at R + q NL (q = 6 pair + 2 square + part)
#pragma unroll 1
    for (int r = 0; r < 3; r++) {
        const int q = r * GRP + g.slot;
        if (r < 2 || g.slot < 2) {  // 18 products: the last round uses two lanes
            const int p = q / 6, sq = (q % 6) >> 1;
            const fp2 x = rd(p), y = rd(p + 3);
            const fp2 v = sq == 0 ? x : sq == 1 ? y : f2_add(x, y);
            const bool part = (q & 1) != 0;  // f2_sqr: (c0 + c1)(c0 - c1), then c0 c1
            const fp pr = fp_mul(part ? v.c0 : fp_add(v.c0, v.c1), part ? v.c1 : fp_sub(v.c0, v.c1));
            st_fp(R + q * NL, pr);
        }
    }
    g_sync();
    const int k = g.k;
    const int p = (k == 0 || k == 3) ? 0 : (k == 2 || k == 5) ? 1 : 2;
    const uint32_t* Rp = R + 6 * p * NL;
    const fp2 t0 = fp2{ld_fp(Rp), fp_dbl(ld_fp(Rp + NL))};
    const fp2 t1 = fp2{ld_fp(Rp + 2 * NL), fp_dbl(ld_fp(Rp + 3 * NL))};
    const fp2 s = fp2{ld_fp(Rp + 4 * NL), fp_dbl(ld_fp(Rp + 5 * NL))};
    const bool second = (k & 1) != 0;
    fp2 o = second ? f2_sub(f2_sub(s, t0), t1) : f2_add(f2_mul_xi(t1), t0);
    if (k == 1) o = f2_mul_xi(o);
    const fp2 z = a.v;
    return G12{second ? f2_add(f2_dbl(f2_add(o, z)), o) : f2_add(f2_dbl(f2_sub(o, z)), o)};
}
__device__ inline G12 g_conj(const GCtx& g, const G12& a) { return G12{(g.k & 1) ? f2_neg(a.v) : a.v}; }
__device__ inline G12 g_frob(const GCtx& g, const G12& a) { return G12{f2_mul(f2_conj(a.v), w_gamma(g.k))}; }
__device__ inline G12 g_one(const GCtx& g) { return G12{g.k == 0 ? f2_one() : f2_zero()}; }
__device__ inline fp12 g_gather(const GCtx& g, const G12& a) {
    g_sync();
    g_put(g, 0, a.v);
    g_sync();
    const GRead rd = g_reader(g, 0);
    fp12 f;
    for (int k = 0; k < 6; k++) w_slot(f, k) = rd(k);
    return f;
}
__device__ inline G12 g_scatter(const GCtx& g, const fp12& f) {
    fp2 r = f.c0.c0;  // a select chain: no dynamically indexed private array
    if (g.k == 1) r = f.c1.c0;
    if (g.k == 2) r = f.c0.c1;
    if (g.k == 3) r = f.c1.c1;
    if (g.k == 4) r = f.c0.c2;
    if (g.k == 5) r = f.c1.c2;
    return G12{r};
}
// coefficient 0 of the group's element, on every lane
__device__ inline fp2 g_coef0(const GCtx& g, const G12& a) {
    g_sync();
    g_put(g, 0, a.v);
    g_sync();
    return g_reader(g, 0)(0);
}
__device__ inline G12 g_scale(const GCtx& g, const G12& a, const fp2& s) { return G12{f2_mul(a.v, s)}; }
// every lane of the group: a == 1
__device__ inline bool g_is_one(const GCtx& g, const G12& a) {
    const bool ok = g.k == 0 ? f2_eq(a.v, f2_one()) : f2_is_zero(a.v);
    const uint64_t bad = __ballot(!ok);
    const int first = (int)(threadIdx.x & 63) & ~(GRP - 1);
    return ((bad >> first) & 0x3fu) == 0;
}
// the group's element to / from memory in W order (6 x F2W words); lanes 6, 7 do not store
__device__ inline void g_store(const GCtx& g, uint32_t* o, const G12& a) {
    if (g.slot < 6) st_f2(o + g.k * F2W, a.v);
}
__device__ inline G12 g_load(const GCtx& g, const uint32_t* o) { return G12{ld_f2(o + g.k * F2W)}; }

#else  // host form: all six coefficients, the same per-coefficient code

struct GCtx {};
struct G12 {
    fp2 v[6];
};
struct HRead {
    const fp2* v;
    fp2 operator()(int i) const { return v[i]; }
};
inline G12 g_mul(const GCtx&, const G12& a, const G12& b) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = coef_mul(k, HRead{a.v}, HRead{b.v});
    return c;
}
inline G12 g_sqr(const GCtx&, const G12& a) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = coef_sqr(k, HRead{a.v});
    return c;
}
inline G12 g_mul_line(const GCtx&, const G12& a, const fp2& L0, const fp2& L2, const fp2& L3) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = coef_line(k, HRead{a.v}, L0, L2, L3);
    return c;
}
inline G12 g_cyc_sqr(const GCtx&, const G12& a) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = coef_cyc_sqr(k, HRead{a.v});
    return c;
}
inline G12 g_conj(const GCtx&, const G12& a) {
    G12 c = a;
    for (int k = 1; k < 6; k += 2) c.v[k] = f2_neg(a.v[k]);
    return c;
}
inline G12 g_frob(const GCtx&, const G12& a) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = f2_mul(f2_conj(a.v[k]), w_gamma(k));
    return c;
}
inline G12 g_one(const GCtx&) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = k == 0 ? f2_one() : f2_zero();
    return c;
}
inline fp12 g_gather(const GCtx&, const G12& a) {
    fp12 f;
    for (int k = 0; k < 6; k++) w_slot(f, k) = a.v[k];
    return f;
}
inline G12 g_scatter(const GCtx&, const fp12& f) {
    fp12 t = f;
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = w_slot(t, k);
    return c;
}
inline fp2 g_coef0(const GCtx&, const G12& a) { return a.v[0]; }
inline G12 g_scale(const GCtx&, const G12& a, const fp2& s) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = f2_mul(a.v[k], s);
    return c;
}
inline bool g_is_one(const GCtx&, const G12& a) {
    bool ok = f2_eq(a.v[0], f2_one());
    for (int k = 1; k < 6; k++) ok = ok && f2_is_zero(a.v[k]);
    return ok;
}
inline void g_store(const GCtx&, uint32_t* o, const G12& a) {
    for (int k = 0; k < 6; k++) st_f2(o + k * F2W, a.v[k]);
}
inline G12 g_load(const GCtx&, const uint32_t* o) {
    G12 c;
    for (int k = 0; k < 6; k++) c.v[k] = ld_f2(o + k * F2W);
    return c;
}

#endif

// ---- pairing building blocks over a group ---------------------------------------------------
// device-only in the lane-group form (they use LDS and the lane id), plain host code in the
// CPU test build
#ifdef BLS_GDEV
#define G_HD __device__ inline
#define G_NOINLINE __device__ __attribute__((noinline))
#else
#define G_HD inline
#define G_NOINLINE __attribute__((noinline))
#endif
// ---- independent Fp products spread over the group's lanes ------------------------------------
// r[j] = a[j] * b[j] for j < used (<= GRP).  The operands are the same on every lane of the group:
// slot 0 publishes them through the group's LDS area, lane j computes product j, and every lane
// reads all of them back -- one product deep instead of `used`.  Every index into a, b, r is a
// compile-time constant (a lane-dependent index goes to LDS only).  (Publishing each operand as
// soon as it is formed, so that no operand array stays live, measured 11 % slower on the Miller
// loop: the arrays live in registers between the rounds' products anyway.)
#ifdef BLS_GDEV
__device__ __forceinline__ void g_fp_round(const GCtx& g, const fp (&a)[GRP], const fp (&b)[GRP], fp (&r)[GRP],
                                           const int used) {
    uint32_t* A = g.xa;
    uint32_t* B = g.xa + GRP * NL;
    uint32_t* R = g.xa + 2 * GRP * NL;  // 3 GRP NL = 336 words <= GX_WORDS
    g_sync();
    if (g.slot == 0) {
#pragma unroll
        for (int j = 0; j < GRP; j++)
            if (j < used) {
                st_fp(A + j * NL, a[j]);
                st_fp(B + j * NL, b[j]);
            }
    }
    g_sync();
    const int s = g.slot < used ? g.slot : 0;
    const fp p = fp_mul(ld_fp(A + s * NL), ld_fp(B + s * NL));
    if (g.slot < used) st_fp(R + g.slot * NL, p);
    g_sync();
#pragma unroll
    for (int j = 0; j < GRP; j++)
        if (j < used) r[j] = ld_fp(R + j * NL);
}
#else
inline void g_fp_round(const GCtx&, const fp (&a)[GRP], const fp (&b)[GRP], fp (&r)[GRP], const int used) {
    for (int j = 0; j < used; j++) r[j] = fp_mul(a[j], b[j]);
}
#endif
// operand pairs of f2_sqr / f2_mul / f2_mul_fp (bls381.h) at slots o.., and their results, so
// that a round reproduces those functions' products exactly
NWV_HD void ops_sqr(const fp2& x, fp (&a)[GRP], fp (&b)[GRP], int o) {
    a[o] = fp_add(x.c0, x.c1);
    b[o] = fp_sub(x.c0, x.c1);
    a[o + 1] = x.c0;
    b[o + 1] = x.c1;
}
NWV_HD fp2 res_sqr(const fp (&r)[GRP], int o) { return fp2{r[o], fp_dbl(r[o + 1])}; }
NWV_HD void ops_mul(const fp2& x, const fp2& y, fp (&a)[GRP], fp (&b)[GRP], int o) {
    a[o] = x.c0;
    b[o] = y.c0;
    a[o + 1] = x.c1;
    b[o + 1] = y.c1;
    a[o + 2] = fp_add(x.c0, x.c1);
    b[o + 2] = fp_add(y.c0, y.c1);
}
NWV_HD fp2 res_mul(const fp (&r)[GRP], int o) {
    return fp2{fp_sub(r[o], r[o + 1]), fp_sub(fp_sub(r[o + 2], r[o]), r[o + 1])};
}
NWV_HD void ops_mul_fp(const fp2& x, const fp& s, fp (&a)[GRP], fp (&b)[GRP], int o) {
    a[o] = x.c0;
    b[o] = s;
    a[o + 1] = x.c1;
    b[o + 1] = s;
}
NWV_HD fp2 res_mul_fp(const fp (&r)[GRP], int o) { return fp2{r[o], r[o + 1]}; }

// ml_dbl of bls381.h followed by the line's scaling by (x_P, y_P), as four rounds of products over
// the group (8 + 8 + 6 + 7 of its 29 Fp products) instead of 29 on every lane; the same
// operations in the same order, so T and the line come out bit for bit as ml_dbl's.
//   A: X^2, Y^2, Z^2, (Z + Y)^2   B: t1^2, (t1 + X)^2, t4^2, t6^2   C: t4 zz, Z' zz
//   D: (t3 - X') t4, l1 x_P, l4 y_P
// z3 (optional): the line is evaluated times z3 (l0 z3 as well), for a Jacobian P (g_rlc_ml).
G_HD void g_ml_dbl(const GCtx& g, jac<fp2>& T, const fp& px, const fp& py, fp2& l0, fp2& l1p, fp2& l4p,
                   const fp* z3 = nullptr) {
    fp a[GRP], b[GRP], r[GRP];
    ops_sqr(T.x, a, b, 0);
    ops_sqr(T.y, a, b, 2);
    ops_sqr(T.z, a, b, 4);
    ops_sqr(f2_add(T.z, T.y), a, b, 6);
    g_fp_round(g, a, b, r, 8);
    const fp2 t0 = res_sqr(r, 0), t1 = res_sqr(r, 2), zz = res_sqr(r, 4);
    const fp2 zn = f2_sub(f2_sub(res_sqr(r, 6), t1), zz);
    const fp2 t4 = f2_add(f2_dbl(t0), t0);
    const fp2 t6 = f2_add(T.x, t4);
    ops_sqr(t1, a, b, 0);
    ops_sqr(f2_add(t1, T.x), a, b, 2);
    ops_sqr(t4, a, b, 4);
    ops_sqr(t6, a, b, 6);
    g_fp_round(g, a, b, r, 8);
    const fp2 t2 = res_sqr(r, 0), t5 = res_sqr(r, 4);
    const fp2 t3 = f2_dbl(f2_sub(f2_sub(res_sqr(r, 2), t0), t2));
    const fp2 xn = f2_sub(f2_sub(t5, t3), t3);
    l0 = f2_sub(f2_sub(f2_sub(res_sqr(r, 6), t0), t5), f2_dbl(f2_dbl(t1)));
    const fp2 t2x8 = f2_dbl(f2_dbl(f2_dbl(t2)));
    ops_mul(t4, zz, a, b, 0);
    ops_mul(zn, zz, a, b, 3);
    if (z3) ops_mul_fp(l0, *z3, a, b, 6);
    g_fp_round(g, a, b, r, z3 ? 8 : 6);
    const fp2 l1 = f2_neg(f2_dbl(res_mul(r, 0)));
    const fp2 l4 = f2_dbl(res_mul(r, 3));
    if (z3) l0 = res_mul_fp(r, 6);
    ops_mul(f2_sub(t3, xn), t4, a, b, 0);
    ops_mul_fp(l1, px, a, b, 3);
    ops_mul_fp(l4, py, a, b, 5);
    g_fp_round(g, a, b, r, 7);
    T.x = xn;
    T.y = f2_sub(res_mul(r, 0), t2x8);
    T.z = zn;
    l1p = res_mul_fp(r, 3);
    l4p = res_mul_fp(r, 5);
}

// a^-1 through norms, in group operations only (the one-lane f12_inv spills and took ~1.9 ms):
// t = a conj(a) lies in Fp6, N(t) = t t^(p^2) t^(p^4) in Fp2, so a^-1 = conj(a) t^(p^2) t^(p^4) / N(t)
G_HD G12 g_inv(const GCtx& g, const G12& a) {
    const G12 ac = g_conj(g, a);
    const G12 t = g_mul(g, a, ac);
    const G12 t2 = g_frob(g, g_frob(g, t));
    const G12 t4 = g_frob(g, g_frob(g, t2));
    const G12 u = g_mul(g, t2, t4);
    const fp2 nrm = g_coef0(g, g_mul(g, t, u));
    return g_mul(g, ac, g_scale(g, u, f2_inv(nrm)));
}

// prod_{i < N} f_{|x|, Q_i}(P_i), conjugated (x < 0) (miller_loop2 over a group).  N is a template
// parameter so the per-pair loops unroll and the G2 points stay in registers (a runtime pair count
// indexes T[], px[], ... dynamically and puts them in scratch: 2x slower, measured)
// PROJ: P_i given as (X Z, Y) with pz3[i] = Z^3 of a Jacobian P_i; every line is evaluated times
// Z^3, a factor in Fp* that the final exponentiation maps to 1 (g_rlc_ml)
template <int N, bool PROJ = false>
G_NOINLINE G12 g_miller(const GCtx& g, const fp* px, const fp* py, const fp2* qx, const fp2* qy,
                        const fp* pz3 = nullptr) {
    jac<fp2> T[N];
#pragma unroll
    for (int i = 0; i < N; i++) T[i] = jac_from_affine(qx[i], qy[i]);
    G12 f = g_one(g);
    fp2 l0, l1, l4;
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        if (b != 62) f = g_sqr(g, f);
#pragma unroll
        for (int i = 0; i < N; i++) {
            g_ml_dbl(g, T[i], px[i], py[i], l0, l1, l4, PROJ ? &pz3[i] : nullptr);  // products over the lanes
            f = g_mul_line(g, f, l0, l1, l4);
        }
        if ((BLS_X_ABS >> b) & 1) {
#pragma unroll
            for (int i = 0; i < N; i++) {
                ml_add(T[i], qx[i], qy[i], l0, l1, l4);
                if (PROJ) l0 = f2_mul_fp(l0, pz3[i]);
                f = g_mul_line(g, f, l0, f2_mul_fp(l1, px[i]), f2_mul_fp(l4, py[i]));
            }
        }
    }
    return g_conj(g, f);
}

// f^x (x = -BLS_X_ABS) for f in the cyclotomic subgroup
G_NOINLINE G12 g_cyc_exp_x(const GCtx& g, const G12& f) {
    G12 acc = f;
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        acc = g_cyc_sqr(g, acc);
        if ((BLS_X_ABS >> b) & 1) acc = g_mul(g, acc, f);
    }
    return g_conj(g, acc);
}

// f^(3 (p^12 - 1) / r): final_exp of bls381.h over a group
G_NOINLINE G12 g_final_exp(const GCtx& g, const G12& f) {
    G12 m = g_mul(g, g_conj(g, f), g_inv(g, f));  // f^(p^6 - 1)
    m = g_mul(g, g_frob(g, g_frob(g, m)), m);      // ^(p^2 + 1)
    G12 a = g_mul(g, g_cyc_exp_x(g, m), g_conj(g, m));
    a = g_mul(g, g_cyc_exp_x(g, a), g_conj(g, a));
    const G12 b = g_mul(g, g_cyc_exp_x(g, a), g_frob(g, a));
    G12 c = g_cyc_exp_x(g, g_cyc_exp_x(g, b));
    c = g_mul(g, g_mul(g, c, g_frob(g, g_frob(g, b))), g_conj(g, b));
    return g_mul(g, c, g_mul(g, g_cyc_sqr(g, m), m));
}

}  // namespace bls
