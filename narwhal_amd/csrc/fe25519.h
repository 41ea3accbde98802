// fe25519.h -- GF(2^255-19) arithmetic for gfx950 VALU, radix 2^25.5 (ten 32-bit limbs).
//
// Replaces the field layer of curve25519-dalek-ng 4.1.1 (u64_backend, radix 2^51,
// /root/reference/workspace-hack/Cargo.toml:91).  On CDNA4 the natural multiply is the
// 32x32->64 multiply-accumulate `v_mad_u64_u32`, so limbs are 26/25 bits wide and a
// product is 100 multiply-adds into ten 64-bit column accumulators.  Everything here is
// __host__ __device__ so a test-only host build (tests/hostemu) can run it with limb-bound
// assertions enabled (NWV_BOUNDS_CHECK); the product only runs it on the GPU.
//
// Magnitude discipline (m = max limb / 2^26 or 2^25):
//   "L"  carried output of mul/sq/carry: m <= 1.01
//   add(L, L) -> m <= 2.02      sub(L, L) = a + 2p - b -> m <= 3.02 (b must be L)
//   mul/sq inputs must have m <= 3.36 (19 * limb must fit 32 bits; column sums < 2^64)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef NWV_HD
#define NWV_HD __host__ __device__ __forceinline__
#endif

// Scheduling fence around every field multiply: hipcc otherwise interleaves the independent
// multiplies of a point formula (4-way ILP) and doubles the VGPR footprint; one multiply
// already carries ten independent accumulation chains, so occupancy is worth more.
#if defined(__HIP_DEVICE_COMPILE__)
#define NWV_SEQ() __builtin_amdgcn_sched_barrier(0)
#else
#define NWV_SEQ() ((void)0)
#endif

#ifdef NWV_BOUNDS_CHECK
#include <assert.h>
#define NWV_ASSERT(x) assert(x)
#else
#define NWV_ASSERT(x) ((void)0)
#endif

// host-emulation op counting (tests/hostemu, -DNWV_COUNT_OPS): algorithmic multiply counts
// per phase, the numerator of the VALU roofline in bench.py
#ifdef NWV_COUNT_OPS
extern unsigned long long nwv_count_mul, nwv_count_sq;
#define NWV_COUNT(x) (++(x))
#else
#define NWV_COUNT(x) ((void)0)
#endif

namespace nwv {

struct fe {
    uint32_t v[10];
};

static constexpr uint32_t M26 = (1u << 26) - 1;
static constexpr uint32_t M25 = (1u << 25) - 1;

NWV_HD constexpr int limb_bits(int i) { return (i & 1) ? 25 : 26; }

NWV_HD void fe_check(const fe& a, double m) {
#ifdef NWV_BOUNDS_CHECK
    for (int i = 0; i < 10; i++) NWV_ASSERT((double)a.v[i] <= m * (double)(1u << limb_bits(i)));
#else
    (void)a; (void)m;
#endif
}

NWV_HD fe fe_zero() { fe r; for (int i = 0; i < 10; i++) r.v[i] = 0; return r; }
NWV_HD fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }
NWV_HD fe fe_small(uint32_t x) { fe r = fe_zero(); r.v[0] = x; return r; }

NWV_HD fe fe_add(const fe& a, const fe& b) {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + b.v[i];
    return r;
}

// a - b + 2p; b must be carried (limb0 <= 2^27-38, others <= 2^(bits+1)-2)
NWV_HD fe fe_sub(const fe& a, const fe& b) {
    fe_check(b, 1.9);
    fe r;
    r.v[0] = a.v[0] + 0x7FFFFDAu - b.v[0];
#pragma unroll
    for (int i = 1; i < 10; i++) r.v[i] = a.v[i] + ((i & 1) ? 0x3FFFFFEu : 0x7FFFFFEu) - b.v[i];
    return r;
}
NWV_HD fe fe_neg(const fe& b) { return fe_sub(fe_zero(), b); }

// weak reduction of 32-bit limbs (inputs up to ~2^31): every limb ends below 2^26/2^25
// except limb 1, which may exceed 2^25 by < 2^7.
NWV_HD fe fe_carry(const fe& a) {
    fe r = a;
    uint32_t c;
    c = r.v[0] >> 26; r.v[0] &= M26; r.v[1] += c;
    c = r.v[4] >> 26; r.v[4] &= M26; r.v[5] += c;
    c = r.v[1] >> 25; r.v[1] &= M25; r.v[2] += c;
    c = r.v[5] >> 25; r.v[5] &= M25; r.v[6] += c;
    c = r.v[2] >> 26; r.v[2] &= M26; r.v[3] += c;
    c = r.v[6] >> 26; r.v[6] &= M26; r.v[7] += c;
    c = r.v[3] >> 25; r.v[3] &= M25; r.v[4] += c;
    c = r.v[7] >> 25; r.v[7] &= M25; r.v[8] += c;
    c = r.v[4] >> 26; r.v[4] &= M26; r.v[5] += c;
    c = r.v[8] >> 26; r.v[8] &= M26; r.v[9] += c;
    c = r.v[9] >> 25; r.v[9] &= M25; r.v[0] += 19 * c;
    c = r.v[0] >> 26; r.v[0] &= M26; r.v[1] += c;
    return r;
}

// carry of ten 64-bit column sums (each < 2^63) into a carried element
NWV_HD fe fe_carry64(uint64_t h[10]) {
    uint64_t c;
    c = h[0] >> 26; h[1] += c; h[0] &= M26;
    c = h[4] >> 26; h[5] += c; h[4] &= M26;
    c = h[1] >> 25; h[2] += c; h[1] &= M25;
    c = h[5] >> 25; h[6] += c; h[5] &= M25;
    c = h[2] >> 26; h[3] += c; h[2] &= M26;
    c = h[6] >> 26; h[7] += c; h[6] &= M26;
    c = h[3] >> 25; h[4] += c; h[3] &= M25;
    c = h[7] >> 25; h[8] += c; h[7] &= M25;
    c = h[4] >> 26; h[5] += c; h[4] &= M26;
    c = h[8] >> 26; h[9] += c; h[8] &= M26;
    c = h[9] >> 25; h[0] += c * 19; h[9] &= M25;
    fe r;
#pragma unroll
    for (int i = 2; i < 10; i++) r.v[i] = (uint32_t)h[i];
    // last carry in 32 bits: limbs 0 and 1 leave as plain 32-bit values (keeps the compiler
    // from carrying them as 64-bit quantities into the next multiply)
    r.v[0] = (uint32_t)h[0] & M26;
    r.v[1] = (uint32_t)h[1] + (uint32_t)(h[0] >> 26);
    return r;
}

NWV_HD uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// h = f * g.  Column k collects f_i g_j with i + j = k (mod 10); the term is doubled when
// i and j are both odd (radix 2^25.5) and multiplied by 19 when i + j >= 10 (2^255 = 19).
NWV_HD fe fe_mul(const fe& f, const fe& g) {
    NWV_SEQ();
    NWV_COUNT(nwv_count_mul);
    fe_check(f, 3.36);
    fe_check(g, 3.36);
    uint32_t g19[10], f2[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        g19[i] = g.v[i] * 19u;
        f2[i] = (i & 1) ? (f.v[i] << 1) : f.v[i];
    }
    uint64_t h[10];
#pragma unroll
    for (int k = 0; k < 10; k++) {
        uint64_t acc = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const int j = (k - i + 10) % 10;
            const bool wrap = (i + j) >= 10;
            const bool dbl = (i & 1) && (j & 1);
            const uint32_t fa = dbl ? f2[i] : f.v[i];
            const uint32_t gb = wrap ? g19[j] : g.v[j];
            acc = mad(fa, gb, acc);
        }
        h[k] = acc;
    }
    fe r = fe_carry64(h);
    NWV_SEQ();
    return r;
}

// h = f^2 (55 products): pair (i<j) is doubled on f_i, the odd/odd doubling and the 19 of
// the wrap go on f_j; diagonal terms carry the odd doubling and the wrap on one side.
NWV_HD fe fe_sq(const fe& f) {
    NWV_SEQ();
    NWV_COUNT(nwv_count_sq);
    fe_check(f, 3.36);
    uint64_t h[10];
#pragma unroll
    for (int k = 0; k < 10; k++) h[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
#pragma unroll
        for (int j = i; j < 10; j++) {
            const int k = (i + j) % 10;
            const bool wrap = (i + j) >= 10;
            const bool dbl = (i & 1) && (j & 1);
            uint32_t a = (i == j) ? f.v[i] : (f.v[i] << 1);
            uint32_t b = f.v[j] * ((dbl ? 2u : 1u) * (wrap ? 19u : 1u));
            h[k] = mad(a, b, h[k]);
        }
    }
    fe r = fe_carry64(h);
    NWV_SEQ();
    return r;
}

NWV_HD void fe_pin(fe& a);
NWV_HD fe fe_sqn(fe f, int n) {
#pragma unroll 1
    for (int i = 0; i < n; i++) {
        fe_pin(f);  // loop-carried limbs stay plain 32-bit values
        f = fe_sq(f);
    }
    return f;
}

// canonical little-endian 8x32-bit words of a (value reduced into [0, p))
NWV_HD void fe_freeze(const fe& a, uint32_t w[8]) {
    NWV_SEQ();
    fe h = fe_carry(fe_carry(a));
    uint32_t q = (h.v[0] + 19) >> 26;
#pragma unroll
    for (int i = 1; i < 10; i++) q = (h.v[i] + q) >> limb_bits(i);
    h.v[0] += 19 * q;
    uint32_t c;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        c = h.v[i] >> limb_bits(i);
        h.v[i] &= (i & 1) ? M25 : M26;
        h.v[i + 1] += c;
    }
    h.v[9] &= M25;
    // pack limbs at bit positions 0,26,51,77,102,128,153,179,204,230
    w[0] = h.v[0] | (h.v[1] << 26);
    w[1] = (h.v[1] >> 6) | (h.v[2] << 19);
    w[2] = (h.v[2] >> 13) | (h.v[3] << 13);
    w[3] = (h.v[3] >> 19) | (h.v[4] << 6);
    w[4] = h.v[5] | (h.v[6] << 25);
    w[5] = (h.v[6] >> 7) | (h.v[7] << 19);
    w[6] = (h.v[7] >> 13) | (h.v[8] << 12);
    w[7] = (h.v[8] >> 20) | (h.v[9] << 6);
    NWV_SEQ();
}

// FieldElement::from_bytes semantics: bit 255 ignored, values >= p kept (they reduce lazily)
NWV_HD fe fe_from_words(const uint32_t w[8]) {
    fe r;
    r.v[0] = w[0] & M26;
    r.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
    r.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
    r.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
    r.v[4] = (w[3] >> 6) & M26;
    r.v[5] = w[4] & M25;
    r.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
    r.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
    r.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
    r.v[9] = (w[7] >> 6) & M25;
    return r;
}

NWV_HD bool fe_is_zero(const fe& a) {
    uint32_t w[8];
    fe_freeze(a, w);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= w[i];
    return acc == 0;
}
NWV_HD bool fe_eq(const fe& a, const fe& b) { return fe_is_zero(fe_sub(fe_carry(a), fe_carry(b))); }
NWV_HD uint32_t fe_is_negative(const fe& a) {
    uint32_t w[8];
    fe_freeze(a, w);
    return w[0] & 1;
}
NWV_HD fe fe_select(const fe& a, const fe& b, bool pick_b) {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; i++) r.v[i] = pick_b ? b.v[i] : a.v[i];
    return r;
}

// x^(2^250 - 1) and x^11 (the shared head of inversion and the (p-5)/8 power)
NWV_HD void fe_pow22501(const fe& x, fe& t19, fe& t3) {
    fe t0 = fe_sq(x);
    fe t1 = fe_sqn(t0, 2);
    fe t2 = fe_mul(x, t1);
    t3 = fe_mul(t0, t2);
    fe t4 = fe_sq(t3);
    fe t5 = fe_mul(t2, t4);
    fe t6 = fe_sqn(t5, 5);
    fe t7 = fe_mul(t6, t5);
    fe t8 = fe_sqn(t7, 10);
    fe t9 = fe_mul(t8, t7);
    fe t10 = fe_sqn(t9, 20);
    fe t11 = fe_mul(t10, t9);
    fe t12 = fe_sqn(t11, 10);
    fe t13 = fe_mul(t12, t7);
    fe t14 = fe_sqn(t13, 50);
    fe t15 = fe_mul(t14, t13);
    fe t16 = fe_sqn(t15, 100);
    fe t17 = fe_mul(t16, t15);
    fe t18 = fe_sqn(t17, 50);
    t19 = fe_mul(t18, t13);
}
NWV_HD fe fe_invert(const fe& x) {
    fe t19, t3;
    fe_pow22501(x, t19, t3);
    return fe_mul(fe_sqn(t19, 5), t3);
}
NWV_HD fe fe_pow_p58(const fe& x) {
    fe t19, t3;
    fe_pow22501(x, t19, t3);
    return fe_mul(fe_sqn(t19, 2), x);
}

// curve constants (radix 2^25.5 limbs)
NWV_HD fe fe_d() {
    const uint32_t c[10] = {56195235, 13857412, 51736253, 6949390, 114729,
                            24766616, 60832955, 30306712, 48412415, 21499315};
    fe r; for (int i = 0; i < 10; i++) r.v[i] = c[i]; return r;
}
NWV_HD fe fe_d2() {
    const uint32_t c[10] = {45281625, 27714825, 36363642, 13898781, 229458,
                            15978800, 54557047, 27058993, 29715967, 9444199};
    fe r; for (int i = 0; i < 10; i++) r.v[i] = c[i]; return r;
}
NWV_HD fe fe_sqrtm1() {
    const uint32_t c[10] = {34513072, 25610706, 9377949, 3500415, 12389472,
                            33281959, 41962654, 31548777, 326685, 11406482};
    fe r; for (int i = 0; i < 10; i++) r.v[i] = c[i]; return r;
}

// Optimisation fence for a field element: the value is "redefined" here, so nothing computed
// from it can be hoisted above this point (keeps IR-level code motion from stretching live
// ranges across the long exponentiation chains).
NWV_HD void fe_pin(fe& a) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < 10; i++) asm volatile("" : "+v"(a.v[i]));
#else
    (void)a;
#endif
}

// FieldElement::sqrt_ratio_i (dalek): returns was_nonzero_square; r = nonnegative sqrt(u/v)
//   r = (u v^3) (u v^7)^((p-5)/8); check = v r^2;
//   correct = check == u, flipped = check == -u, flipped_i = check == -u sqrt(-1)
NWV_HD bool fe_sqrt_ratio_i(const fe& u_in, const fe& v_in, fe& r) {
    fe u = u_in, v = v_in;
    fe v3 = fe_mul(fe_sq(v), v);
    fe uv7 = fe_mul(u, fe_mul(fe_sq(v3), v));
    fe uv3 = fe_mul(u, v3);
    fe pw = fe_pow_p58(uv7);
    fe_pin(pw);
    r = fe_mul(uv3, pw);
    fe_pin(v);
    fe check = fe_carry(fe_mul(v, fe_sq(r)));
    fe_pin(u);
    const bool correct = fe_is_zero(fe_sub(check, u));
    const bool flipped = fe_is_zero(fe_add(check, u));
    fe_pin(u);
    const bool flipped_i = fe_is_zero(fe_add(check, fe_mul(u, fe_sqrtm1())));
    fe_pin(r);
    fe r_prime = fe_mul(r, fe_sqrtm1());
    r = fe_select(r, r_prime, flipped || flipped_i);
    r = fe_select(r, fe_carry(fe_neg(r)), fe_is_negative(r) != 0);
    return correct || flipped;
}

}  // namespace nwv
