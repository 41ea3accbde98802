// fe_row.h -- GF(2^255-19) spread over a 16-lane DPP row, for latency-bound point chains.
//
// The batch MSM ends in one dependent chain: the Horner over the window sums (~250 doublings
// plus one addition per window, SURVEY §8a a9: the reference's batch::Verifier computes the
// same multiscalar sum on one CPU core).  That chain runs on a single wave, where a lane-local
// field multiply (100 v_mad_u64_u32 on ten 26/25-bit limbs, fe25519.h) is pure issue latency.
// Here one field element lives on one row of 16 lanes, lane k holding limb k of radix 2^16, so
// a multiply is a 16-step cyclic convolution (2^256 = 38 mod p) with one 64-bit multiply-add per
// lane per step, and the four rows of a wave compute the four independent multiplies of a
// doubling or an addition at once.  Row data movement is DPP within a row (row_shr / row_shl /
// row_share / row_ror) and the gfx950 permlane16/32 swaps across rows (gather4).
//
// The code is generic over the lane type so the same functions run on the host for tests:
//   device:  V = uint32_t (this lane), M = bool, DPP / permlane builtins;
//   host:    V = 64 lanes of one wave, every operation checked for 32/64-bit overflow
//            (tests/hostemu, NWV_BOUNDS_CHECK), DPP / permlane emulated with the semantics
//            measured on gfx950 (tools/probe/dpp_probe.hip).
//
// Magnitudes: mul() takes operands with limbs a_k, b_k such that the column sums fit (checked
// on the host): in practice "loose" limbs <= 2^17.7.  Its output has limbs < 2^16 + 2^12 (two
// carry passes; round 3 ran a third that tightened this to 2^16 + 2^11).  sub uses 8p, whose
// limbs (>= 2^18) dominate any loose limb.
#pragma once
#include "fe25519.h"

namespace nwv {
namespace rowf {

#if defined(__HIP_DEVICE_COMPILE__)

using V = uint32_t;
using V64 = uint64_t;
using M = bool;
__device__ __forceinline__ V lane_id() { return __lane_id(); }
__device__ __forceinline__ V bc(uint32_t x) { return x; }
__device__ __forceinline__ V mul24(V a, V b) { return __umul24(a, b); }
__device__ __forceinline__ V mul32(V a, V b) { return a * b; }
__device__ __forceinline__ V64 mad64(V a, V b, V64 c) { return (uint64_t)a * b + c; }
__device__ __forceinline__ V64 zero64() { return 0; }
__device__ __forceinline__ V64 add64(V64 a, V64 b) { return a + b; }
__device__ __forceinline__ void phase_fence() { __builtin_amdgcn_sched_barrier(0); }

__device__ __forceinline__ V lo16(V64 x) { return (uint32_t)x & 0xFFFFu; }
__device__ __forceinline__ V shr16(V64 x) { return (uint32_t)(x >> 16); }
__device__ __forceinline__ V sel(M m, V a, V b) { return m ? b : a; }
__device__ __forceinline__ M row_is(int q) { return ((__lane_id() >> 4) & 3) == (uint32_t)q; }
__device__ __forceinline__ M limb_is(int k) { return (__lane_id() & 15) == (uint32_t)k; }
__device__ __forceinline__ M limb_lt(int k) { return (__lane_id() & 15) < (uint32_t)k; }
template <int R>
__device__ __forceinline__ V shr(V x) { return (V)__builtin_amdgcn_mov_dpp((int)x, 0x110 + R, 0xF, 0xF, true); }
template <int R>
__device__ __forceinline__ V shl(V x) { return (V)__builtin_amdgcn_mov_dpp((int)x, 0x100 + R, 0xF, 0xF, true); }
template <int R>
__device__ __forceinline__ V share(V x) { return (V)__builtin_amdgcn_mov_dpp((int)x, 0x150 + R, 0xF, 0xF, true); }
__device__ __forceinline__ V ror1(V x) { return (V)__builtin_amdgcn_mov_dpp((int)x, 0x121, 0xF, 0xF, true); }
// row_ror:R -- lane k of a row gets lane (k - R) mod 16 of the same row
template <int R>
__device__ __forceinline__ V ror(V x) { return (V)__builtin_amdgcn_mov_dpp((int)x, 0x120 + R, 0xF, 0xF, true); }
// v_permlane16_swap: old.rows(1,3) <-> src.rows(0,2);  v_permlane32_swap: old.rows(2,3) <-> src.rows(0,1)
__device__ __forceinline__ void swap16(V& a, V& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
__device__ __forceinline__ void swap32(V& a, V& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
// per-lane LDS / memory access
__device__ __forceinline__ V ld(const uint32_t* base, V idx) { return base[idx]; }
__device__ __forceinline__ void st(uint32_t* base, V idx, V x, M m) {
    if (m) base[idx] = x;
}
__device__ __forceinline__ void st_all(uint32_t* base, V idx, V x) { base[idx] = x; }
// four consecutive words at a 16-byte aligned index (one ds_read_b128)
__device__ __forceinline__ void ld4(const uint32_t* base, V idx, V& x0, V& x1, V& x2, V& x3) {
    const uint4 q = *reinterpret_cast<const uint4*>(base + idx);
    x0 = q.x;
    x1 = q.y;
    x2 = q.z;
    x3 = q.w;
}
// LDS accesses of one wave execute in issue order; this keeps the compiler from moving them
// across each other when one lane reads what another lane of the wave wrote
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

#else  // host emulation of one wave

#include <cstdio>
#include <cstdlib>

struct V {
    uint32_t l[64];
};
struct V64 {
    uint64_t l[64];
};
struct M {
    bool l[64];
};
#define NWV_ROW_FOR for (int i = 0; i < 64; i++)
inline void row_check(bool ok) {
    if (!ok) {
        fprintf(stderr, "fe_row: magnitude overflow\n");
        abort();
    }
}
inline V bc(uint32_t x) { V r; NWV_ROW_FOR r.l[i] = x; return r; }
inline V lane_id() { V r; NWV_ROW_FOR r.l[i] = (uint32_t)i; return r; }
inline V operator+(V a, V b) {
    V r;
    NWV_ROW_FOR { const uint64_t s = (uint64_t)a.l[i] + b.l[i]; row_check(s >> 32 == 0); r.l[i] = (uint32_t)s; }
    return r;
}
inline V operator-(V a, V b) {
    V r;
    NWV_ROW_FOR { row_check(a.l[i] >= b.l[i]); r.l[i] = a.l[i] - b.l[i]; }
    return r;
}
inline V operator&(V a, uint32_t m) { V r; NWV_ROW_FOR r.l[i] = a.l[i] & m; return r; }
inline V operator>>(V a, int s) { V r; NWV_ROW_FOR r.l[i] = a.l[i] >> s; return r; }
inline V mul24(V a, V b) {
    V r;
    NWV_ROW_FOR {
        row_check(a.l[i] < (1u << 24) && b.l[i] < (1u << 24));
        const uint64_t p = (uint64_t)a.l[i] * b.l[i];
        row_check(p >> 32 == 0);
        r.l[i] = (uint32_t)p;
    }
    return r;
}
inline V mul32(V a, V b) {
    V r;
    NWV_ROW_FOR { const uint64_t p = (uint64_t)a.l[i] * b.l[i]; row_check(p >> 32 == 0); r.l[i] = (uint32_t)p; }
    return r;
}
inline V64 zero64() { V64 r; NWV_ROW_FOR r.l[i] = 0; return r; }
inline V64 add64(V64 a, V64 b) {
    V64 r;
    NWV_ROW_FOR { r.l[i] = a.l[i] + b.l[i]; row_check(r.l[i] >= a.l[i]); }
    return r;
}
inline void phase_fence() {}
inline V64 mad64(V a, V b, V64 c) {
    V64 r;
    NWV_ROW_FOR {
        const unsigned __int128 s = (unsigned __int128)a.l[i] * b.l[i] + c.l[i];
        row_check((s >> 64) == 0);
        r.l[i] = (uint64_t)s;
    }
    return r;
}
inline V lo16(V64 x) { V r; NWV_ROW_FOR r.l[i] = (uint32_t)x.l[i] & 0xFFFFu; return r; }
// the device takes bits 16..47 of the column: the column must stay below 2^48
inline V shr16(V64 x) { V r; NWV_ROW_FOR { row_check(x.l[i] >> 48 == 0); r.l[i] = (uint32_t)(x.l[i] >> 16); } return r; }
inline V sel(M m, V a, V b) { V r; NWV_ROW_FOR r.l[i] = m.l[i] ? b.l[i] : a.l[i]; return r; }
inline M row_is(int q) { M m; NWV_ROW_FOR m.l[i] = ((i >> 4) & 3) == q; return m; }
inline M limb_is(int k) { M m; NWV_ROW_FOR m.l[i] = (i & 15) == k; return m; }
inline M limb_lt(int k) { M m; NWV_ROW_FOR m.l[i] = (i & 15) < k; return m; }
template <int R>
inline V shr(V x) { V r; NWV_ROW_FOR r.l[i] = (i & 15) >= R ? x.l[i - R] : 0u; return r; }
template <int R>
inline V shl(V x) { V r; NWV_ROW_FOR r.l[i] = (i & 15) + R <= 15 ? x.l[i + R] : 0u; return r; }
template <int R>
inline V share(V x) { V r; NWV_ROW_FOR r.l[i] = x.l[(i & ~15) + R]; return r; }
inline V ror1(V x) { V r; NWV_ROW_FOR r.l[i] = x.l[(i & ~15) + (((i & 15) + 15) & 15)]; return r; }
template <int R>
inline V ror(V x) { V r; NWV_ROW_FOR r.l[i] = x.l[(i & ~15) + (((i & 15) + 16 - R) & 15)]; return r; }
inline void swap16(V& a, V& b) {
    V ra = a, rb = b;
    NWV_ROW_FOR {
        const int row = i >> 4, j = i & 15;
        if (row & 1) ra.l[i] = b.l[(row - 1) * 16 + j];  // old rows 1,3 <- src rows 0,2
        else rb.l[i] = a.l[(row + 1) * 16 + j];          // src rows 0,2 <- old rows 1,3
    }
    a = ra;
    b = rb;
}
inline void swap32(V& a, V& b) {
    V ra = a, rb = b;
    NWV_ROW_FOR {
        if (i >= 32) ra.l[i] = b.l[i - 32];  // old rows 2,3 <- src rows 0,1
        else rb.l[i] = a.l[i + 32];          // src rows 0,1 <- old rows 2,3
    }
    a = ra;
    b = rb;
}
inline V ld(const uint32_t* base, V idx) { V r; NWV_ROW_FOR r.l[i] = base[idx.l[i]]; return r; }
inline void st(uint32_t* base, V idx, V x, M m) { NWV_ROW_FOR if (m.l[i]) base[idx.l[i]] = x.l[i]; }
inline void st_all(uint32_t* base, V idx, V x) { NWV_ROW_FOR base[idx.l[i]] = x.l[i]; }
inline void ld4(const uint32_t* base, V idx, V& x0, V& x1, V& x2, V& x3) {
    NWV_ROW_FOR {
        row_check(idx.l[i] % 4 == 0);
        x0.l[i] = base[idx.l[i]];
        x1.l[i] = base[idx.l[i] + 1];
        x2.l[i] = base[idx.l[i] + 2];
        x3.l[i] = base[idx.l[i] + 3];
    }
}
inline void lds_order() {}
#undef NWV_ROW_FOR

#endif

// ---- field operations on a row -------------------------------------------------------------

struct RowConsts {
    V w15;  // carry-out weight: 38 on limb 15 (2^256 = 38 mod p), 1 elsewhere
    V k8p;  // limb k of 8p: 8 * (0xFFED | 0xFFFF | 0x7FFF)
    M r1, r2, r3;
    uint32_t* sc = nullptr;  // 192 words of LDS for this wave: operands of mul() go through LDS
    int rot = 0;             // mul() by row rotations (mul_ror; 2: two multiply-add chains) instead of LDS or shifts
};
NWV_HD RowConsts row_consts() {
    RowConsts c;
    c.w15 = sel(limb_is(15), bc(1), bc(38));
    c.k8p = sel(limb_is(0), sel(limb_is(15), bc(8u * 0xFFFFu), bc(8u * 0x7FFFu)), bc(8u * 0xFFEDu));
    c.r1 = row_is(1);
    c.r2 = row_is(2);
    c.r3 = row_is(3);
    return c;
}

// value of row q selected per row: row 0 a, row 1 b, row 2 c, row 3 d
NWV_HD V rowsel(const RowConsts& k, V a, V b, V c, V d) { return sel(k.r3, sel(k.r2, sel(k.r1, a, b), c), d); }

// x0..x3 <- row q's element of x, broadcast to every row (3 permlane swaps)
NWV_HD void gather4(V x, V& x0, V& x1, V& x2, V& x3) {
    V a = x, b = x;
    swap16(a, b);  // a = [x0 x0 x2 x2], b = [x1 x1 x3 x3]
    V a2 = a, b2 = b;
    swap32(a, a2);  // a = [x0 x0 x0 x0], a2 = [x2 x2 x2 x2]
    swap32(b, b2);
    x0 = a;
    x1 = b;
    x2 = a2;
    x3 = b2;
}

// one carry pass over 32-bit limbs: limb k keeps 16 bits and receives limb k-1's carry (limb 0
// receives 38 x limb 15's); needs limbs < 2^32 and carries < 2^24 / 38
NWV_HD V carry32(V x, const RowConsts& k) { return (x & 0xFFFFu) + ror1(mul24(x >> 16, k.w15)); }

NWV_HD V sub(V a, V b, const RowConsts& k) { return a + k.k8p - b; }

// a * b mod p (every row its own product).  Lane k accumulates sum_R op_R * b_R with op_R =
// a_{k-R} (k >= R) or 38 a_{k-R+16} (k < R).  All sixteen operand pairs are formed first (DPP
// moves with no dependence on each other, so no DPP read-after-write waits), then one chain of
// sixteen multiply-adds.
NWV_HD V mul_dpp(V a, V b, const RowConsts& k) {
    const V a38 = mul24(a, bc(38));
    V op[16], bs[16];
    op[0] = a;
    bs[0] = share<0>(b);
#define NWV_ROW_OPERANDS(R)                    \
    op[R] = shr<R>(a) + shl<16 - R>(a38);      \
    bs[R] = share<R>(b);
    NWV_ROW_OPERANDS(1) NWV_ROW_OPERANDS(2) NWV_ROW_OPERANDS(3) NWV_ROW_OPERANDS(4)
    NWV_ROW_OPERANDS(5) NWV_ROW_OPERANDS(6) NWV_ROW_OPERANDS(7) NWV_ROW_OPERANDS(8)
    NWV_ROW_OPERANDS(9) NWV_ROW_OPERANDS(10) NWV_ROW_OPERANDS(11) NWV_ROW_OPERANDS(12)
    NWV_ROW_OPERANDS(13) NWV_ROW_OPERANDS(14) NWV_ROW_OPERANDS(15)
#undef NWV_ROW_OPERANDS
    phase_fence();
    V64 acc = mad64(op[0], bs[0], zero64());
#pragma unroll
    for (int r = 1; r < 16; r++) acc = mad64(op[r], bs[r], acc);
    // first pass on the 64-bit columns (< 2^48): limb 15's carry x38 stays < 2^32; one more pass
    // leaves limbs < 2^16 + 2^12 (operands of the next multiply, of sub's 8p and of carry32 all
    // take that: a third pass, as before round 4, only tightened it to 2^16 + 2^11)
    const V x = lo16(acc) + ror1(mul32(shr16(acc), k.w15));
    return carry32(x, k);
}

// The same product with the operands exchanged through LDS instead of 45 DPP moves: each row
// writes ext = [38 a | a | b] (48 words), then lane k reads op_R = ext[16 + k - R] (the wrapped,
// x38 limbs sit below a) and b_R = ext[32 + R] (four 16-byte broadcast reads per row).
NWV_HD V mul_lds(V a, V b, const RowConsts& k) {
    const V lane = lane_id() & 63u;
    const V limb = lane & 15u;
    const V base = mul32(lane >> 4, bc(48));
    st_all(k.sc, base + limb, mul24(a, bc(38)));
    st_all(k.sc, base + bc(16) + limb, a);
    st_all(k.sc, base + bc(32) + limb, b);
    lds_order();
    V op[16], bs[16];
#pragma unroll
    for (int r = 0; r < 16; r++) op[r] = ld(k.sc, base + bc(16 - r) + limb);
#pragma unroll
    for (int r = 0; r < 16; r += 4) ld4(k.sc, base + bc(32 + r), bs[r], bs[r + 1], bs[r + 2], bs[r + 3]);
    lds_order();
    // one multiply-add chain: a wave64 v_mad_u64_u32 is issue-bound, so splitting the chain
    // (measured: 4 chains, 904 vs 808 cycles per doubling) only adds the final additions
    V64 acc = mad64(op[0], bs[0], zero64());
#pragma unroll
    for (int r = 1; r < 16; r++) acc = mad64(op[r], bs[r], acc);
    const V x = lo16(acc) + ror1(mul32(shr16(acc), k.w15));
    return carry32(x, k);  // two passes (see mul_dpp)
}

// The same product with each wrapped operand made by ONE instruction: op_R = ror<R>(a) x w_R,
// w_R = 38 on limbs k < R (the wrapped ones), else 1 -- a row_ror DPP source folded into
// v_mul_u32_u24 -- and b_R by one row_newbcast move.  No LDS round trip, 31 operand instructions.
NWV_HD V mul_ror(V a, V b, const RowConsts& k) {
    V op[16], bs[16];
    op[0] = a;
    bs[0] = share<0>(b);
#define NWV_ROW_OPERANDS(R)                                         \
    op[R] = mul24(ror<R>(a), sel(limb_lt(R), bc(1), bc(38)));       \
    bs[R] = share<R>(b);
    NWV_ROW_OPERANDS(1) NWV_ROW_OPERANDS(2) NWV_ROW_OPERANDS(3) NWV_ROW_OPERANDS(4)
    NWV_ROW_OPERANDS(5) NWV_ROW_OPERANDS(6) NWV_ROW_OPERANDS(7) NWV_ROW_OPERANDS(8)
    NWV_ROW_OPERANDS(9) NWV_ROW_OPERANDS(10) NWV_ROW_OPERANDS(11) NWV_ROW_OPERANDS(12)
    NWV_ROW_OPERANDS(13) NWV_ROW_OPERANDS(14) NWV_ROW_OPERANDS(15)
#undef NWV_ROW_OPERANDS
    V64 acc;
    if (k.rot == 2) {  // two interleaved multiply-add chains
        V64 a0 = mad64(op[0], bs[0], zero64()), a1 = mad64(op[1], bs[1], zero64());
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
            a0 = mad64(op[r], bs[r], a0);
            a1 = mad64(op[r + 1], bs[r + 1], a1);
        }
        acc = add64(a0, a1);
    } else {
        acc = mad64(op[0], bs[0], zero64());
#pragma unroll
        for (int r = 1; r < 16; r++) acc = mad64(op[r], bs[r], acc);
    }
    const V x = lo16(acc) + ror1(mul32(shr16(acc), k.w15));
    return carry32(x, k);  // two passes (see mul_dpp)
}

// a * b mod p on every row: the rotation form (k.rot), the LDS form when the wave has scratch
// (k.sc), else the shift form
NWV_HD V mul(V a, V b, const RowConsts& k) {
    return k.rot ? mul_ror(a, b, k) : k.sc ? mul_lds(a, b, k) : mul_dpp(a, b, k);
}

// x^(2^n) on every row
NWV_HD V row_sqn(V x, int n, const RowConsts& k) {
#pragma unroll 1
    for (int i = 0; i < n; i++) x = mul(x, x, k);
    return x;
}

// x^((p-5)/8) on every row: fe_pow22501 and fe_pow_p58's addition chain (fe25519.h), 250
// squarings and 11 multiplies, each one row product (the decompression's power, ge25519.h, for
// latency-bound small batches: a rotation-form round is ~0.17 us against ~0.27 us for one
// lane-local squaring)
NWV_HD V row_pow_p58(V x, const RowConsts& k) {
    const V t0 = mul(x, x, k);
    const V t1 = row_sqn(t0, 2, k);
    const V t2 = mul(x, t1, k);
    const V t3 = mul(t0, t2, k);
    const V t4 = mul(t3, t3, k);
    const V t5 = mul(t2, t4, k);
    const V t6 = row_sqn(t5, 5, k);
    const V t7 = mul(t6, t5, k);
    const V t8 = row_sqn(t7, 10, k);
    const V t9 = mul(t8, t7, k);
    const V t10 = row_sqn(t9, 20, k);
    const V t11 = mul(t10, t9, k);
    const V t12 = row_sqn(t11, 10, k);
    const V t13 = mul(t12, t7, k);
    const V t14 = row_sqn(t13, 50, k);
    const V t15 = mul(t14, t13, k);
    const V t16 = row_sqn(t15, 100, k);
    const V t17 = mul(t16, t15, k);
    const V t18 = row_sqn(t17, 50, k);
    const V t19 = mul(t18, t13, k);
    return mul(row_sqn(t19, 2, k), x, k);
}

NWV_HD V row_d2();
// a field constant given as 16 radix-2^16 limbs, lane k of every row holding limb k
NWV_HD V row_const(const uint32_t c[16]) {
    V x = bc(c[0]);
#pragma unroll
    for (int i = 1; i < 16; i++) x = sel(limb_is(i), x, bc(c[i]));
    return x;
}
NWV_HD V row_d() {  // the curve's d = -121665 / 121666
    const uint32_t c[16] = {30883, 4953, 19914, 30187, 55467, 16705, 2637, 112,
                            59544, 30585, 16505, 36039, 65139, 11119, 27886, 20995};
    return row_const(c);
}
NWV_HD V row_sqrtm1() {  // sqrt(-1) = 2^((p - 1) / 4)
    const uint32_t c[16] = {41136, 18958, 6951, 50414, 58488, 44335, 6150, 12099,
                            55207, 15867, 153, 11085, 57099, 20417, 9344, 11139};
    return row_const(c);
}

// Point decompression (ge25519.h ge_decompress, CompressedEdwardsY::decompress) on rows, one
// point per row, for latency-bound small batches: the prelude and the square-root test's
// products as row products; only the canonical tests (zero, sign) and the record's conversion
// stay lane-local (msm_points_rows_block).
//   y: the encoding's low 255 bits as 16 limbs (values >= p accepted, reduced lazily)
NWV_HD void row_dec_pre(V y, const RowConsts& k, V& u, V& v, V& uv3, V& uv7) {
    const V one = sel(limb_is(0), bc(0), bc(1));
    const V yy = mul(y, y, k);
    u = carry32(sub(yy, one, k), k);          // y^2 - 1
    v = carry32(mul(yy, row_d(), k) + one, k);  // d y^2 + 1
    const V v3 = mul(mul(v, v, k), v, k);
    uv3 = mul(u, v3, k);
    uv7 = mul(uv3, mul(v3, v, k), k);  // u v^7 = (u v^3) v^4
}
// after pw = uv7^((p-5)/8): the candidate root r = u v^3 pw, r sqrt(-1), and the three values
// whose zero tests decide the root: check - u, check + u, check + u sqrt(-1) (check = v r^2)
NWV_HD void row_dec_mid(V uv3, V pw, V u, V v, const RowConsts& k, V& r, V& ri, V& c0, V& c1, V& c2) {
    const V i = row_sqrtm1();
    r = mul(uv3, pw, k);
    ri = mul(r, i, k);
    const V check = mul(v, mul(r, r, k), k);
    c0 = carry32(sub(check, u, k), k);
    c1 = carry32(check + u, k);
    c2 = carry32(check + mul(u, i, k), k);
}
// the MSM record's coordinates (affine Niels, msm.h msm_store_point) from the root x (sign
// applied, limbs < 2^16 + 2^12) and y: y + x, y - x, 2d x y
NWV_HD void row_dec_record(V x, V y, const RowConsts& k, V& ypx, V& ymx, V& xy2d) {
    ypx = carry32(y + x, k);
    ymx = carry32(sub(y, x, k), k);
    xy2d = mul(mul(x, y, k), row_d2(), k);
}

// ---- points: every row holds the whole point (X, Y, Z, T one V each) ------------------------

struct RowP3 {
    V X, Y, Z, T;
};

// completed (X1 : Y1 : Z1 : T1) -> extended: rows compute X1 T1, Y1 Z1, Z1 T1, X1 Y1
NWV_HD RowP3 row_complete(V X1, V Y1, V Z1, V T1, const RowConsts& k) {
    const V o1 = carry32(rowsel(k, X1, Y1, Z1, X1), k);
    const V o2 = carry32(rowsel(k, T1, Z1, T1, Y1), k);
    RowP3 r;
    gather4(mul(o1, o2, k), r.X, r.Y, r.Z, r.T);
    return r;
}

// [2] p: rows square X, Y, Z, X + Y (T of the input unused)
NWV_HD RowP3 row_dbl(const RowP3& p, const RowConsts& k) {
    const V in = rowsel(k, p.X, p.Y, p.Z, p.X + p.Y);
    V XX, YY, ZZ, S;
    gather4(mul(in, in, k), XX, YY, ZZ, S);
    const V Y1 = YY + XX;
    const V Z1 = carry32(sub(YY, XX, k), k);
    const V X1 = sub(S, Y1, k);
    const V T1 = sub(ZZ + ZZ, Z1, k);
    return row_complete(X1, Y1, Z1, T1, k);
}

// p + q, q in cached form held row-wise: row 0 Y+X, row 1 Y-X, row 2 2dT, row 3 2Z (limbs < 2^16)
NWV_HD RowP3 row_add_cached(const RowP3& p, V qc, const RowConsts& k) {
    const V in = carry32(rowsel(k, p.Y + p.X, sub(p.Y, p.X, k), p.T, p.Z), k);
    V PP, MM, TT, ZZ;
    gather4(mul(in, qc, k), PP, MM, TT, ZZ);
    return row_complete(sub(PP, MM, k), PP + MM, ZZ + TT, sub(ZZ, TT, k), k);
}

// Horner over the window sums of an MSM layout on one wave, then [8] (the round-1 final kernel's
// chain; now the host-emulation tests' check of row_dbl / row_add_cached against the lane chain):
//   d = W_{nw-1};  d = [2^width[w]] d + W_w  for w = nw-2 .. 0;  d = [8] d.
// cq: [nw][4][16] row limbs of each window sum in cached form (Y+X | Y-X | 2dT | 2Z);
// top: [4][16] row limbs of W_{nw-1} (X | Y | Z | T).  Row 0 writes d's X | Y | Z limbs to
// out[0..48).
template <class Layout>
NWV_HD void row_horner(const uint32_t* cq, const uint32_t* top, const Layout& lay, uint32_t* out) {
    const RowConsts k = row_consts();
    const V lane = lane_id() & 63u;
    const V limb = lane & 15u;
    RowP3 d{ld(top, limb), ld(top, limb + bc(16)), ld(top, limb + bc(32)), ld(top, limb + bc(48))};
#pragma unroll 1
    for (int w = lay.nw - 2; w >= 0; w--) {
#pragma unroll 1
        for (int i = 0; i < lay.width[w]; i++) d = row_dbl(d, k);
        d = row_add_cached(d, ld(cq, bc(64u * (uint32_t)w) + lane), k);
    }
#pragma unroll 1
    for (int i = 0; i < 3; i++) d = row_dbl(d, k);
    const M r0 = row_is(0);
    st(out, limb, d.X, r0);
    st(out, limb + bc(16), d.Y, r0);
    st(out, limb + bc(32), d.Z, r0);
}

// Scaled window sum of the fused MSM tail (k_msm_tail) on one wave, from the window's bit planes:
//   W = sum_{k < m} 2^k T_k + U  ->  d = T_{m-1};  d = [2] d + T_k (k = m-2 .. 0);  d = d + U;
//   d = [2^post] d.
// planes: [m + 1][4][16] row limbs of cached points (Y+X | Y-X | 2dT | 2Z): T_0 .. T_{m-1}, then
// U.  Row 0 writes d's X | Y | Z | T limbs to out[0..64).  Multiplies by row rotations (mul_ror,
// the fastest form on gfx950: 0.340 us per doubling against 0.418 with the LDS exchange and 0.383
// with DPP shifts, profiles/round5_ubench_row.jsonl); rot = 0 selects the LDS form when sc (192
// words) is given, else the shift form (host-emulation cross-checks).
NWV_HD RowP3 row_planes_chain(const uint32_t* planes, int m, int post, uint32_t* out, uint32_t* sc = nullptr,
                              int rot = 1) {
    RowConsts k = row_consts();
    k.rot = rot;
    k.sc = rot ? nullptr : sc;
    const V lane = lane_id() & 63u;
    const V limb = lane & 15u;
    // d = identity (X = 0, Y = Z = 1, T = 0), then the planes from the top
    RowP3 d{bc(0), sel(limb_is(0), bc(0), bc(1)), sel(limb_is(0), bc(0), bc(1)), bc(0)};
#pragma unroll 1
    for (int j = m - 1; j >= 0; j--) {
        if (j < m - 1) d = row_dbl(d, k);
        d = row_add_cached(d, ld(planes, bc(64u * (uint32_t)j) + lane), k);
    }
    d = row_add_cached(d, ld(planes, bc(64u * (uint32_t)m) + lane), k);
#pragma unroll 1
    for (int i = 0; i < post; i++) d = row_dbl(d, k);
    if (out) {
        const M r0 = row_is(0);
        st(out, limb, d.X, r0);
        st(out, limb + bc(16), d.Y, r0);
        st(out, limb + bc(32), d.Z, r0);
        st(out, limb + bc(48), d.T, r0);
    }
    return d;
}

// 2d mod p in radix-2^16 limbs
NWV_HD V row_d2() {
    const uint32_t c[16] = {61785, 9906, 39828, 60374, 45398, 33411, 5274, 224,
                            53552, 61171, 33010, 6542, 64743, 22239, 55772, 9222};
    V x = bc(c[0]);
#pragma unroll
    for (int i = 1; i < 16; i++) x = sel(limb_is(i), x, bc(c[i]));
    return x;
}

// cached form of an extended point held on every row: row 0 Y+X, row 1 Y-X, row 2 2dT, row 3
// 2Z -- one row product (rows 0, 1 multiply by 1, row 2 by 2d, row 3 by 2)
NWV_HD V row_to_cached(const RowP3& d, const RowConsts& k) {
    const V in = carry32(rowsel(k, d.Y + d.X, sub(d.Y, d.X, k), d.T, d.Z), k);
    const V l0 = sel(limb_is(0), bc(0), bc(1));
    return mul(in, rowsel(k, l0, l0, row_d2(), l0 + l0), k);
}

// One step of the MSM tail's final sum: acc (X | Y | Z | T limbs, 64 words) + q (cached row form,
// lane-major: row r's limbs at 16 r) -> out (X | Y | Z | T limbs, row 0 writes them)
NWV_HD void row_ladder_step(const uint32_t* acc, const uint32_t* q, uint32_t* out, int rot = 1) {
    RowConsts k = row_consts();
    k.rot = rot;
    const V lane = lane_id() & 63u;
    const V limb = lane & 15u;
    RowP3 d{ld(acc, limb), ld(acc, limb + bc(16)), ld(acc, limb + bc(32)), ld(acc, limb + bc(48))};
    d = row_add_cached(d, ld(q, lane), k);
    const M r0 = row_is(0);
    st(out, limb, d.X, r0);
    st(out, limb + bc(16), d.Y, r0);
    st(out, limb + bc(32), d.Z, r0);
    st(out, limb + bc(48), d.T, r0);
}

}  // namespace rowf

// ---- conversions between the lane-local ten-limb form and 16-bit row limbs ----------------

// 16 limbs of 16 bits (value < 2^256) of a field element, from its canonical words
NWV_HD void fe_to_limbs16(const fe& a, uint32_t out[16]) {
    uint32_t w[8];
    fe_freeze(a, w);
#pragma unroll
    for (int k = 0; k < 16; k++) out[k] = (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
}
// field element from 16 loose limbs (each < 2^32): sum x_k 2^(16k) reduced below 2^255
NWV_HD fe fe_from_limbs16(const uint32_t x[16]) {
    uint32_t y[16];
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        t += x[k];
        y[k] = (uint32_t)t & 0xFFFFu;
        t >>= 16;
    }
    // fold 2^256 = 38 (t < 2^17), then bit 255 (2^255 = 19), twice each to settle the carries
#pragma unroll 1
    for (int it = 0; it < 2; it++) {
        uint64_t c = t * 38 + (uint64_t)(y[15] >> 15) * 19;
        y[15] &= 0x7FFFu;
        t = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            c += y[k];
            y[k] = (uint32_t)c & 0xFFFFu;
            c >>= 16;
        }
        t = c;
    }
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = y[2 * j] | (y[2 * j + 1] << 16);
    return fe_from_words(w);
}

}  // namespace nwv
