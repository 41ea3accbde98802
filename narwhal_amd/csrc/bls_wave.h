// bls_wave.h -- the BLS12-381 pairing check on one 64-lane wave (gfx950), for SURVEY.md §8 row f4.
//
// bls_group.h spreads an Fp12 over 8 lanes; a verification's pairing check is still thousands of
// dependent Fp products on those lanes (~1 us each on one wave).  Here the whole wave works on one
// item: the Miller loop and the final exponentiation are sequences of small straight-line
// PROGRAMS (tools/gen_bls_wave.py) compiled into STAGES.  In a stage every lane forms one linear
// combination of values in the wave's LDS slots (a few power-of-two-weighted terms plus 2^k p, so
// the result is non-negative: exact 32-bit limb sums and one carry pass), then either multiplies it
// by a second combination (the Montgomery product fp_mul of bls381.h) or keeps it (optionally
// reduced below 2p by the top limb), and writes the result to a slot.  An Fp12 product is one
// stage of 54 products and two stages of additions; a cyclotomic square 18 products and one stage
// of additions.  The tables (bls_wave_prog.h: slots, constants, lane records, the precomputed
// lines of g2) are generated, and the generator checks every program against its formulas
// evaluated with Python integers, and the whole pairing check against independent curve
// arithmetic; the CPU test build (tests/hostemu) runs this same interpreter against the oracle.
//
// Slot = one Fp in 14 limbs of 28 bits (Montgomery, value < 2^392).  Within a stage all reads of
// every lane precede its writes (one wave: LDS operations execute in order; the host form runs
// the lanes' reads first, then their writes).
#pragma once
#include "bls381.h"

namespace bls {
namespace wave {

struct Stage {
    uint16_t nl, nap, nan, nbp, nbn, flags, rec_len;
    uint32_t off;
};
struct Prog {
    uint16_t first, n;
};

}  // namespace wave
}  // namespace bls

#if defined(__HIP_DEVICE_COMPILE__) || (defined(__HIPCC__) && !defined(BLS_GROUP_HOST_EMU))
#define BLS_WAVE_TABLE __constant__ const
#define BLS_WAVE_DEV 1
#else
#define BLS_WAVE_TABLE static const
#endif
#include "bls_wave_prog.h"

namespace bls {
namespace wave {

constexpr int SW = NL;  // words per slot

// A lane's record in registers: REC u16 words (five 16-byte loads).  [0] destination slot, [1]
// flags (1 product, 2 reduce, 4 A signed, 8 B signed), [2] k+1 of A's 2^k p (0 none), [3] k+1 of
// B's, then A's positive terms at [4, 4+TMAX), A's negative, B's positive, B's negative, each term
// slot | weight << 12.  Every term index below is a compile-time constant after unrolling (the
// per-stage counts only predicate the loop bodies), so the record stays in VGPRs.
struct Rec {
    uint32_t w[REC / 2];
};
NWV_HD uint32_t rec_u16(const Rec& r, int i) { return (r.w[i >> 1] >> ((i & 1) * 16)) & 0xffffu; }
NWV_HD Rec load_rec(const uint16_t* p) {
    Rec r;
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int k = 0; k < REC / 8; k++) {
        const uint4 v = q[k];
        r.w[4 * k] = v.x;
        r.w[4 * k + 1] = v.y;
        r.w[4 * k + 2] = v.z;
        r.w[4 * k + 3] = v.w;
    }
    return r;
}

// the n terms of a section into 32-bit limb sums
template <int BASE>
NWV_HD void acc_terms(const uint32_t* wm, const Rec& r, int n, uint32_t* a) {
#pragma unroll
    for (int t = 0; t < TMAX; t++) {
        if (t < n) {
            const uint32_t w = rec_u16(r, BASE + t);
            const uint32_t* x = wm + SW * (w & 0xfffu);
            const int sh = (int)(w >> 12);
#pragma unroll
            for (int j = 0; j < NL; j++) a[j] += x[j] << sh;
        }
    }
}

// a combination: positive terms + 2^k p - negative terms, one carry pass (signed when the lane
// has negative terms), normalised limbs
template <int BASE>
NWV_HD fp lin_comb(const uint32_t* wm, const Rec& r, int np, int nn, uint32_t k1, bool sgn) {
    uint32_t a[NL], b[NL];
#pragma unroll
    for (int j = 0; j < NL; j++) a[j] = b[j] = 0;
    acc_terms<BASE>(wm, r, np, a);
    acc_terms<BASE + TMAX>(wm, r, nn, b);
    if (k1) {
        const uint32_t* kp = T_KP[k1 - 1];
#pragma unroll
        for (int j = 0; j < NL; j++) a[j] += kp[j];
    }
    fp v;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < NL - 1; j++) {
        const uint32_t d = a[j] - b[j] + c;
        v.l[j] = d & LM;
        c = sgn ? (uint32_t)((int32_t)d >> 28) : d >> 28;
    }
    v.l[NL - 1] = a[NL - 1] - b[NL - 1] + c;
    return v;
}

// x - q p with q = floor(top limb * QM / 2^32) <= x / p: the result is < 1.1 p (< 2p)
NWV_HD fp quick_reduce(const fp& x) {
    const uint32_t q = (uint32_t)(((uint64_t)x.l[NL - 1] * QM) >> 32);
    const fp P = k_p();
    fp r;
    int32_t c = 0;
    uint32_t hi = 0;
#pragma unroll
    for (int j = 0; j < NL - 1; j++) {
        const uint64_t qp = (uint64_t)q * P.l[j];
        const int32_t d = (int32_t)x.l[j] - (int32_t)((uint32_t)qp & LM) - (int32_t)hi + c;
        hi = (uint32_t)(qp >> 28);
        r.l[j] = (uint32_t)d & LM;
        c = d >> 28;
    }
    r.l[NL - 1] = (uint32_t)((int32_t)x.l[NL - 1] - (int32_t)(q * P.l[NL - 1]) - (int32_t)hi + c);
    return r;
}

NWV_HD fp lane_value(const uint32_t* wm, const Stage& h, const Rec& r) {
    const uint32_t fl = rec_u16(r, 1);
    fp v = lin_comb<4>(wm, r, h.nap, h.nan, rec_u16(r, 2), (fl & 4) != 0);
    if (fl & 1) {
        const fp b = lin_comb<4 + 2 * TMAX>(wm, r, h.nbp, h.nbn, rec_u16(r, 3), (fl & 8) != 0);
        v = fp_mul(v, b);
    } else if (fl & 2) {
        v = quick_reduce(v);
    }
    return v;
}

#ifdef BLS_WAVE_DEV
// ---- device: one wave, wm = its LDS slots ------------------------------------------------------
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
struct Wave {
    uint32_t* wm;
    int lane;
    __device__ void sync() const { wsync(); }
    // the program's stages; each lane's record for the next stage is loaded while this one runs
    __device__ void run(Prog p) const {
        const int end = p.first + p.n;
        Stage h = T_STAGES[p.first];
        Rec cur = load_rec(T_DATA + h.off + (uint32_t)min(lane, (int)h.nl) * REC);
#pragma unroll 1
        for (int s = p.first; s < end; s++) {
            Stage hn = h;
            Rec nxt = cur;
            if (s + 1 < end) {
                hn = T_STAGES[s + 1];
                nxt = load_rec(T_DATA + hn.off + (uint32_t)min(lane, (int)hn.nl) * REC);
            }
            if (lane < h.nl) {
                const uint32_t dst = rec_u16(cur, 0);
                const fp v = lane_value(wm, h, cur);
#pragma unroll
                for (int j = 0; j < NL; j++) wm[SW * dst + j] = v.l[j];
            }
            wsync();
            h = hn;
            cur = nxt;
        }
    }
    // up to 128 words of global memory fetched into registers ahead of use (a prefetch), and
    // written into slots later
    struct Pre {
        uint32_t a, b;
    };
    __device__ Pre fetch(const uint32_t* src, int nw) const {
        Pre p;
        p.a = lane < nw ? src[lane] : 0u;
        p.b = lane + 64 < nw ? src[lane + 64] : 0u;
        return p;
    }
    __device__ void put_pre(int slot, const Pre& p, int nw) const {
        if (lane < nw) wm[SW * slot + lane] = p.a;
        if (lane + 64 < nw) wm[SW * slot + lane + 64] = p.b;
    }
    // n consecutive slots from 14 n words (global or LDS), lane-parallel
    __device__ void put_words(int slot, const uint32_t* src, int n) const {
        for (int w = lane; w < SW * n; w += 64) wm[SW * slot + w] = src[w];
    }
    __device__ void zero(int slot, int n) const {
        for (int w = lane; w < SW * n; w += 64) wm[SW * slot + w] = 0;
    }
    __device__ void get_words(int slot, uint32_t* dst, int n) const {
        for (int w = lane; w < SW * n; w += 64) dst[w] = wm[SW * slot + w];
    }
    // fn(j) on lanes j < n (lane-local work: hashing, square roots, inversions)
    template <class Fn>
    __device__ void lanes(int n, Fn fn) const {
        if (lane < n) fn(lane);
    }
    // a value written by the calling lane
    __device__ void set(int slot, const fp& v) const {
        for (int j = 0; j < NL; j++) wm[SW * slot + j] = v.l[j];
    }
    // one value written by lane `who` (a lane-local result)
    __device__ void put_fp(int slot, const fp& v, int who = 0) const {
        if (lane == who)
            for (int j = 0; j < NL; j++) wm[SW * slot + j] = v.l[j];
    }
    __device__ fp get(int slot) const {
        fp v;
        for (int j = 0; j < NL; j++) v.l[j] = wm[SW * slot + j];
        return v;
    }
    // every lane: the 12 F slots == the Fp12 one
    __device__ bool f_is_one() const {
        bool ok = true;
        if (lane < 12) {
            const fp v = get(REG_F + lane);
            ok = lane == 0 ? fp_eq(v, k_one()) : fp_is_zero(v);
        }
        return __ballot(!ok) == 0;
    }
};
#else
// ---- host: the same programs over an array, lanes run one after another -------------------------
struct Wave {
    uint32_t* wm;
    int lane = 0;
    void sync() const {}
    void run(Prog p) const {
        fp out[64];
        uint32_t dst[64];
        for (int s = p.first; s < p.first + p.n; s++) {
            const Stage h = T_STAGES[s];
            for (int l = 0; l < h.nl; l++) {  // every lane's reads ...
                const Rec r = load_rec(T_DATA + h.off + (uint32_t)l * REC);
                dst[l] = rec_u16(r, 0);
                out[l] = lane_value(wm, h, r);
            }
            for (int l = 0; l < h.nl; l++)  // ... then its writes
                for (int j = 0; j < NL; j++) wm[SW * dst[l] + j] = out[l].l[j];
        }
    }
    struct Pre {
        const uint32_t* src;
    };
    Pre fetch(const uint32_t* src, int) const { return Pre{src}; }
    void put_pre(int slot, const Pre& p, int nw) const {
        for (int w = 0; w < nw; w++) wm[SW * slot + w] = p.src[w];
    }
    void put_words(int slot, const uint32_t* src, int n) const {
        for (int w = 0; w < SW * n; w++) wm[SW * slot + w] = src[w];
    }
    void zero(int slot, int n) const {
        for (int w = 0; w < SW * n; w++) wm[SW * slot + w] = 0;
    }
    void get_words(int slot, uint32_t* dst, int n) const {
        for (int w = 0; w < SW * n; w++) dst[w] = wm[SW * slot + w];
    }
    template <class Fn>
    void lanes(int n, Fn fn) const {
        for (int j = 0; j < n; j++) fn(j);
    }
    void set(int slot, const fp& v) const {
        for (int j = 0; j < NL; j++) wm[SW * slot + j] = v.l[j];
    }
    void put_fp(int slot, const fp& v, int = 0) const {
        for (int j = 0; j < NL; j++) wm[SW * slot + j] = v.l[j];
    }
    fp get(int slot) const {
        fp v;
        for (int j = 0; j < NL; j++) v.l[j] = wm[SW * slot + j];
        return v;
    }
    bool f_is_one() const {
        for (int k = 0; k < 12; k++) {
            const fp v = get(REG_F + k);
            if (k == 0 ? !fp_eq(v, k_one()) : !fp_is_zero(v)) return false;
        }
        return true;
    }
};
#endif

// slot 0 = 0, then the constant table
template <class W>
NWV_HD void init_slots(const W& w) {
    w.zero(0, 1);
    w.put_words(1, &T_CONSTS[0][0], NCONSTS);
    w.sync();
}

// F <- F^|x| by cyclotomic squarings (F starts as the base, which is also in register `base`)
template <class W>
NWV_HD void cyc_exp_x(const W& w, Prog mul_base) {
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        w.run(P_CYC_SQR_F);
        if ((BLS_X_ABS >> b) & 1) w.run(mul_base);
    }
}

// U <- [k] V (U = V on entry; k's top bit is bit 63), complete formulas (exact on every point)
template <class W>
NWV_HD void g1_chain(const W& w, uint64_t k) {
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        w.run(P_G1_DBL_U);
        if ((k >> b) & 1) w.run(P_G1_ADD_UV);
    }
}

// F <- F^(3 (p^12 - 1) / r), the final_exp of bls381.h; the one Fp inversion runs on lane 0
template <class W>
NWV_HD void final_exp(const W& w) {
    w.run(P_INV_A);
    const fp n = w.get(REG_N);
    w.put_fp(REG_N + 1, fp_inv_vt(n));
    w.sync();
    w.run(P_INV_B);
    w.run(P_EASY1);
    w.run(P_EASY2);
    w.run(P_COPY_F_TO_M);
    cyc_exp_x(w, P_MUL_F_M);
    w.run(P_MULCONJ_F_M);
    w.run(P_COPY_F_TO_A);
    cyc_exp_x(w, P_MUL_F_A);
    w.run(P_MULCONJ_F_A);
    w.run(P_COPY_F_TO_A);
    cyc_exp_x(w, P_MUL_F_A);
    w.run(P_CONJMULFROB_F_A);
    w.run(P_COPY_F_TO_B);
    cyc_exp_x(w, P_MUL_F_B);
    w.run(P_CONJ_F);
    w.run(P_COPY_F_TO_C);
    cyc_exp_x(w, P_MUL_F_C);
    w.run(P_CONJMULFROB2_F_B);
    w.run(P_MULCONJ2_F_B);
    w.run(P_CYCSQRM_MUL_M_TO_G);
    w.run(P_MUL_F_G);
}

// e(-sig, g2) e(H, Q) == 1 for one item, the wave's verdict on every lane:
//   sig: affine x, y (identity -> x = y = 0: pair A then contributes only its lines' l0 in Fp2,
//        which the final exponentiation maps to 1);
//   H:   homogeneous X, Y, Z (x = X / Z);  Q: Jacobian X, Y, Z (Fp2 each; affine -> Z = 1);
//   qlines: Q's precomputed line table (NSTEPS x 6 slots) or null (computed from T in the loop).
// The caller has run init_slots and filled PA (x, -y), PB, QB; this sets F = 1, TB = QB.
template <class W>
NWV_HD bool pairing_check(const W& w, const uint32_t* qlines) {
    w.zero(REG_F, 12);
    w.sync();
    w.put_fp(REG_F, k_one());
    w.put_words(REG_TB, w.wm + SW * REG_QB, 6);
    w.sync();
    const char* steps = BLS_WAVE_STEPS_STR;
    constexpr int LW = 6 * SW;  // words of a step's line
    auto la = w.fetch(&T_G2_LINES[0][0][0], LW);
    auto lb = w.fetch(qlines ? qlines : &T_G2_LINES[0][0][0], qlines ? LW : 0);
#pragma unroll 1
    for (int k = 0; k < NSTEPS; k++) {
        w.put_pre(REG_LA, la, LW);
        if (qlines) w.put_pre(REG_LB, lb, LW);
        w.sync();
        if (k + 1 < NSTEPS) {  // the next step's lines load while this step runs
            la = w.fetch(&T_G2_LINES[k + 1][0][0], LW);
            if (qlines) lb = w.fetch(qlines + (size_t)(k + 1) * LW, LW);
        }
        const bool add = steps[k] == 'a';
        w.run(qlines ? (add ? P_ML_ADD_FIXED : P_ML_DBL_FIXED) : (add ? P_ML_ADD_STEP : P_ML_DBL_STEP));
    }
    w.run(P_CONJ_F);
    final_exp(w);
    return w.f_is_one();
}

}  // namespace wave
}  // namespace bls
