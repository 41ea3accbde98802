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
#include <cassert>

#include "bls381.h"

namespace bls {
namespace wave {

// a program: its first lane record (u16 index into T_DATA), its stages, the first stage's lanes.
// A stage's records follow the previous stage's, and every record carries its stage's header (lanes,
// A's and B's term counts) and the next stage's lanes, so the interpreter walks a program from
// the records alone.
struct Prog {
    uint32_t off;
    uint16_t n, nl0;
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
// the slot words as the interpreter addresses them: LDS on the device (explicit, so the one
// out-of-line copy of the stage loop issues LDS instructions), plain memory on the host
#ifdef BLS_WAVE_DEV
typedef __attribute__((address_space(3))) uint32_t wword;
typedef __attribute__((address_space(3))) uint64_t wword2;
#else
typedef uint32_t wword;
typedef uint64_t wword2;
#endif
// the wave's LDS: P << k (k < 16, the combinations' offsets) just BELOW slot 0, then the slots:
// a kernel allocates KP_WORDS + SW x (its programs' slots) words and works from wm = base +
// KP_WORDS, so kernels that run only the pairing and G1-check programs (NSLOTS_PAIR slots) take
// less LDS -- more resident waves -- than those that also run the hash's isogeny map (NSLOTS),
// and the packed pairing kernel's banks hold only the pairing check's run of NSLOTS_PC slots
// (tools/gen_bls_wave.py lays its constants, registers and temporaries out first)
constexpr int KP_WORDS = 16 * NL;
constexpr int WM_WORDS = KP_WORDS + SW * NSLOTS;
constexpr int WM_WORDS_PAIR = KP_WORDS + SW * NSLOTS_PAIR;
constexpr int WM_WORDS_PC = KP_WORDS + SW * NSLOTS_PC;

// A lane's record in registers: REC u16 words (five 16-byte loads).  [0] destination slot, [1]
// flags (1 product, 2 reduce, 4 A signed, 8 B signed), [2] k+1 of A's 2^k p (0 none), [3] k+1 of
// B's, then A's positive terms at [4, 4+TMAX), A's negative, B's positive, B's negative, each term
// slot | weight << 12.  Every term index below is a compile-time constant after unrolling (the
// per-stage counts only predicate the loop bodies), so the record stays in VGPRs.
struct Rec {
    uint32_t w[REC / 2];
};
NWV_HD uint32_t rec_u16(const Rec& r, int i) { return (r.w[i >> 1] >> ((i & 1) * 16)) & 0xffffu; }
// the stage header at the record's end
struct Hdr {
    int nl, nap, nan, nbp, nbn, nl_next;
};
NWV_HD Hdr rec_hdr(const Rec& r) {
    const uint32_t a = r.w[REC / 2 - 2], b = r.w[REC / 2 - 1];  // (nl | na << 16), (nb | nl_next << 16)
    Hdr h;
    h.nl = (int)(a & 0xffffu);
    h.nap = (int)((a >> 16) & 0xffu);
    h.nan = (int)(a >> 24);
    h.nbp = (int)(b & 0xffu);
    h.nbn = (int)((b >> 8) & 0xffu);
    h.nl_next = (int)(b >> 16);
    return h;
}
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

// A combination's limb sums: the offset 2^k p (when the lane has negative terms) is stored in a
// redundant form whose limbs 0..12 are each >= 2^31 - 8 >= the most that 8 units of negative
// terms can take from a limb (T_KP: P << k with 8 borrowed from each next limb), so every limb
// sum below the top is a non-negative 32-bit value (< 2^32 with <= 7 positive units; <= 16 units
// without negative terms) and only the top limb can be negative (the value never is).
//
// n terms of a section (n wave-uniform: one switch, then every LDS read in flight at once -- one
// wave per SIMD has nothing else to hide their latency behind -- then the sums)
// Limb sums are kept as seven packed pairs (limb 2j in the low half of a 64-bit word, 2j+1 in the
// high half): a slot's 8-byte LDS words are already such pairs, a term is seven 64-bit
// shift-and-adds (v_lshl_add_u64), and no half ever carries into the next (every limb sum stays
// below 2^32, and a term's shift of <= 3 keeps a 28-bit limb inside its half).
template <int BASE, int N>
NWV_HD void acc_n(const wword* wm, const Rec& r, uint64_t* a) {
    uint64_t x[N][NL / 2];
    int sh[N];
#pragma unroll
    for (int u = 0; u < N; u++) {
        const uint32_t w = rec_u16(r, BASE + u);
        // a slot is 56 bytes at an 8-byte aligned offset: seven 8-byte reads
        const wword2* p = reinterpret_cast<const wword2*>(wm + SW * (w & 0xfffu));
        sh[u] = (int)(w >> 12);
#pragma unroll
        for (int j = 0; j < NL / 2; j++) x[u][j] = p[j];
    }
#pragma unroll
    for (int u = 0; u < N; u++)
#pragma unroll
        for (int j = 0; j < NL / 2; j++) a[j] += x[u][j] << sh[u];
}
// at most G terms' reads in flight at once (8: all of a section's; 4 halves the registers they
// hold, for the packed pairing kernel, which must fit two waves per SIMD)
template <int BASE, int G = 8>
NWV_HD void acc_terms(const wword* wm, const Rec& r, int n, uint64_t* a) {
    if (G < 8 && n > G) {
        acc_n<BASE, (G < 8 ? G : 1)>(wm, r, a);
        switch (n - G) {
            case 1: acc_n<BASE + G, 1>(wm, r, a); break;
            case 2: acc_n<BASE + G, 2>(wm, r, a); break;
            case 3: acc_n<BASE + G, 3>(wm, r, a); break;
            case 4: acc_n<BASE + G, 4>(wm, r, a); break;
            default: break;
        }
        return;
    }
    switch (n) {
        case 1: acc_n<BASE, 1>(wm, r, a); break;
        case 2: acc_n<BASE, 2>(wm, r, a); break;
        case 3: acc_n<BASE, 3>(wm, r, a); break;
        case 4: acc_n<BASE, 4>(wm, r, a); break;
        case 5: acc_n<BASE, 5>(wm, r, a); break;
        case 6: acc_n<BASE, 6>(wm, r, a); break;
        case 7: acc_n<BASE, 7>(wm, r, a); break;
        case 8: acc_n<BASE, 8>(wm, r, a); break;
        default: break;
    }
}
// the limb sums of a combination: positive terms + 2^k p - negative terms (the subtraction per
// 32-bit limb: with the redundant offset no limb below the top goes negative)
// (kpt: the P << k table, KP_WORDS words; a one-item wave keeps it just below slot 0)
template <int BASE, int G = 8>
NWV_HD void comb_sums(const wword* wm, const wword* kpt, const Rec& r, int np, int nn, uint32_t k1, uint32_t* out) {
    uint64_t a[NL / 2];
    if (k1) {
        const wword2* kp = reinterpret_cast<const wword2*>(kpt + NL * (k1 - 1));
#pragma unroll
        for (int j = 0; j < NL / 2; j++) a[j] = kp[j];
    } else {
#pragma unroll
        for (int j = 0; j < NL / 2; j++) a[j] = 0;
    }
    acc_terms<BASE, G>(wm, r, np, a);
    if (nn) {
        uint64_t b[NL / 2];
#pragma unroll
        for (int j = 0; j < NL / 2; j++) b[j] = 0;
        acc_terms<BASE + TMAX, G>(wm, r, nn, b);
#pragma unroll
        for (int j = 0; j < NL / 2; j++) {
            out[2 * j] = (uint32_t)a[j] - (uint32_t)b[j];
            out[2 * j + 1] = (uint32_t)(a[j] >> 32) - (uint32_t)(b[j] >> 32);
        }
    } else {
#pragma unroll
        for (int j = 0; j < NL / 2; j++) {
            out[2 * j] = (uint32_t)a[j];
            out[2 * j + 1] = (uint32_t)(a[j] >> 32);
        }
    }
}
template <int BASE>
NWV_HD void comb_sums(const wword* wm, const Rec& r, int np, int nn, uint32_t k1, uint32_t* out) {
    comb_sums<BASE>(wm, wm - KP_WORDS, r, np, nn, k1, out);
}
// normalised limbs (< 2^28): one sequential carry pass (the top limb takes the rest)
NWV_HD fp carry_seq(const uint32_t* a) {
    fp v;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < NL - 1; j++) {
        const uint32_t d = a[j] + c;
        v.l[j] = d & LM;
        c = d >> 28;
    }
    v.l[NL - 1] = a[NL - 1] + c;
    return v;
}
// a product operand: limbs below 2^28 + 16, each from its own sum and the one below (no carry
// chain); fp_mul takes such limbs.  A negative top limb (possible only for a value within 2^-24 of
// a multiple of 2^364) takes the sequential pass.
NWV_HD fp carry_par(const uint32_t* a) {
    fp v;
    v.l[0] = a[0] & LM;
#pragma unroll
    for (int j = 1; j < NL - 1; j++) v.l[j] = (a[j] & LM) + (a[j - 1] >> 28);
    v.l[NL - 1] = a[NL - 1] + (a[NL - 2] >> 28);
    if ((int32_t)v.l[NL - 1] < 0) v = carry_seq(a);
    return v;
}
// a combination as a normalised value (the tests' and the G1/G2 helpers' form)
template <int BASE>
NWV_HD fp lin_comb(const wword* wm, const Rec& r, int np, int nn, uint32_t k1, bool) {
    uint32_t a[NL];
    comb_sums<BASE>(wm, r, np, nn, k1, a);
    return carry_seq(a);
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

template <int G = 8>
NWV_HD fp lane_value(const wword* wm, const wword* kpt, const Hdr& h, const Rec& r) {
    const uint32_t fl = rec_u16(r, 1);
    uint32_t a[NL];
    comb_sums<4, G>(wm, kpt, r, h.nap, h.nan, rec_u16(r, 2), a);
    fp v;
    if (fl & 1) {
        uint32_t b[NL];
        comb_sums<4 + 2 * TMAX, G>(wm, kpt, r, h.nbp, h.nbn, rec_u16(r, 3), b);
        v = fp_mul(carry_par(a), carry_par(b));
    } else {
        v = carry_seq(a);
        if (fl & 2) v = quick_reduce(v);
    }
    return v;
}
NWV_HD fp lane_value(const wword* wm, const Hdr& h, const Rec& r) { return lane_value<8>(wm, wm - KP_WORDS, h, r); }

// ---- the pairing check as one flat script ------------------------------------------------------
// The throughput kernel (k_blsw_pair_k) runs a whole pairing check as ONE loop over a script of
// ops instead of one interpreter call per program run: an out-of-line interpreter call saves and
// restores the callee-saved VGPRs it uses (~100 per lane) through scratch memory on every call, and
// a check makes a few hundred calls -- that was ~616 KB of scratch writes per item and 31 K VMEM
// instructions per wave (profiles/round5_bls_pmc_n16384.json).  With the stage loop at
// one call site the kernel makes no calls in the loop.  Ops: RUN a program `reps` times over; LINES,
// the Miller loop's next step lines into every bank (prefetched one step ahead); INV, each item's
// Fp inversion (the final exponentiation's one).  next_run links every op to the next RUN op, so
// the interpreter loads that op's first lane record while the current op runs.  The script is built
// from the same templates as pairing_check / final_exp (a recording W), so there is one definition
// of the sequence.
enum : uint32_t { SOP_RUN = 0, SOP_LINES = 1, SOP_INV = 2 };
struct SOp {
    uint32_t a;         // RUN: program offset; LINES: step; INV: destination slot
    uint32_t b;         // RUN: stages | first stage's lanes << 16; INV: source slot
    uint32_t c;         // reps | kind << 16
    int32_t next_run;   // index of the next RUN op, -1 at the end
};
constexpr int SCRIPT_MAX = 512;
struct ScriptRec {
    SOp* ops;
    int* n;
    void sync() const {}
    void run(Prog p, int reps = 1) const {
        if (reps <= 0) return;
        ops[(*n)++] = SOp{p.off, (uint32_t)p.n | ((uint32_t)p.nl0 << 16), (uint32_t)reps | (SOP_RUN << 16), -1};
    }
    void invert_slot(int dst, int src) const {
        ops[(*n)++] = SOp{(uint32_t)dst, (uint32_t)src, 1u | (SOP_INV << 16), -1};
    }
};
inline uint32_t sop_kind(const SOp& o) { return o.c >> 16; }

#ifdef BLS_WAVE_DEV
// ---- device: one wave, wm = its LDS slots ------------------------------------------------------
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// the program's stages; each lane's record for the next stage is loaded while this one runs (a
// lane past a stage's last record loads the last one: every record holds the header).  One copy
// of the interpreter per kernel (not inlined at every call site): the kernels stay within the
// instruction cache.
__device__ __attribute__((noinline)) void wave_run(uint32_t* wm_generic, int lane, uint32_t off, int n, int nl0,
                                                   int reps) {
    wword* wm = (wword*)wm_generic;
    const uint16_t* base0 = T_DATA + off;
    const uint16_t* base = base0;
    int nl = nl0;
    Rec cur = load_rec(base0 + (uint32_t)min(lane, nl0 - 1) * REC);
    const int total = n * reps;
#pragma unroll 1
    for (int t = 0, s = 0; t < total; t++) {
        Hdr h = rec_hdr(cur);
        h.nap = __builtin_amdgcn_readfirstlane(h.nap);  // wave-uniform: term counts in SGPRs
        h.nan = __builtin_amdgcn_readfirstlane(h.nan);
        h.nbp = __builtin_amdgcn_readfirstlane(h.nbp);
        h.nbn = __builtin_amdgcn_readfirstlane(h.nbn);
        const bool wrap = s + 1 == n;  // the program's last stage: the next one is its first again
        const int nl_next = wrap ? nl0 : __builtin_amdgcn_readfirstlane(h.nl_next);
        const uint16_t* nbase = wrap ? base0 : base + (uint32_t)nl * REC;
        Rec nxt = cur;
        if (t + 1 < total) nxt = load_rec(nbase + (uint32_t)min(lane, nl_next - 1) * REC);
        if (lane < nl) {
            const uint32_t dst = rec_u16(cur, 0);
            const fp v = lane_value(wm, h, cur);
#pragma unroll
            for (int j = 0; j < NL; j++) wm[SW * dst + j] = v.l[j];
        }
        wsync();
        base = nbase;
        nl = nl_next;
        cur = nxt;
        s = wrap ? 0 : s + 1;
    }
}
// k items on one wave (the throughput path): item j's slots in bank j (the one-item layout: P << k
// below its slot 0), banks `bank` words apart.  A stage of nl lanes per item runs 64 / nl items per
// pass (lane l: item l / nl of the pass, record l % nl), ceil(k / (64 / nl)) passes, then one wave
// sync.  So the narrow stages -- the final exponentiation's cyclotomic squarings (18 products, then
// 12 combinations), which are most of a pairing check's stages -- run k items for the instructions
// of one, and a wide one (an Fp12 product's 54) takes k passes as k waves would.  The pairing
// kernel's time did not move with 4 instead of 10 resident waves per CU (LDS padded per wave, 37.5
// ms for 16,384 items either way, profiles/round5_bls_occupancy.txt): one wave per SIMD already
// keeps its VALU busy, so fewer instructions per item is what raises throughput.
__device__ __attribute__((noinline)) void wave_run_k(uint32_t* wm0_generic, uint32_t bank, int k, int lane,
                                                     uint32_t off, int n, int nl0, int reps) {
    wword* wm0 = (wword*)wm0_generic;
    const uint16_t* base0 = T_DATA + off;
    const uint16_t* base = base0;
    int nl = nl0;
    Rec cur = load_rec(base0 + (uint32_t)(lane % nl0) * REC);
    const int total = n * reps;
#pragma unroll 1
    for (int t = 0, s = 0; t < total; t++) {
        Hdr h = rec_hdr(cur);
        h.nap = __builtin_amdgcn_readfirstlane(h.nap);
        h.nan = __builtin_amdgcn_readfirstlane(h.nan);
        h.nbp = __builtin_amdgcn_readfirstlane(h.nbp);
        h.nbn = __builtin_amdgcn_readfirstlane(h.nbn);
        const bool wrap = s + 1 == n;
        const int nl_next = wrap ? nl0 : __builtin_amdgcn_readfirstlane(h.nl_next);
        const uint16_t* nbase = wrap ? base0 : base + (uint32_t)nl * REC;
        Rec nxt = cur;
        if (t + 1 < total) nxt = load_rec(nbase + (uint32_t)(lane % nl_next) * REC);
        const int ipp = 64 / nl, first = lane / nl;
        if (first < ipp) {
            const uint32_t dst = rec_u16(cur, 0);
#pragma unroll 1
            for (int item = first; item < k; item += ipp) {
                wword* wm = wm0 + (uint32_t)item * bank;
                const fp v = lane_value(wm, h, cur);
#pragma unroll
                for (int j = 0; j < NL; j++) wm[SW * dst + j] = v.l[j];
            }
        }
        wsync();
        base = nbase;
        nl = nl_next;
        cur = nxt;
        s = wrap ? 0 : s + 1;
    }
}
// The Wave interface over k banks (final_exp, exp_chain and cyc_exp_x run on it unchanged)
struct WaveK {
    uint32_t* wm;   // bank 0's slot 0
    uint32_t bank;  // words from one bank to the next
    int k;          // items
    int lane;
    __device__ uint32_t* bk(int j) const { return wm + (uint32_t)j * bank; }
    __device__ void sync() const { wsync(); }
    __device__ void run(Prog p, int reps = 1) const { wave_run_k(wm, bank, k, lane, p.off, p.n, p.nl0, reps); }
    __device__ void zero(int slot, int n) const {
        for (int j = 0; j < k; j++)
            for (int w = lane; w < SW * n; w += 64) bk(j)[SW * slot + w] = 0;
    }
    __device__ void copy_slots(int dst, int src, int n) const {
        for (int j = 0; j < k; j++)
            for (int w = lane; w < SW * n; w += 64) bk(j)[SW * dst + w] = bk(j)[SW * src + w];
    }
    // item j's words (global or LDS) into its bank
    __device__ void put_words(int j, int slot, const uint32_t* src, int n) const {
        for (int w = lane; w < SW * n; w += 64) bk(j)[SW * slot + w] = src[w];
    }
    // a value every lane holds, written to item j's bank (j < 0: every bank) by lane 0
    __device__ void put_fp(int j, int slot, const fp& v) const {
        if (lane != 0) return;
        for (int b = j < 0 ? 0 : j; b < (j < 0 ? k : j + 1); b++)
            for (int i = 0; i < NL; i++) bk(b)[SW * slot + i] = v.l[i];
    }
    __device__ fp get(int j, int slot) const {
        fp v;
        for (int i = 0; i < NL; i++) v.l[i] = bk(j)[SW * slot + i];
        return v;
    }
    // each item's inverse, one wave-wide inversion after another
    __device__ void invert_slot(int dst, int src) const {
        for (int j = 0; j < k; j++) {
            const fp x = get(j, src);
            put_fp(j, dst, fp_inv_wave(x));
        }
    }
    // bit j set when item j's 12 F slots are the Fp12 one (lanes 12 j .. 12 j + 11, k <= 5)
    __device__ uint32_t f_is_one_mask() const {
        const int j = lane / 12, c = lane % 12;
        bool bad = false;
        if (j < k) {
            const fp v = get(j, REG_F + c);
            bad = c == 0 ? !fp_eq(v, k_one()) : !fp_is_zero(v);
        }
        const uint64_t b = __ballot(bad);
        uint32_t ok = 0;
        for (int i = 0; i < k; i++)
            if (((b >> (12 * i)) & 0xfffull) == 0) ok |= 1u << i;
        return ok;
    }
};

struct Wave {
    uint32_t* wm;
    int lane;
    __device__ void sync() const { wsync(); }
    // x^-1 for a wave-uniform x (every lane calls it; the four update rows on four lanes)
    __device__ fp inv(const fp& x) const { return fp_inv_wave(x); }
    // the program `reps` times over (one call: runs of squarings / doublings)
    __device__ void run(Prog p, int reps = 1) const { wave_run(wm, lane, p.off, p.n, p.nl0, reps); }
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
    // n slots copied within the wave's LDS
    __device__ void copy_slots(int dst, int src, int n) const { put_words(dst, wm + SW * src, n); }
    // slot dst <- slot src ^ -1 (every lane reads the value; the four update rows on four lanes)
    __device__ void invert_slot(int dst, int src) const { put_fp(dst, inv(get(src))); }
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
    fp inv(const fp& x) const { return inv_rows(x); }
    void run(Prog p, int reps) const {
        for (int r = 0; r < reps; r++) run(p);
    }
    void run(Prog p) const {
        fp out[64];
        uint32_t dst[64];
        const uint16_t* base = T_DATA + p.off;
        int nl = p.nl0;
        for (int s = 0; s < (int)p.n; s++) {
            int nl_next = 0;
            for (int l = 0; l < nl; l++) {  // every lane's reads ...
                const Rec r = load_rec(base + (uint32_t)l * REC);
                const Hdr h = rec_hdr(r);
                assert(h.nl == nl);
                nl_next = h.nl_next;
                dst[l] = rec_u16(r, 0);
                out[l] = lane_value(wm, h, r);
            }
            for (int l = 0; l < nl; l++)  // ... then its writes
                for (int j = 0; j < NL; j++) wm[SW * dst[l] + j] = out[l].l[j];
            base += (uint32_t)nl * REC;
            nl = nl_next;
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
    void copy_slots(int dst, int src, int n) const { put_words(dst, wm + SW * src, n); }
    void invert_slot(int dst, int src) const { put_fp(dst, inv(get(src))); }
    bool f_is_one() const {
        for (int k = 0; k < 12; k++) {
            const fp v = get(REG_F + k);
            if (k == 0 ? !fp_eq(v, k_one()) : !fp_is_zero(v)) return false;
        }
        return true;
    }
};
#endif

// slot 0 = 0, the pairing check's constants at slots 1.., the others at CONST2_SLOT..; P << k
// below slot 0
template <class W>
NWV_HD void init_slots(const W& w) {
    w.zero(0, 1);
    w.put_words(1, &T_CONSTS[0][0], NCONSTS_PC);
    w.put_words(CONST2_SLOT, &T_CONSTS[NCONSTS_PC][0], NCONSTS - NCONSTS_PC);
    w.put_words(-16, &T_KP[0][0], 16);  // below slot 0
    w.sync();
}
// a packed pairing bank of NSLOTS_PC slots: slot 0, the pairing check's constants, P << k
template <class W>
NWV_HD void init_slots_pc(const W& w) {
    w.zero(0, 1);
    w.put_words(1, &T_CONSTS[0][0], NCONSTS_PC);
    w.put_words(-16, &T_KP[0][0], 16);
    w.sync();
}
#ifdef BLS_WAVE_DEV
// the device form: every lane fetches all its words of both tables before storing any (one memory
// round trip; put_words' loop waits for each 64-word load in turn).  PC_ONLY: a bank of
// NSLOTS_PC slots (the packed pairing kernel), which the other constants lie beyond.
template <bool PC_ONLY>
__device__ __forceinline__ void init_slots_t(const Wave& w) {
    constexpr int NC = SW * (PC_ONLY ? NCONSTS_PC : NCONSTS), NC1 = SW * NCONSTS_PC, NK = 16 * SW;
    constexpr int NT = (NC + NK + 63) / 64;
    const uint32_t* c = &T_CONSTS[0][0];
    const uint32_t* k = &T_KP[0][0];
    uint32_t v[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int i = w.lane + 64 * t;
        v[t] = i < NC ? c[i] : i < NC + NK ? k[i - NC] : 0u;
    }
    if (w.lane < SW) w.wm[w.lane] = 0;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int i = w.lane + 64 * t;
        if (i < NC1) w.wm[SW + i] = v[t];
        else if (i < NC) w.wm[SW * CONST2_SLOT + (i - NC1)] = v[t];
        else if (i < NC + NK) w.wm[(i - NC) - KP_WORDS] = v[t];
    }
    w.sync();
}
__device__ __forceinline__ void init_slots(const Wave& w) { init_slots_t<false>(w); }
__device__ __forceinline__ void init_slots_pc(const Wave& w) { init_slots_t<true>(w); }
#endif

// the square-and-multiply chain of a 64-bit k (top bit 63) below its top bit: each run of
// squarings (doublings) up to the next set bit is one interpreter call
template <class W>
NWV_HD void exp_chain(const W& w, uint64_t k, Prog sq, Prog mul) {
    int b = 62;
    while (b >= 0) {
        int r = 0;
        while (b - r >= 0 && !((k >> (b - r)) & 1)) r++;
        if (b - r < 0) {  // trailing zeros: squarings only
            w.run(sq, r);
            break;
        }
        w.run(sq, r + 1);  // the zeros, then the set bit's squaring
        w.run(mul);
        b -= r + 1;
    }
}

// F <- F^|x| by cyclotomic squarings (F starts as the base, which is also in register `base`)
template <class W>
NWV_HD void cyc_exp_x(const W& w, Prog mul_base) {
    exp_chain(w, BLS_X_ABS, P_CYC_SQR_F, mul_base);
}

// U <- [k] V (U = V on entry; k's top bit is bit 63), complete formulas (exact on every point)
template <class W>
NWV_HD void g1_chain(const W& w, uint64_t k) {
    exp_chain(w, k, P_G1_DBL_U, P_G1_ADD_UV);
}

// F <- F^(3 (p^12 - 1) / r), the final_exp of bls381.h; the one Fp inversion runs on lane 0
template <class W>
NWV_HD void final_exp(const W& w) {
    w.run(P_INV_A);
    w.invert_slot(REG_N + 1, REG_N);  // the norm's inverse (every lane reads the norm)
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
    w.run(P_CYCSQR_M_TO_G);
    w.run(P_MUL_G_M);
    w.run(P_MUL_F_G);
}

// e(-sig, g2) e(H, Q) == 1 for one item, the wave's verdict on every lane:
//   sig: affine x, y (identity -> x = y = 0: pair A then contributes only its lines' l0 in Fp2,
//        which the final exponentiation maps to 1);
//   H:   homogeneous X, Y, Z (x = X / Z);  Q: Jacobian X, Y, Z (Fp2 each; affine -> Z = 1);
//   qlines: Q's precomputed line table (NSTEPS x 6 slots) or null (computed from T in the loop);
//   two_step: with qlines, the one- to three-step programs of BLS_WAVE_GROUPS_STR (NSLOTS_PAIR2
//   slots), else one program a step (NSLOTS_PC slots suffice).
// The caller has run init_slots and filled PA (x, -y), PB, QB; this sets F = 1, TB = QB.
template <class W>
NWV_HD bool pairing_check(const W& w, const uint32_t* qlines, bool two_step = true) {
    w.zero(REG_F, 12);
    w.sync();
    w.put_fp(REG_F, k_one());
    w.copy_slots(REG_TB, REG_QB, 6);
    w.sync();
    const char* steps = BLS_WAVE_STEPS_STR;
    constexpr int LW = 6 * SW;  // words of a step's line
    if (qlines && two_step) {
        // both pairs' lines precomputed: programs of one to three steps (BLS_WAVE_GROUPS_STR: a
        // multi-step program folds each step's output combinations into the next one's operands
        // and schedules the later steps' line products beside the first's work: 308 stages
        // against 408), the lines of the group's steps in LA / LB, LA2 / LB2, LA3 / LB3, the next
        // group's fetched while this one runs (LDS of NSLOTS_PAIR2 slots)
        const char* groups = BLS_WAVE_GROUPS_STR;
        auto la = w.fetch(&T_G2_LINES[0][0][0], LW), lb = w.fetch(qlines, LW);
        auto la2 = w.fetch(&T_G2_LINES[1][0][0], LW), lb2 = w.fetch(qlines + LW, LW);
        auto la3 = w.fetch(&T_G2_LINES[2][0][0], LW), lb3 = w.fetch(qlines + 2 * LW, LW);
        int k = 0;
#pragma unroll 1
        for (int g = 0; g < NGROUPS; g++) {
            const char c = groups[g];
            const int ns = (c == 'd' || c == 'a') ? 1 : (c == 'D' || c == 'E' || c == 'A') ? 2 : 3;
            w.put_pre(REG_LA, la, LW);
            w.put_pre(REG_LB, lb, LW);
            if (ns > 1) {
                w.put_pre(REG_LA2, la2, LW);
                w.put_pre(REG_LB2, lb2, LW);
            }
            if (ns > 2) {
                w.put_pre(REG_LA3, la3, LW);
                w.put_pre(REG_LB3, lb3, LW);
            }
            w.sync();
            k += ns;
            if (k < NSTEPS) {
                la = w.fetch(&T_G2_LINES[k][0][0], LW);
                lb = w.fetch(qlines + (size_t)k * LW, LW);
            }
            if (k + 1 < NSTEPS) {
                la2 = w.fetch(&T_G2_LINES[k + 1][0][0], LW);
                lb2 = w.fetch(qlines + (size_t)(k + 1) * LW, LW);
            }
            if (k + 2 < NSTEPS) {
                la3 = w.fetch(&T_G2_LINES[k + 2][0][0], LW);
                lb3 = w.fetch(qlines + (size_t)(k + 2) * LW, LW);
            }
            Prog p = P_ML_DBL_FIXED;
            switch (c) {
                case 'a': p = P_ML_ADD_FIXED; break;
                case 'D': p = P_ML2_DD_FIXED; break;
                case 'E': p = P_ML2_DA_FIXED; break;
                case 'A': p = P_ML2_AD_FIXED; break;
                case 'T': p = P_ML3_DDD_FIXED; break;
                case 'U': p = P_ML3_DDA_FIXED; break;
                case 'V': p = P_ML3_DAD_FIXED; break;
                case 'W': p = P_ML3_ADD_FIXED; break;
                default: break;
            }
            w.run(p);
        }
        w.run(P_CONJ_F);
        final_exp(w);
        return w.f_is_one();
    }
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
        const Prog pd = qlines ? P_ML_DBL_FIXED : P_ML_DBL_STEP, pa = qlines ? P_ML_ADD_FIXED : P_ML_ADD_STEP;
        w.run(steps[k] == 'a' ? pa : pd);
    }
    w.run(P_CONJ_F);
    final_exp(w);
    return w.f_is_one();
}

// the ops of pairing_check after its set-up (F = 1, TB = QB): the Miller loop with precomputed key
// lines (fixed) or computed ones, the conjugation, the final exponentiation.  Returns the count.
inline int pairing_script(bool fixed, SOp* ops) {
    int n = 0;
    const ScriptRec w{ops, &n};
    const char* steps = BLS_WAVE_STEPS_STR;
    // with both lines precomputed, the steps scheduled into stages of at most 21 lanes (mlp_*:
    // three items of a packed wave share every pass; a doubling takes 9 passes for three items
    // against 11 for ml_dbl_fixed's 46- and 51-lane stages)
    const Prog pd = fixed ? P_MLP_DBL_FIXED : P_ML_DBL_STEP, pa = fixed ? P_MLP_ADD_FIXED : P_ML_ADD_STEP;
    for (int k = 0; k < NSTEPS; k++) {
        ops[n++] = SOp{(uint32_t)k, 0u, 1u | (SOP_LINES << 16), -1};
        w.run(steps[k] == 'a' ? pa : pd);
    }
    w.run(P_CONJ_F);
    final_exp(w);
    int nxt = -1;
    for (int i = n - 1; i >= 0; i--) {
        ops[i].next_run = nxt;
        if (sop_kind(ops[i]) == SOP_RUN) nxt = i;
    }
    return n;
}

}  // namespace wave
}  // namespace bls
