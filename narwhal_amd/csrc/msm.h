// msm.h -- lane-level pieces of the batch-verification multi-scalar multiplication (K5).
//
// Restates ed25519_consensus 2.0.1 batch::Verifier::verify (SURVEY.md Appendix A "Batch
// verify"; called through fastcrypto's Ed25519 verify_batch_empty_fail / AggregateSignature
// ::verify from Certificate::verify, types/src/primary.rs:531-534): for n signatures with
// random 128-bit z_i the batch is accepted iff
//     [8]( -(sum z_i s_i) B  +  sum z_i R_i  +  sum (z_i k_i) A_i ) == identity.
// Any undecodable R/A or non-canonical s rejects the whole batch, exactly as the reference.
// A single invalid signature makes the check fail deterministically (its error term has a
// nonzero prime-order component and 0 < z_i < l); several can cancel with probability
// ~2^-128, the same bound as the reference's.
//
// The MSM is Pippenger's bucket method over 2n + 1 points laid out as
//     j in [0, n)        A_i   scalar z_i k_i mod l   (253 bits)
//     j = n              B     scalar -sum z_i s_i mod l
//     j in [n+1, 2n+1)   R_i   scalar z_i             (128 bits)
// so that the windows above bit 128 only visit the prefix [0, n]. Scalars are recoded to signed
// digits over the windows of an MsmLayout; bucket |d| - 1 of window w collects sign(d) P_j.
// Everything here is __host__ __device__ so tests/hostemu can run the same arithmetic on the
// CPU with limb-bound assertions.
#pragma once
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"

namespace nwv {

static constexpr int P3_WORDS = 40;  // X | Y | Z | T, ten carried limbs each

NWV_HD void store_p3(uint32_t* d, const ge_p3& p) {
    store_fe(d, p.X);
    store_fe(d + 10, p.Y);
    store_fe(d + 20, p.Z);
    store_fe(d + 30, p.T);
}
NWV_HD ge_p3 load_p3(const uint32_t* s) {
    return ge_p3{load_fe(s), load_fe(s + 10), load_fe(s + 20), load_fe(s + 30)};
}
NWV_HD ge_p3 p3_add(const ge_p3& a, const ge_p3& b) {
    return ge_p1p1_to_p3(ge_add(a, ge_p3_to_cached(b)));
}
// [2^k] p, k >= 1, through the projective doubling chain
NWV_HD ge_p3 p3_dbl_n(const ge_p3& p, int k) {
    ge_p2 r = ge_p3_to_p2(p);
    ge_p1p1 t = ge_p2_dbl(r);
#pragma unroll 1
    for (int i = 1; i < k; i++) {
        r = ge_p1p1_to_p2(t);
        t = ge_p2_dbl(r);
    }
    return ge_p1p1_to_p3(t);
}
// [8] p == identity (the cofactored acceptance test)
NWV_HD bool p3_mul8_is_identity(const ge_p3& p) {
    ge_p2 q = ge_p3_to_p2(p);
    ge_p1p1 t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    return ge_p1p1_is_identity(t);
}

// ChaCha20 block function (RFC 8439 2.3): 16 output words for key[8], 32-bit block counter and
// nonce[3].
NWV_HD uint32_t chacha_rotl(uint32_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(x, x, 32 - n);
#else
    return (x << n) | (x >> (32 - n));
#endif
}
NWV_HD void chacha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d = chacha_rotl(d ^ a, 16);
    c += d; b = chacha_rotl(b ^ c, 12);
    a += b; d = chacha_rotl(d ^ a, 8);
    c += d; b = chacha_rotl(b ^ c, 7);
}
NWV_HD void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], counter, nonce[0], nonce[1], nonce[2]};
    uint32_t s[16];
#pragma unroll
    for (int k = 0; k < 16; k++) s[k] = x[k];
#pragma unroll 2
    for (int r = 0; r < 10; r++) {
        chacha_qr(x[0], x[4], x[8], x[12]);
        chacha_qr(x[1], x[5], x[9], x[13]);
        chacha_qr(x[2], x[6], x[10], x[14]);
        chacha_qr(x[3], x[7], x[11], x[15]);
        chacha_qr(x[0], x[5], x[10], x[15]);
        chacha_qr(x[1], x[6], x[11], x[12]);
        chacha_qr(x[2], x[7], x[8], x[13]);
        chacha_qr(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) out[k] = x[k] + s[k];
}

// Per-signature random coefficient z_i in [1, 2^128), odd: the first 16 bytes of the ChaCha20 block
// keyed by the caller's 32-byte seed with counter = low word of i and nonce = (high word of i,
// "nwv-", "z128").  ed25519-consensus draws z_i from the thread RNG (a ChaCha CSPRNG in rand);
// here the caller's CSPRNG seed keys the stream so the kernels need no device RNG state.
// The low bit is forced to 1 (127 random bits): z_i != 0, so a batch holding one invalid
// signature fails deterministically -- a one-signature batch verdict is then exactly the
// signature's ZIP-215 verdict (nwv_ed25519_pubkey_verify relies on it).
NWV_HD void msm_z(const uint32_t seed[8], uint64_t i, uint32_t z[8]) {
    const uint32_t nonce[3] = {(uint32_t)(i >> 32), 0x2d76776eu /* "nwv-" */, 0x3832317au /* "z128" */};
    uint32_t blk[16];
    chacha20_block(seed, (uint32_t)i, nonce, blk);
#pragma unroll
    for (int k = 0; k < 8; k++) z[k] = k < 4 ? blk[k] : 0u;
    z[0] |= 1u;
}

// Window layout.  Windows have near-equal widths <= c chosen so that every window's bucket range
// is fully used (no skewed top window):  widths 0..nw_z-1 sum to 129 = 128 bits of z plus the
// signed-digit headroom, and all nw windows sum to 254 = 253 bits of a scalar mod l plus headroom.
// The top window of each range holds width-1 raw bits plus the incoming carry, i.e. digits in
// [0, 2^(width-1)], exactly the bucket range of the window; every lower window holds signed
// digits in [-2^(width-1), 2^(width-1)).  Bucket key of digit d in window w: kbase[w] + |d| - 1.
static constexpr int MSM_MAX_WINDOWS = 48;
static constexpr int MSM_BITS_FULL = 253;  // scalars mod l
static constexpr int MSM_BITS_Z = 128;     // z_i

struct MsmLayout {
    int32_t nw, nw_z, cmax, pad;
    uint8_t width[MSM_MAX_WINDOWS];
    uint16_t pos[MSM_MAX_WINDOWS];
    uint32_t kbase[MSM_MAX_WINDOWS + 1];  // kbase[nw] = number of bucket keys
};

// narrow_top: the wider windows of a range go at its bottom and the narrower at its top.  A
// window's doubling chain in k_msm_tail is as long as its position, so the top windows' chains
// are the longest; a narrower top window has fewer buckets, a shorter butterfly before that
// chain, and its chunk butterflies fit one pass of lane quads (65,536: 12-bit windows, C = 128;
// tail 167 -> 154 us).  Batches whose tails run on quads throughout (<= 16,384) keep the evenly
// spread widths (1,024: 118 us against 123 us narrow-top).
NWV_HD void msm_split(MsmLayout& L, int first, int count, int total_bits, bool narrow_top = false) {
    const int q = total_bits / count, r = total_bits % count;
    for (int k = 0; k < count; k++) {
        const int lo = total_bits * k / count, hi = total_bits * (k + 1) / count;
        L.width[first + k] = (uint8_t)(narrow_top ? (k < r ? q + 1 : q) : hi - lo);
    }
}

// base width c (6..16) -> layout; false if it does not fit MSM_MAX_WINDOWS
// c_lo bounds the widths of the z range (every point has digits there), c_hi those above it
// (only the A points and B: far fewer entries when a keyed batch has few distinct keys)
NWV_HD bool msm_make_layout2(int c_lo, int c_hi, MsmLayout& L, bool narrow_top = false) {
    const int lo_bits = MSM_BITS_Z + 1, hi_bits = MSM_BITS_FULL + 1 - lo_bits;
    const int nz = (lo_bits + c_lo - 1) / c_lo, nh = (hi_bits + c_hi - 1) / c_hi;
    if (nz + nh > MSM_MAX_WINDOWS) return false;
    L.nw = nz + nh;
    L.nw_z = nz;
    msm_split(L, 0, nz, lo_bits, narrow_top);
    msm_split(L, nz, nh, hi_bits, narrow_top);
    int pos = 0, cm = 0;
    uint32_t kb = 0;
    for (int w = 0; w < L.nw; w++) {
        L.pos[w] = (uint16_t)pos;
        L.kbase[w] = kb;
        pos += L.width[w];
        kb += 1u << (L.width[w] - 1);
        cm = L.width[w] > cm ? L.width[w] : cm;
    }
    L.kbase[L.nw] = kb;
    L.cmax = cm;
    L.pad = 0;
    return true;
}
NWV_HD bool msm_make_layout(int c, MsmLayout& L, bool narrow_top = false) {
    return msm_make_layout2(c, c, L, narrow_top);
}
// z range only (nw == nw_z): every scalar < 2^128, as in a keyed batch over the key cache
// (split scalars, msm_split128)
NWV_HD bool msm_make_layout_z(int c, MsmLayout& L) {
    const int nz = (MSM_BITS_Z + 1 + c - 1) / c;
    if (nz > MSM_MAX_WINDOWS) return false;
    L.nw = nz;
    L.nw_z = nz;
    msm_split(L, 0, nz, MSM_BITS_Z + 1);
    int pos = 0, cm = 0;
    uint32_t kb = 0;
    for (int w = 0; w < L.nw; w++) {
        L.pos[w] = (uint16_t)pos;
        L.kbase[w] = kb;
        pos += L.width[w];
        kb += 1u << (L.width[w] - 1);
        cm = L.width[w] > cm ? L.width[w] : cm;
    }
    L.kbase[L.nw] = kb;
    L.cmax = cm;
    L.pad = 0;
    return true;
}
// s = lo + 2^128 hi (both < 2^128)
NWV_HD void msm_split128(const uint32_t s[8], uint32_t lo[8], uint32_t hi[8]) {
    for (int k = 0; k < 8; k++) {
        lo[k] = k < 4 ? s[k] : 0u;
        hi[k] = k < 4 ? s[k + 4] : 0u;
    }
}

// Fixed-base comb for the basepoint term.  B's scalar b = -sum z_i s_i is known only after every
// signature is hashed, and as an MSM point B would put a full-width scalar (and a sort / bucket
// dependency on b) into every window.  Instead [8 b]B = sum_j [d_j 16^j] B over the 64 signed
// radix-16 digits d_j in [-8, 8] of c = 8 b mod l, from a per-device table of i 16^j B
// (i = 1..8, affine Niels records), is summed by the last hash workgroup of k_msm_prep while
// the other blocks still decompress, and joins the MSM tail's final sum.  (B has prime order l,
// so [8]([b]B) = [8 b mod l]B.)
static constexpr int COMB_TABLES = 64, COMB_ENTRIES = 8;

// i 16^j P (1 <= i <= 8) as an MSM point record (affine Niels)
NWV_HD void comb_entry_of(const ge_p3& P, int j, int i, uint32_t* e) {
    ge_p3 Q = j ? p3_dbl_n(P, 4 * j) : P;
    const ge_cached cq = ge_p3_to_cached(Q);
    ge_p3 acc = ge_p3_identity();
    for (int bit = 3; bit >= 0; bit--) {
        acc = ge_p3_dbl(acc);
        if ((i >> bit) & 1) acc = ge_p1p1_to_p3(ge_add(acc, cq));
    }
    const ge_precomp q = ge_p3_to_precomp(acc);
    store_fe(e, q.ypx);
    store_fe(e + 10, q.ymx);
    store_fe(e + 20, q.xy2d);
    e[30] = e[31] = 0u;
}
// i 16^j B
NWV_HD void comb_entry(int j, int i, uint32_t* e) {
    uint32_t bw[8];
    ge_basepoint_words(bw);
    ge_p3 B;
    ge_decompress(bw, B);
    comb_entry_of(B, j, i, e);
}

// signed radix-16 digits of c < 2^253: c = sum_{j < 64} d_j 16^j, d_j in [-8, 8)  (d_63 <= 2)
NWV_HD void comb_digits(const uint32_t c[8], int d[COMB_TABLES]) {
    int carry = 0;
    for (int j = 0; j < COMB_TABLES; j++) {
        int v = (int)((c[j >> 3] >> (4 * (j & 7))) & 15u) + carry;
        carry = 0;
        if (j + 1 < COMB_TABLES && v >= 8) {
            v -= 16;
            carry = 1;
        }
        d[j] = v;
    }
}

// Committee key cache slot: A's point record, then 2^128 A's (msm_store_point layout); word
// MSM_PT_WORDS - 1 of the first record is 1 when A failed to decode.  Slot 0 holds B.
static constexpr int KC_SLOT_WORDS = 64;

// chunks of chunk_pts points in window w (all na + 1 + n points below nw_z, else na + 1)
NWV_HD uint32_t msm_window_chunks(uint64_t n, uint64_t na, int w, int nw_z, uint32_t chunk_pts) {
    const uint64_t cnt = w < nw_z ? na + 1 + n : na + 1;
    return (uint32_t)((cnt + chunk_pts - 1) / chunk_pts);
}

// k_msm_scatter's XCD grouping.  Workgroups b and b + 8 share an XCD (MI355X_MICROARCH.md,
// "Workgroup dispatch"), so group g = blockIdx.x % 8 runs every chunk of the windows win[g][..]:
// all (bucket, chunk) slices of one window are then written through ONE XCD's L2, which
// assembles whole lines, instead of up to eight partial write-backs of each line.
static constexpr int MSM_XCD_GROUPS = 8, MSM_XCD_WIN = 8;
struct MsmXcdMap {
    uint32_t slots;  // workgroups per group: grid = MSM_XCD_GROUPS x slots
    uint8_t nwin[MSM_XCD_GROUPS];
    uint8_t win[MSM_XCD_GROUPS][MSM_XCD_WIN];
};

// windows -> groups, largest first onto the least-loaded group (load = chunks)
NWV_HD void msm_xcd_map(const MsmLayout& L, uint64_t n, uint64_t na, uint32_t chunk_pts, MsmXcdMap& m) {
    uint32_t load[MSM_XCD_GROUPS];
    bool done[MSM_MAX_WINDOWS];
    for (int g = 0; g < MSM_XCD_GROUPS; g++) load[g] = 0, m.nwin[g] = 0;
    for (int w = 0; w < L.nw; w++) done[w] = false;
    m.slots = 0;
    for (int it = 0; it < L.nw; it++) {
        int wb = -1;
        uint32_t cb = 0;
        for (int w = 0; w < L.nw; w++) {
            const uint32_t c = msm_window_chunks(n, na, w, L.nw_z, chunk_pts);
            if (!done[w] && (wb < 0 || c > cb)) wb = w, cb = c;
        }
        int gb = -1;  // MSM_MAX_WINDOWS <= MSM_XCD_GROUPS * MSM_XCD_WIN: some group has room
        for (int g = 0; g < MSM_XCD_GROUPS; g++)
            if (m.nwin[g] < MSM_XCD_WIN && (gb < 0 || load[g] < load[gb])) gb = g;
        done[wb] = true;
        m.win[gb][m.nwin[gb]++] = (uint8_t)wb;
        load[gb] += cb;
        m.slots = load[gb] > m.slots ? load[gb] : m.slots;
    }
}
static_assert(MSM_MAX_WINDOWS <= MSM_XCD_GROUPS * MSM_XCD_WIN, "every window needs a group slot");

// raw bits [pos, pos + width) of a 256-bit little-endian scalar (width <= 16)
NWV_HD uint32_t msm_window_bits(const uint32_t s[8], int pos, int width) {
    uint64_t v = 0;
    const int word = pos >> 5, sh = pos & 31;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (k == word) v |= (uint64_t)s[k];
        if (k == word + 1) v |= (uint64_t)s[k] << 32;
    }
    return (uint32_t)(v >> sh) & ((1u << width) - 1u);
}

// Signed recoding of a scalar over windows [0, nw) of layout L (nw = L.nw for scalars mod l,
// L.nw_z for z); emit(w, d) for every window.
template <class Emit>
NWV_HD void msm_recode(const uint32_t s[8], const MsmLayout& L, int nw, Emit emit) {
    uint32_t carry = 0;
#pragma unroll 1
    for (int w = 0; w < nw; w++) {
        const int c = L.width[w];
        int d = (int)(msm_window_bits(s, L.pos[w], c) + carry);
        carry = 0;
        if (w + 1 < nw && d >= (1 << (c - 1))) {
            d -= 1 << c;
            carry = 1;
        }
        emit(w, d);
    }
}

// Bucket entry encoding: point index | sign bit
static constexpr uint32_t MSM_NEG = 0x80000000u;

// Two-level counting sort of large batches.  A one-level scatter of a window with 2^14 buckets
// and 64 chunks writes runs of ~4 entries per (bucket, chunk) slice: every line of the entry
// array is written piecemeal by many workgroups, and once a window's entries (16 MB at 2M
// signatures) exceed an XCD's 4 MB L2 the pieces are written back separately.  The first level
// sorts by the top bits of the bucket (bin (|d| - 1) >> shift: runs of ~64 entries per slice),
// packing the low bits into the entry; the second (k_msm_lsort) orders each coarse bin by its low
// bits inside one workgroup.  Packed entry: sign (bit 31) | low bits (shift of them, below bit 31)
// | point index (31 - shift bits).
static constexpr int MSM_SORT2_MAX_SHIFT = 8;
NWV_HD uint32_t msm_pack2(uint32_t j, uint32_t b, bool neg, int shift) {
    return j | ((b & ((1u << shift) - 1u)) << (31 - shift)) | (neg ? MSM_NEG : 0u);
}
NWV_HD uint32_t msm_unpack2_low(uint32_t e, int shift) { return (e >> (31 - shift)) & ((1u << shift) - 1u); }
NWV_HD uint32_t msm_unpack2_entry(uint32_t e, int shift) {
    return (e & ((1u << (31 - shift)) - 1u)) | (e & MSM_NEG);
}

// MSM point record: affine Niels (y+x | y-x | 2dxy) of a decompressed point (Z = 1, T = xy),
// padded to 32 words = 128 bytes so a bucket lane's random gather touches one cache line; a
// negative digit swaps y+x / y-x and negates 2dxy on the fly.
static constexpr int MSM_PT_WORDS = 32;
// words of one point's comb table (COMB_TABLES x COMB_ENTRIES records: i 16^j P)
static constexpr int COMB_WORDS = MSM_PT_WORDS * COMB_TABLES * COMB_ENTRIES;

NWV_HD void msm_store_point(uint32_t* e, const ge_p3& p) {
    store_fe(e, fe_carry(fe_add(p.Y, p.X)));
    store_fe(e + 10, fe_carry(fe_sub(p.Y, p.X)));
    store_fe(e + 20, fe_mul(p.T, fe_d2()));
    e[30] = 0u;
    e[31] = 0u;
}
// record from a basepoint-table precomp entry (y+x | y-x | 2dxy | -2dxy)
NWV_HD void msm_point_from_precomp(uint32_t* e, const uint32_t* pre) {
    for (int k = 0; k < 30; k++) e[k] = pre[k];
    e[30] = 0u;
    e[31] = 0u;
}
NWV_HD ge_precomp msm_point_select(const fe& ypx, const fe& ymx, const fe& xy2d, bool neg) {
    const fe nxy = fe_neg(xy2d);  // 2p - 2dxy: limbs < 2^27, a valid multiply input
    return ge_precomp{fe_select(ypx, ymx, neg), fe_select(ymx, ypx, neg), fe_select(xy2d, nxy, neg)};
}
NWV_HD ge_precomp msm_load_point(const uint32_t* e, bool neg) {
    return msm_point_select(load_fe(e), load_fe(e + 10), load_fe(e + 20), neg);
}

// Weighted bucket sums.  For one window with buckets S_1..S_NB (bucket b has weight b), a lane
// g owns the L consecutive buckets b = gL+1 .. gL+L and returns, scanning down,
//     run = sum S_b           acc = sum (b - gL) S_b
// so that  sum_b b S_b = sum_g acc_g + L * sum_{g >= 1} suffix_g,  suffix_g = sum_{g' >= g} run_g'.
template <class LoadBucket>
NWV_HD void msm_segment_sums(int L, LoadBucket load_bucket, ge_p3& run, ge_p3& acc) {
    run = ge_p3_identity();
    acc = ge_p3_identity();
#pragma unroll 1
    for (int k = L - 1; k >= 0; k--) {
        run = p3_add(run, load_bucket(k));
        acc = p3_add(acc, run);
    }
}

}  // namespace nwv
