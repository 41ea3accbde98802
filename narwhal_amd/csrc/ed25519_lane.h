// ed25519_lane.h -- one ZIP-215 Ed25519 verification per lane (kernel K4 body).
//
// Restates ed25519_consensus 2.0.1 VerificationKey::verify:
//   1. A = decompress(pk) else reject          (VerificationKey::try_from)
//   2. s < l else reject                       (Scalar::from_canonical_bytes)
//   3. R = decompress(sig[0..32]) else reject
//   4. k = SHA-512(R_bytes || A_bytes || M) mod l over the RAW received bytes
//   5. accept iff [8](R' - R) == identity, R' = [s]B - [k]A  (cofactored check)
// Callers on the reference side: Header::verify types/src/primary.rs:179-182,
// Vote::verify :325-327, and the per-signature fallback of batch verification.
//
// The check runs on half-size scalars: a truncated extended Euclid on (l, k) gives u = v k
// (mod l) with 0 <= u < 2^127, 0 < |v| < 2^126, and [8]([v s]B - [v]R - [u]A) == identity holds
// iff [8]([s]B - R - [k]A) does (v is invertible mod l, and [8] maps every point into the
// prime-order subgroup, where [v k] and [u] act alike).  [v s mod l]B + [-v]R + [-u]A is one
// Straus pass over 132 bits: v and u in signed radix 16 (33 digits each, per-lane tables 0..8 R
// and 0..8 A in global scratch), v s = w_lo + 2^128 w_hi in signed radix 256 (17 digits each,
// the 129-entry affine-Niels tables of j B and j 2^128 B shared by all lanes): 132 doublings
// instead of 252.  Control flow is uniform across the wave apart from the Euclid's iteration
// count: every digit (zero digits included, via an identity entry) costs one addition.
#pragma once
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"

namespace nwv {

// per-lane scratch: entries 0..8 = j*A (entry 0 = identity), entries 9..17 = j*R; 3.5 KiB per lane
static constexpr int A_TABLE_ENTRIES = 9;
static constexpr int R_ENTRY = 9;
static constexpr int LANE_SCRATCH_WORDS = 2 * A_TABLE_ENTRIES * CACHED_ENTRY_WORDS;
// basepoint tables (one buffer): entries 0..128 = j*B (entry 0 = identity), one cached identity
// entry, then entries 0..128 = j*2^128*B
static constexpr int BASE_TABLE_ENTRIES = 129;
static constexpr int BASE_TABLE_WORDS = BASE_TABLE_ENTRIES * PRECOMP_ENTRY_WORDS;
static constexpr int BASE128_TABLE_OFFSET = BASE_TABLE_WORDS + CACHED_ENTRY_WORDS;
static constexpr int BTAB_WORDS = BASE128_TABLE_OFFSET + BASE_TABLE_WORDS;

// signed digit from the top window of y (256-bit, little-endian words), then shift y left
NWV_HD int take_top_digit(uint32_t y[8], int w) {
    const int d = (int)(y[7] >> (32 - w)) - (1 << (w - 1));
#pragma unroll
    for (int i = 7; i > 0; i--) y[i] = (y[i] << w) | (y[i - 1] >> (32 - w));
    y[0] <<= w;
    return d;
}

// k = SHA-512(R || A || M) mod l
NWV_HD void challenge_scalar(const uint32_t Rw[8], const uint32_t Aw[8], const uint8_t* msg,
                             uint32_t mlen, uint32_t k[8]) {
    uint32_t pre[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        pre[i] = Rw[i];
        pre[8 + i] = Aw[i];
    }
    sha512_state st;
    sha512_prefixed_msg(st, pre, msg, mlen);
    uint32_t hw[16];
    sha512_digest_words(st, hw);
    sc_reduce512(hw, k);
}

// entries 0..8 = identity, A, 2A, ..., 8A (cached form with -2dT)
NWV_HD void build_a_table(const ge_p3& A, uint32_t* tbl) {
    store_cached_entry(tbl, ge_cached_identity());
    const ge_cached c1 = ge_p3_to_cached(A);
    store_cached_entry(tbl + CACHED_ENTRY_WORDS, c1);
    ge_p3 cur = A;
#pragma unroll 1
    for (int j = 2; j < A_TABLE_ENTRIES; j++) {
        cur = ge_p1p1_to_p3(ge_add_entry(cur, tbl + CACHED_ENTRY_WORDS, false));
        store_cached_entry(tbl + j * CACHED_ENTRY_WORDS, ge_p3_to_cached(cur));
    }
}

// four doublings r <- 16 r, the last one left in completed form
NWV_HD ge_p1p1 dbl4(ge_p2 r) {
    ge_p1p1 t = ge_p2_dbl(r);
    r = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(r);
    r = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(r);
    r = ge_p1p1_to_p2(t);
    return ge_p2_dbl(r);
}

// R' = [s]B + [k](-A); tbl = lane's 0..8 A table, btab = 0..128 B table (nullptr tbl is
// allowed when k == 0: every A digit is then 0 and the identity entry is used)
NWV_HD ge_p3 straus_sB_minus_kA(const uint32_t k[8], const uint32_t s[8], const uint32_t* tbl,
                                const uint32_t* btab, const uint32_t* ident_cached) {
    uint32_t ky[8], sy[8];
    sc_recode_offset(k, ky, 0x88888888u);
    sc_recode_offset(s, sy, 0x80808080u);
    ge_p2 r = ge_p2_identity();
    ge_p1p1 t;
#pragma unroll 1
    for (int i = 63; i >= 0; i--) {
        ge_p3 p = (i == 63) ? ge_p3_identity() : ge_p1p1_to_p3(dbl4(r));
        // coefficient of A is -k: digit -kd
        const int ad = -take_top_digit(ky, 4);
        const int am = ad < 0 ? -ad : ad;
        const uint32_t* ea = (am == 0 || tbl == nullptr) ? ident_cached : tbl + am * CACHED_ENTRY_WORDS;
        t = ge_add_entry(p, ea, ad < 0);
        if ((i & 1) == 0) {
            const int sd = take_top_digit(sy, 8);
            const int sm = sd < 0 ? -sd : sd;
            p = ge_p1p1_to_p3(t);
            t = ge_madd_entry(p, btab + sm * PRECOMP_ENTRY_WORDS, sd < 0);
        }
        if (i != 0) r = ge_p1p1_to_p2(t);
    }
    return ge_p1p1_to_p3(t);
}

// ---- half-size scalars ---------------------------------------------------------------------
NWV_HD int bitlen8(const uint32_t x[8]) {
    int b = 0;
#pragma unroll
    for (int i = 7; i >= 0; i--)
        if (b == 0 && x[i] != 0) b = 32 * i + 32 - __builtin_clz(x[i]);
    return b;
}

// Truncated extended Euclid on (l, k), k < l: remainders r_0 = l, r_1 = k, ...; r_i = t_i k (mod l)
// with t_0 = 0, t_1 = 1 and t_i alternating in sign (t_i > 0 for odd i), so the magnitudes follow
// a_{i+1} = a_{i-1} + q_i a_i.  Stops at the first r_i < 2^127; then |t_i| <= l / r_{i-1} < 2^126.
// Each quotient step is a binary long division (q_i r_1 and q_i a_1 subtracted / added bit by
// bit: no variable shifts, no register-array indexing).  Out: u = r_i, m = |t_i|, vneg = t_i < 0.
NWV_HD void sc_half_split(const uint32_t k[8], uint32_t u[4], uint32_t m[4], bool& vneg) {
    uint32_t r0[8], r1[8], a0[5], a1[5];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r0[i] = sc_l(i);
        r1[i] = k[i];
    }
#pragma unroll
    for (int i = 0; i < 5; i++) {
        a0[i] = 0;
        a1[i] = i == 0 ? 1u : 0u;
    }
    bool odd = true;
#pragma unroll 1
    while (bitlen8(r1) > 127) {
        const int sh = bitlen8(r0) - bitlen8(r1);  // >= 0: r0 > r1
        uint32_t T[8], A[5];
#pragma unroll
        for (int i = 0; i < 8; i++) T[i] = r1[i];
#pragma unroll
        for (int i = 0; i < 5; i++) A[i] = a1[i];
#pragma unroll 1
        for (int j = 0; j < sh; j++) {  // T = r1 << sh, A = a1 << sh
#pragma unroll
            for (int i = 7; i > 0; i--) T[i] = (T[i] << 1) | (T[i - 1] >> 31);
            T[0] <<= 1;
#pragma unroll
            for (int i = 4; i > 0; i--) A[i] = (A[i] << 1) | (A[i - 1] >> 31);
            A[0] <<= 1;
        }
#pragma unroll 1
        for (int j = sh; j >= 0; j--) {
            uint32_t d[8];
            uint64_t br = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint64_t t = (uint64_t)r0[i] - T[i] - br;
                d[i] = (uint32_t)t;
                br = (t >> 32) & 1u;
            }
            const bool take = br == 0;  // r0 >= T
            uint64_t c = 0;
#pragma unroll
            for (int i = 0; i < 5; i++) {
                const uint64_t t = (uint64_t)a0[i] + A[i] + c;
                a0[i] = take ? (uint32_t)t : a0[i];
                c = t >> 32;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) r0[i] = take ? d[i] : r0[i];
#pragma unroll
            for (int i = 0; i < 7; i++) T[i] = (T[i] >> 1) | (T[i + 1] << 31);
            T[7] >>= 1;
#pragma unroll
            for (int i = 0; i < 4; i++) A[i] = (A[i] >> 1) | (A[i + 1] << 31);
            A[4] >>= 1;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t t = r0[i];
            r0[i] = r1[i];
            r1[i] = t;
        }
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const uint32_t t = a0[i];
            a0[i] = a1[i];
            a1[i] = t;
        }
        odd = !odd;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        u[i] = r1[i];
        m[i] = a1[i];
    }
    vneg = !odd;
}

// signed digits of a value below 2^128 (four words) from the top: y = x + offset (digits of
// 2^(w-1) over 132 / 136 bits), left-aligned in five words; each call returns the top window
// minus 2^(w-1) and shifts y left by w
NWV_HD void recode128(const uint32_t x[4], uint32_t y[5], int w) {
    const uint32_t pat = w == 4 ? 0x88888888u : 0x80808080u;
    const int bits = w == 4 ? 132 : 136;  // 33 radix-16 or 17 radix-256 digits
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint64_t t = (uint64_t)x[i] + pat + c;
        y[i] = (uint32_t)t;
        c = t >> 32;
    }
    y[4] = (uint32_t)c + (w == 4 ? 0x8u : 0x80u);
    const int sh = 160 - bits;  // 28 or 24
#pragma unroll
    for (int i = 4; i > 0; i--) y[i] = (y[i] << sh) | (y[i - 1] >> (32 - sh));
    y[0] <<= sh;
}
NWV_HD int take_top5(uint32_t y[5], int w) {
    const int d = (int)(y[4] >> (32 - w)) - (1 << (w - 1));
#pragma unroll
    for (int i = 4; i > 0; i--) y[i] = (y[i] << w) | (y[i - 1] >> (32 - w));
    y[0] <<= w;
    return d;
}

// [8]([w]B - [m]R + [cu]A) == identity, w = m s mod l, m = |v|, c = -1 (v > 0) or +1 (v < 0):
// the cofactored check [8]([s]B - R - [k]A) == identity on half-size scalars (header comment).
// tbl: entries 0..8 = j A, R_ENTRY + j = j R; btab: BTAB_WORDS (j B, identity, j 2^128 B).
template <bool PF = false>
NWV_HD bool lane_straus_check_half(const uint32_t k[8], const uint32_t Sw[8], const uint32_t* tbl,
                                   const uint32_t* btab) {
    uint32_t yu[5], ym[5], ylo[5], yhi[5];
    bool vneg;
    {
        uint32_t u[4], m[4];
        sc_half_split(k, u, m, vneg);
        uint32_t m8[8] = {m[0], m[1], m[2], m[3], 0, 0, 0, 0}, wv[8];
        sc_mul(m8, Sw, wv);
        recode128(u, yu, 4);
        recode128(m, ym, 4);
        recode128(wv, ylo, 8);
        recode128(wv + 4, yhi, 8);
    }
    const uint32_t* rt = tbl + R_ENTRY * CACHED_ENTRY_WORDS;
    const uint32_t* bt128 = btab + BASE128_TABLE_OFFSET;
    ge_p2 r = ge_p2_identity();
    ge_p1p1 t;
    // the lane's A and R table entries of a window are loaded one window ahead: the loads of
    // window i - 1 are issued once window i's have been consumed, so they complete behind the B
    // additions and the next four doublings instead of stalling the addition that needs them
    // (two 40-word entries in registers)
    // (PF; without it each addition reads its entry when it needs it)
    uint32_t ea[PF ? 40 : 1], er[PF ? 40 : 1];
    int ad = 0, rd = 0;
    if (PF) {
        ad = vneg ? take_top5(yu, 4) : -take_top5(yu, 4);
        rd = -take_top5(ym, 4);
        load_cached_entry(tbl + (ad < 0 ? -ad : ad) * CACHED_ENTRY_WORDS, ad < 0, ea);
        load_cached_entry(rt + (rd < 0 ? -rd : rd) * CACHED_ENTRY_WORDS, rd < 0, er);
    }
#pragma unroll 1
    for (int i = 32; i >= 0; i--) {
        ge_p3 p = (i == 32) ? ge_p3_identity() : ge_p1p1_to_p3(dbl4(r));
        if (PF) {
            t = ge_add_loaded(p, ea);
            p = ge_p1p1_to_p3(t);
            t = ge_add_loaded(p, er);
            if (i > 0) {
                ad = vneg ? take_top5(yu, 4) : -take_top5(yu, 4);
                rd = -take_top5(ym, 4);
                load_cached_entry(tbl + (ad < 0 ? -ad : ad) * CACHED_ENTRY_WORDS, ad < 0, ea);
                load_cached_entry(rt + (rd < 0 ? -rd : rd) * CACHED_ENTRY_WORDS, rd < 0, er);
            }
        } else {
            const int du = take_top5(yu, 4);
            ad = vneg ? du : -du;  // A's coefficient: -u (v > 0) or +u (v < 0)
            t = ge_add_entry(p, tbl + (ad < 0 ? -ad : ad) * CACHED_ENTRY_WORDS, ad < 0);
            rd = -take_top5(ym, 4);  // R's coefficient: -m
            p = ge_p1p1_to_p3(t);
            t = ge_add_entry(p, rt + (rd < 0 ? -rd : rd) * CACHED_ENTRY_WORDS, rd < 0);
        }
        if ((i & 1) == 0) {
            const int dl = take_top5(ylo, 8), dh = take_top5(yhi, 8);
            p = ge_p1p1_to_p3(t);
            t = ge_madd_entry(p, btab + (dl < 0 ? -dl : dl) * PRECOMP_ENTRY_WORDS, dl < 0);
            p = ge_p1p1_to_p3(t);
            t = ge_madd_entry(p, bt128 + (dh < 0 ? -dh : dh) * PRECOMP_ENTRY_WORDS, dh < 0);
        }
        r = ge_p1p1_to_p2(t);
    }
    t = ge_p2_dbl(r);
    ge_p2 q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    return ge_p1p1_is_identity(t);
}

// ---- the three phases of one verification (separate kernels on the GPU) ----
static constexpr uint32_t FLAG_S_OK = 1u, FLAG_R_OK = 2u, FLAG_A_OK = 4u;
static constexpr uint32_t FLAGS_ALL = 7u;

// phase 1: challenge scalar and s < l
NWV_HD uint32_t lane_hash(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                          const uint8_t* msg, uint32_t mlen, uint32_t k[8]) {
    challenge_scalar(Rw, Aw, msg, mlen, k);
    return sc_is_canonical(Sw) ? FLAG_S_OK : 0u;
}
// phase 2: decompress R (entries R_ENTRY + j = j R) and A (entries 0..8 = j A); on the GPU the
// two halves run in two lanes
NWV_HD uint32_t lane_point_R(const uint32_t Rw[8], uint32_t* tbl) {
    ge_p3 R;
    const uint32_t f = ge_decompress(Rw, R) ? FLAG_R_OK : 0u;
    build_a_table(R, tbl + R_ENTRY * CACHED_ENTRY_WORDS);
    return f;
}
NWV_HD uint32_t lane_point_A(const uint32_t Aw[8], uint32_t* tbl) {
    ge_p3 A;
    const uint32_t f = ge_decompress(Aw, A) ? FLAG_A_OK : 0u;
    build_a_table(A, tbl);
    return f;
}
NWV_HD uint32_t lane_points(const uint32_t Aw[8], const uint32_t Rw[8], uint32_t* tbl) {
    return lane_point_R(Rw, tbl) | lane_point_A(Aw, tbl);
}
// phase 3: [8]([s]B - [k]A - R) == identity, on half-size scalars
template <bool PF = false>
NWV_HD bool lane_straus_check(const uint32_t k[8], const uint32_t Sw[8], const uint32_t* tbl,
                              const uint32_t* btab) {
    return lane_straus_check_half<PF>(k, Sw, tbl, btab);
}

// Full single verification.  tbl: lane scratch (LANE_SCRATCH_WORDS words).
NWV_HD bool ed25519_verify_lane(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                                const uint8_t* msg, uint32_t mlen, uint32_t* tbl,
                                const uint32_t* btab) {
    uint32_t k[8];
    const uint32_t f = lane_hash(Aw, Rw, Sw, msg, mlen, k) | lane_points(Aw, Rw, tbl);
    return lane_straus_check(k, Sw, tbl, btab) && f == FLAGS_ALL;
}

// m B for m <= 128 in affine Niels form (basepoint table entry)
NWV_HD ge_precomp base_multiple(int m) {
    uint32_t bw[8];
    ge_basepoint_words(bw);
    ge_p3 B;
    ge_decompress(bw, B);
    const ge_cached cb = ge_p3_to_cached(B);
    ge_p3 acc = ge_p3_identity();
    for (int bit = 7; bit >= 0; bit--) {
        acc = ge_p3_dbl(acc);
        if ((m >> bit) & 1) acc = ge_p1p1_to_p3(ge_add(acc, cb));
    }
    return ge_p3_to_precomp(acc);
}
// m 2^128 B for m <= 128 (the second basepoint table)
NWV_HD ge_precomp base128_multiple(int m) {
    uint32_t bw[8];
    ge_basepoint_words(bw);
    ge_p3 B;
    ge_decompress(bw, B);
    ge_p3 Q = B;
    for (int i = 0; i < 128; i++) Q = ge_p3_dbl(Q);
    const ge_cached cq = ge_p3_to_cached(Q);
    ge_p3 acc = ge_p3_identity();
    for (int bit = 7; bit >= 0; bit--) {
        acc = ge_p3_dbl(acc);
        if ((m >> bit) & 1) acc = ge_p1p1_to_p3(ge_add(acc, cq));
    }
    return ge_p3_to_precomp(acc);
}

}  // namespace nwv
