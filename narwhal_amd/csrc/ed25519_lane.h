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
// [s]B + [k](-A) is one Straus pass with shared doublings: k in signed radix 16 (64 digits,
// per-lane table 0..8 A in global scratch), s in signed radix 256 (32 digits, 129-entry
// affine-Niels basepoint table shared by all lanes).  Control flow is uniform across the
// wave: every digit (zero digits included, via an identity entry) costs one addition.
#pragma once
#include "ge25519.h"
#include "sc25519.h"
#include "sha512.h"

namespace nwv {

// per-lane scratch: entries 0..8 = j*A (entry 0 = identity), entry 9 = R; 2 KiB per lane
static constexpr int A_TABLE_ENTRIES = 9;
static constexpr int LANE_SCRATCH_WORDS = 512;
static constexpr int R_ENTRY = 9;
// basepoint table: entries 0..128 = j*B (entry 0 = identity)
static constexpr int BASE_TABLE_ENTRIES = 129;
static constexpr int BASE_TABLE_WORDS = BASE_TABLE_ENTRIES * PRECOMP_ENTRY_WORDS;

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

// ---- the three phases of one verification (separate kernels on the GPU) ----
static constexpr uint32_t FLAG_S_OK = 1u, FLAG_R_OK = 2u, FLAG_A_OK = 4u;
static constexpr uint32_t FLAGS_ALL = 7u;

// phase 1: challenge scalar and s < l
NWV_HD uint32_t lane_hash(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                          const uint8_t* msg, uint32_t mlen, uint32_t k[8]) {
    challenge_scalar(Rw, Aw, msg, mlen, k);
    return sc_is_canonical(Sw) ? FLAG_S_OK : 0u;
}
// phase 2: decompress R (entry R_ENTRY) and A (entries 0..8 = j A); on the GPU the two halves
// run in two lanes
NWV_HD uint32_t lane_point_R(const uint32_t Rw[8], uint32_t* tbl) {
    ge_p3 R;
    const uint32_t f = ge_decompress(Rw, R) ? FLAG_R_OK : 0u;
    store_cached_entry(tbl + R_ENTRY * CACHED_ENTRY_WORDS, ge_p3_to_cached(R));
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
// phase 3: [8]([s]B - [k]A - R) == identity
NWV_HD bool lane_straus_check(const uint32_t k[8], const uint32_t Sw[8], const uint32_t* tbl,
                              const uint32_t* btab) {
    ge_p3 Rp = straus_sB_minus_kA(k, Sw, tbl, btab, tbl);
    ge_p1p1 t = ge_add_entry(Rp, tbl + R_ENTRY * CACHED_ENTRY_WORDS, true);
    ge_p2 q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    return ge_p1p1_is_identity(t);
}

// Full single verification.  tbl: lane scratch (LANE_SCRATCH_WORDS words).
NWV_HD bool ed25519_verify_lane(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                                const uint8_t* msg, uint32_t mlen, uint32_t* tbl,
                                const uint32_t* btab) {
    bool ok = sc_is_canonical(Sw);
    uint32_t k[8];
    challenge_scalar(Rw, Aw, msg, mlen, k);
    {
        ge_p3 R;
        ok &= ge_decompress(Rw, R);
        store_cached_entry(tbl + R_ENTRY * CACHED_ENTRY_WORDS, ge_p3_to_cached(R));
    }
    {
        ge_p3 A;
        ok &= ge_decompress(Aw, A);
        build_a_table(A, tbl);
    }
    ge_p3 Rp = straus_sB_minus_kA(k, Sw, tbl, btab, tbl);
    // [8](R' - R)
    ge_p1p1 t = ge_add_entry(Rp, tbl + R_ENTRY * CACHED_ENTRY_WORDS, true);
    ge_p2 q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    q = ge_p1p1_to_p2(t);
    t = ge_p2_dbl(q);
    return ok && ge_p1p1_is_identity(t);
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

}  // namespace nwv
