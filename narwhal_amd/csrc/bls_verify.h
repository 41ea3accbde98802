// bls_verify.h -- the per-item steps of BLS12-381 min_sig verification,
// shared by the gfx950 kernels (bls_kernels.hip) and the CPU test build (tests/hostemu).
//
// An item is fastcrypto's AggregateAuthenticator::verify (types/src/primary.rs:531-534) =
// blst fast_aggregate_verify(sig, pks, msg): the aggregate signature decodes and lies in G1, the
// public keys (decoded and validated once, as fastcrypto does at deserialisation) are summed,
// the sum is not the identity, and e(-sig, g2) e(H(msg), apk) = 1.  Verifier::verify
// (Header::verify :179-182, Vote::verify :325-327) is the one-key case.  Status codes are the
// oracle's (oracle/bls_oracle.h ORB_*), checked in its order.
#pragma once
#include "bls381.h"

namespace bls {

// device records (u32 words, Montgomery limbs)
constexpr int G1_REC_WORDS = 2 * NL + 1;   // x, y, flags (bit 0 = identity)
constexpr int G2_REC_WORDS = 4 * NL + 1;   // x.c0, x.c1, y.c0, y.c1, flags

NWV_HD void st_fp(uint32_t* o, const fp& a) { for (int j = 0; j < NL; j++) o[j] = a.l[j]; }
NWV_HD fp ld_fp(const uint32_t* o) { fp a; for (int j = 0; j < NL; j++) a.l[j] = o[j]; return a; }
NWV_HD void st_g1(uint32_t* o, const fp& x, const fp& y, bool inf) {
    st_fp(o, x);
    st_fp(o + NL, y);
    o[2 * NL] = inf ? 1u : 0u;
}
NWV_HD void st_g2(uint32_t* o, const fp2& x, const fp2& y, bool inf) {
    st_fp(o, x.c0);
    st_fp(o + NL, x.c1);
    st_fp(o + 2 * NL, y.c0);
    st_fp(o + 3 * NL, y.c1);
    o[4 * NL] = inf ? 1u : 0u;
}
NWV_HD void ld_g2(const uint32_t* o, fp2& x, fp2& y) {
    x.c0 = ld_fp(o);
    x.c1 = ld_fp(o + NL);
    y.c0 = ld_fp(o + 2 * NL);
    y.c1 = ld_fp(o + 3 * NL);
}

// a public key as fastcrypto deserialises and blst validates it: decodes, is not the identity,
// lies in G2
NWV_HD int32_t key_decode(const uint8_t* pk96, uint32_t* rec) {
    fp2 x, y;
    bool inf;
    int32_t st = g2_decompress(x, y, inf, pk96);
    if (st == ST_OK && inf) st = ST_PK_INFINITY;
    if (st == ST_OK && !g2_in_group(x, y)) st = ST_NOT_IN_GROUP;
    if (st != ST_OK) x = y = f2_zero();
    st_g2(rec, x, y, st != ST_OK);
    return st;
}
// a signature: decodes; unless it is the identity it lies in G1 (blst sig_groupcheck)
NWV_HD int32_t sig_decode(const uint8_t* sig48, uint32_t* rec) {
    fp x, y;
    bool inf;
    int32_t st = g1_decompress(x, y, inf, sig48);
    if (st == ST_OK && !inf && !g1_in_group(x, y)) st = ST_NOT_IN_GROUP;
    if (st != ST_OK || inf) x = y = fp_zero();
    st_g1(rec, x, y, inf);
    return st;
}
// H(msg) as an affine record
NWV_HD void h2c_record(const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl, uint32_t* rec) {
    const jac<fp> h = hash_to_g1(msg, n, dst, dl);
    fp x = fp_zero(), y = fp_zero();
    if (!h.inf) g1_to_affine(x, y, h);
    st_g1(rec, x, y, h.inf);
}
// apk = sum of the item's keys (records of validated keys), affine; status as the oracle orders it
NWV_HD int32_t apk_record(const uint32_t* key_recs, const int32_t* key_status, const uint32_t* idx, uint32_t cnt,
                          uint32_t* rec) {
    if (cnt == 0) {
        st_g2(rec, f2_zero(), f2_zero(), true);
        return ST_AGGR_MISMATCH;
    }
    jac<fp2> acc;
    acc.inf = true;
    acc.x = acc.y = acc.z = f2_zero();
    for (uint32_t i = 0; i < cnt; i++) {
        const uint32_t k = idx[i];
        if (key_status[k] != ST_OK) {
            st_g2(rec, f2_zero(), f2_zero(), true);
            return key_status[k];
        }
        fp2 x, y;
        ld_g2(key_recs + (size_t)k * G2_REC_WORDS, x, y);
        acc = jac_add(acc, jac_from_affine(x, y));
    }
    fp2 x = f2_zero(), y = f2_zero();
    if (!acc.inf) g2_to_affine(x, y, acc);
    st_g2(rec, x, y, acc.inf);
    return acc.inf ? ST_PK_INFINITY : ST_OK;
}
// e(-sig, g2) e(H, apk) == 1 (an identity signature contributes e(O, g2) = 1)
NWV_HD bool pairing_check(const uint32_t* sig_rec, const uint32_t* h_rec, const uint32_t* apk_rec) {
    fp px[2], py[2];
    fp2 qx[2], qy[2];
    int n = 0;
    if (!sig_rec[2 * NL]) {
        px[n] = ld_fp(sig_rec);
        py[n] = fp_neg(ld_fp(sig_rec + NL));
        qx[n] = k_g2x();
        qy[n] = k_g2y();
        n++;
    }
    if (!h_rec[2 * NL]) {
        px[n] = ld_fp(h_rec);
        py[n] = ld_fp(h_rec + NL);
        ld_g2(apk_rec, qx[n], qy[n]);
        n++;
    }
    return f12_is_one(final_exp(miller_loop2(n, px, py, qx, qy)));
}

}  // namespace bls
