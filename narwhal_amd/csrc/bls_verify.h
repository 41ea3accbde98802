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
#include "bls_group.h"
#include "bls_wave.h"

namespace bls {

// device records (u32 words, Montgomery limbs)
constexpr int G1_REC_WORDS = 2 * NL + 1;   // x, y, flags (bit 0 = identity)
constexpr int G2_REC_WORDS = 4 * NL + 1;   // x.c0, x.c1, y.c0, y.c1, flags

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

// ---- the batch check: a random linear combination over a call's items -----------------------
// Every item i that decoded and passed the group checks carries a 64-bit coefficient r_i (odd, so
// nonzero: blst's own multi-verification draws 64-bit coefficients too); the call accepts iff
//   prod_i e([r_i] H_i, apk_i) * e(-sum_i [r_i] sig_i, g2) == 1,
// computed in stages: every item's [r_i] H_i and [r_i] sig_i; the G1 sum S of the latter (a
// tree); the Miller loops of ([r_i] H_i, apk_i) and of (-S, g2), all in one grid; a product tree;
// ONE final exponentiation.  H_i, sig_i lie in G1 and apk_i in G2 (prime order r), so an invalid item makes
// the product differ from 1 except with probability ~2^-63 over the coefficients; when it is not
// 1 the engine runs the per-item check (pairing_check) to name the failing items exactly.
constexpr int F12_REC_WORDS = 12 * NL;     // Fp12, tower order c0.c0.c0 .. c1.c2.c1
constexpr int G1J_REC_WORDS = 3 * NL + 1;  // Jacobian X, Y, Z, flags (bit 0 = identity)

NWV_HD void st_f12(uint32_t* o, const fp12& e) {
    const fp* c[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                       &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
    for (int k = 0; k < 12; k++) st_fp(o + NL * k, *c[k]);
}
NWV_HD fp12 ld_f12(const uint32_t* o) {
    fp12 e;
    fp* c[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                 &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
    for (int k = 0; k < 12; k++) *c[k] = ld_fp(o + NL * k);
    return e;
}
NWV_HD void st_g1j(uint32_t* o, const jac<fp>& p) {
    st_fp(o, p.x);
    st_fp(o + NL, p.y);
    st_fp(o + 2 * NL, p.z);
    o[3 * NL] = p.inf ? 1u : 0u;
}
NWV_HD jac<fp> ld_g1j(const uint32_t* o) {
    jac<fp> p;
    p.x = ld_fp(o);
    p.y = ld_fp(o + NL);
    p.z = ld_fp(o + 2 * NL);
    p.inf = o[3 * NL] != 0;
    return p;
}

// r_i = the first 8 bytes of SHA-256(seed || i_be32), forced odd
NWV_HD uint64_t rlc_scalar(const uint8_t* seed32, uint32_t i) {
    uint32_t h[8], blk[16];
    sha256_iv(h);
    for (int k = 0; k < 8; k++)
        blk[k] = ((uint32_t)seed32[4 * k] << 24) | ((uint32_t)seed32[4 * k + 1] << 16) |
                 ((uint32_t)seed32[4 * k + 2] << 8) | (uint32_t)seed32[4 * k + 3];
    blk[8] = i;
    blk[9] = 0x80000000u;  // padding after the 36 message bytes
    for (int k = 10; k < 15; k++) blk[k] = 0;
    blk[15] = 36 * 8;
    sha256_block(h, blk);
    return (((uint64_t)h[0] << 32) | h[1]) | 1u;
}

// ---- the same checks over a group of lanes (bls_group.h): what the kernels run --------------
// e(-sig, g2) e(H, apk) == 1 (pairing_check), every lane of the group gets the verdict
G_HD bool g_pairing_check(const GCtx& g, const uint32_t* sig_rec, const uint32_t* h_rec, const uint32_t* apk_rec) {
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
    const G12 f = n == 2 ? g_miller<2>(g, px, py, qx, qy)
                : n == 1 ? g_miller<1>(g, px, py, qx, qy) : g_one(g);
    return g_is_one(g, g_final_exp(g, f));
}

// stage 1, item i (one group): P_i = [r] H (affine record, identity flag) and s_i = [r] sig
// (Jacobian).  On the GPU the two scalar multiplications run side by side: lanes 0-3 take [r] H,
// lanes 4-7 [r] sig; lane 0 stores P_i, lane 4 s_i.
G_HD void g_rlc_points(const GCtx& g, const uint32_t* sig_rec, const uint32_t* h_rec, uint64_t r, uint32_t* p_out,
                       uint32_t* s_out) {
    jac<fp> inf;
    inf.inf = true;
    inf.x = inf.y = inf.z = fp_zero();
#ifdef BLS_GDEV
    const bool sig_lane = (g.slot & 4) != 0;
    const uint32_t* src = sig_lane ? sig_rec : h_rec;
    jac<fp> m = inf;
    if (!src[2 * NL]) m = jac_mul64(jac_from_affine(ld_fp(src), ld_fp(src + NL)), r);
    if (g.slot == 4) st_g1j(s_out, m);
    if (g.slot == 0) st_g1j(p_out, m);  // Jacobian: no inversion (g_rlc_ml)
#else
    jac<fp> s = inf, h = inf;
    if (!sig_rec[2 * NL]) s = jac_mul64(jac_from_affine(ld_fp(sig_rec), ld_fp(sig_rec + NL)), r);
    if (!h_rec[2 * NL]) h = jac_mul64(jac_from_affine(ld_fp(h_rec), ld_fp(h_rec + NL)), r);
    st_g1j(s_out, s);
    st_g1j(p_out, h);
#endif
}
// an item outside the batch (failed an earlier check): identity P_i, s_i
G_HD void g_rlc_neutral(const GCtx& g, uint32_t* p_out, uint32_t* s_out) {
    jac<fp> s;
    s.inf = true;
    s.x = s.y = s.z = fp_zero();
#ifdef BLS_GDEV
    if (g.slot != 0) return;
#endif
    st_g1j(s_out, s);
    st_g1j(p_out, s);
}
// stage 3: f = the Miller loop of (P, Q) in W order, 1 for an identity P; P a Jacobian record
// (X, Y, Z), Q = apk (affine record) or g2 for the combination's signature side.  With
// x_P = X / Z^2, y_P = Y / Z^3 every line is evaluated times Z^3 (l0 Z^3 + l1 X Z v + l4 Y v w):
// f picks up a factor in Fp*, which the final exponentiation maps to 1, and no P is inverted.
G_HD void g_rlc_ml(const GCtx& g, const uint32_t* p_rec, const uint32_t* apk_rec, uint32_t* f_out) {
    G12 f = g_one(g);
    const jac<fp> P = ld_g1j(p_rec);
    if (!P.inf) {
        const fp px = fp_mul(P.x, P.z), py = P.y, z3 = fp_mul(fp_sqr(P.z), P.z);
        fp2 qx, qy;
        ld_g2(apk_rec, qx, qy);
        f = g_miller<1, true>(g, &px, &py, &qx, &qy, &z3);
    }
    g_store(g, f_out, f);
}
// the combination's signature side as one more item: P = -S (affine record) and Q = g2, so the
// Miller-loop grid runs one code path on every group (a different path on one group of a wave
// would serialise the wave: measured 2x)
NWV_HD void rlc_sig_item(const uint32_t* s_rec, uint32_t* p_out, uint32_t* q_out) {
    jac<fp> S = ld_g1j(s_rec);
    S.y = fp_neg(S.y);  // -S, still Jacobian (g_rlc_ml)
    st_g1j(p_out, S);
    st_g2(q_out, k_g2x(), k_g2y(), false);
}
// the trees: f_a <- f_a f_b (a group), s_a <- s_a + s_b (a lane)
G_HD void g_rlc_ffold(const GCtx& g, uint32_t* fa, const uint32_t* fb) {
    const G12 f = g_mul(g, g_load(g, fa), g_load(g, fb));
    g_store(g, fa, f);
}
NWV_HD void rlc_sfold(uint32_t* sa, const uint32_t* sb) { st_g1j(sa, jac_add(ld_g1j(sa), ld_g1j(sb))); }
// stage 5: the batch verdict, FE(f) == 1
G_HD bool g_rlc_final(const GCtx& g, const uint32_t* f_rec) { return g_is_one(g, g_final_exp(g, g_load(g, f_rec))); }

// ---- the same check on one whole wave (bls_wave.h) -------------------------------------------
// the line table of an affine Q (a G2 record): (l0, l1, l4) of every Miller-loop step, NSTEPS x 6
// slots of 14 words -- what the loop computes from T when no table is given
template <class W>
NWV_HD void w_key_lines(const W& w, const uint32_t* q_rec, uint32_t* out) {
    using namespace wave;
    init_slots(w);
    w.zero(REG_QB, 6);
    w.sync();
    w.put_words(REG_QB, q_rec, 4);
    w.put_fp(REG_QB + 4, k_one());
    w.sync();
    w.put_words(REG_TB, w.wm + SW * REG_QB, 6);
    w.sync();
    const char* steps = BLS_WAVE_STEPS_STR;
#pragma unroll 1
    for (int k = 0; k < NSTEPS; k++) {
        w.run(steps[k] == 'a' ? P_LINES_ADD : P_LINES_DBL);
        w.get_words(REG_LB, out + (size_t)k * 6 * SW, 6);
        w.sync();
    }
}

// e(-sig, g2) e(H, apk) == 1 from the item's records (sig, H affine G1 records, apk an affine G2
// record); qlines = apk's precomputed line table (a cached key) or null.  The identity signature
// enters as P = (0, 0): its lines reduce to their l0 in Fp2, which the final exponentiation maps
// to 1 (e(O, g2) = 1); every l0 of g2's table is nonzero (checked by the generator).
template <class W>
NWV_HD bool w_pairing_check(const W& w, const uint32_t* sig_rec, const uint32_t* h_rec, const uint32_t* apk_rec,
                            const uint32_t* qlines) {
    using namespace wave;
    init_slots(w);
    w.zero(REG_PA, 2);
    w.zero(REG_PB, 3);
    w.zero(REG_QB, 6);
    w.sync();
    if (!sig_rec[2 * NL]) {
        w.put_words(REG_PA, sig_rec, 1);
        w.put_fp(REG_PA + 1, fp_neg(ld_fp(sig_rec + NL)));
    }
    if (!h_rec[2 * NL]) w.put_words(REG_PB, h_rec, 2);
    w.put_fp(REG_PB + 2, k_one());
    w.put_words(REG_QB, apk_rec, 4);
    w.put_fp(REG_QB + 4, k_one());
    w.sync();
    return wave::pairing_check(w, qlines);
}

// H(msg) on a wave: lanes 0 and 1 each expand the message and map u_0 / u_1 with SSWU (x as a
// fraction: no inversion); the two isogeny maps (homogeneous), their sum and [h_eff] run as
// stage programs.  out: X, Y, Z (x = X / Z, y = Y / Z) and an identity flag (3 NL + 1 words).
constexpr int G1H_REC_WORDS = 3 * NL + 1;
template <class W>
NWV_HD void w_hash_to_g1(const W& w, const uint8_t* msg, uint32_t n, const uint8_t* dst, uint32_t dl, uint32_t* out,
                         bool clear = true) {
    using namespace wave;
    init_slots(w);
    w.lanes(2, [&](int j) {
        uint32_t uw[32];
        expand_xmd_128w(uw, msg, n, dst, dl);
        const fp u0 = fp_from_be64w(uw), u1 = fp_from_be64w(uw + 16);  // constant offsets, then a select
        fp xn, xd, y;
        map_sswu_frac(xn, xd, y, fp_sel(j == 0, u0, u1));
        w.set(REG_S + 3 * j, xn);
        w.set(REG_S + 3 * j + 1, xd);
        w.set(REG_S + 3 * j + 2, y);
    });
    w.sync();
    w.run(P_ISO2_ADD);
    if (clear) g1_chain(w, BLS_H_EFF);  // (else U holds the sum of the two maps)
    w.get_words(REG_U, out, 3);
    w.sync();
    const bool inf = fp_is_zero(w.get(REG_U + 2));
    w.lanes(1, [&](int) { out[3 * NL] = inf ? 1u : 0u; });
}

// the signature's G1 membership on a wave (sig_decode's g1_in_group): [x^2] P = -phi(P) with
// complete formulas; P = the affine record (not the identity)
template <class W>
NWV_HD bool w_g1_in_group(const W& w, const uint32_t* rec) {
    using namespace wave;
    init_slots(w);
    w.put_words(REG_V, rec, 2);
    w.put_words(REG_U, rec, 2);
    w.put_words(REG_S, rec, 2);
    w.put_fp(REG_V + 2, k_one());
    w.put_fp(REG_U + 2, k_one());
    w.sync();
    g1_chain(w, BLS_X_ABS);
    w.run(P_COPY_U_TO_V);
    g1_chain(w, BLS_X_ABS);
    w.run(P_G1_PHI_CHECK);
    return fp_is_zero(w.get(REG_S + 2)) && fp_is_zero(w.get(REG_S + 3));
}

// the general form: H as an affine record (G1_REC_WORDS) or w_hash_to_g1's homogeneous one
// (h_hom), apk as an affine G2 record or a Jacobian one (X, Y, Z; q_jac: k_blsw_apk's)
template <class W>
NWV_HD bool w_pairing_check_g(const W& w, const uint32_t* sig_rec, const uint32_t* h_rec, bool h_hom,
                              const uint32_t* q_rec, bool q_jac, const uint32_t* qlines, bool pc_bank = false) {
    using namespace wave;
    if (pc_bank) init_slots_pc(w);  // a bank of NSLOTS_PC slots (the packed kernel's)
    else init_slots(w);
    w.zero(REG_PA, 2);
    w.zero(REG_PB, 3);
    w.zero(REG_QB, 6);
    w.sync();
    if (!sig_rec[2 * NL]) {
        w.put_words(REG_PA, sig_rec, 1);
        w.put_fp(REG_PA + 1, fp_neg(ld_fp(sig_rec + NL)));
    }
    const bool h_inf = h_rec[(h_hom ? 3 : 2) * NL] != 0;
    if (!h_inf) w.put_words(REG_PB, h_rec, h_hom ? 3 : 2);  // H = O (never from a hash): only l0 remain
    if (h_inf || !h_hom) w.put_fp(REG_PB + 2, k_one());
    w.put_words(REG_QB, q_rec, q_jac ? 6 : 4);
    if (!q_jac) w.put_fp(REG_QB + 4, k_one());
    w.sync();
    return wave::pairing_check(w, qlines, !pc_bank);  // a PC bank holds the one-step programs only
}
// w_pairing_check with H in homogeneous coordinates (w_hash_to_g1's record)
template <class W>
NWV_HD bool w_pairing_check_h(const W& w, const uint32_t* sig_rec, const uint32_t* hh_rec, const uint32_t* apk_rec,
                              const uint32_t* qlines) {
    return w_pairing_check_g(w, sig_rec, hh_rec, true, apk_rec, false, qlines);
}


// ---- AggregateAuthenticator::aggregate (types/src/primary.rs:476-477) on a wave: g1_sum16 adds
// G1SUM_N points with complete formulas (the identity and equal points need no branches); point k
// sits in slots g1sum_slot(k) + 0..2 as (X : Y : Z) and the sum lands in U
constexpr int G1P_WORDS = 3 * NL;  // a homogeneous partial sum (X, Y, Z)
// the smallest sum program over cnt points (1 <= cnt <= G1SUM_N) and its input count
NWV_HD uint32_t g1_sum_width(uint32_t cnt) { return cnt <= 2 ? 2u : cnt <= 4 ? 4u : cnt <= 8 ? 8u : 16u; }
NWV_HD wave::Prog g1_sum_prog(uint32_t cnt) {
    const uint32_t k = g1_sum_width(cnt);
    return k == 2 ? wave::P_G1_SUM2 : k == 4 ? wave::P_G1_SUM4 : k == 8 ? wave::P_G1_SUM8 : wave::P_G1_SUM16;
}
// points a wave takes at a level of m > G1SUM_N inputs
NWV_HD uint32_t g1_sum_per(uint32_t) { return (uint32_t)wave::G1SUM_N; }

// the program's inputs: affine records (hom = 0: G1_REC_WORDS each, identity flagged; record j at
// idx[j] when idx, else at j) or partial sums (hom = 1: G1P_WORDS each); inputs past m are the
// identity.  The caller has run init_slots (the one comes from its constant slot).
template <class W>
NWV_HD void w_g1_sum_put(const W& w, const uint32_t* in, const uint32_t* idx, int hom, uint32_t first, uint32_t m,
                         uint32_t width = wave::G1SUM_N) {
    using namespace wave;
    const uint32_t* one = w.wm + SW * SLOT_ONE;
    for (int k = 0; k < (int)width; k++) {
        const uint32_t j = first + (uint32_t)k;
        const int s = g1sum_slot(k);
        if (j < m && hom) {
            w.put_words(s, in + (size_t)G1P_WORDS * j, 3);
            continue;
        }
        const uint32_t* r = j < m ? in + (size_t)G1_REC_WORDS * (idx ? idx[j] : j) : nullptr;
        if (r && !r[2 * NL]) {
            w.put_words(s, r, 2);
            w.put_words(s + 2, one, 1);
        } else {
            w.zero(s, 3);
            w.sync();
            w.put_words(s + 1, one, 1);
        }
    }
    w.sync();
}

// U (the program's sum) -> the 48-byte compressed point, x = X / Z, y = Y / Z (every lane calls
// it: the inversion runs on the wave; lane 0 writes)
template <class W>
NWV_HD void w_g1_sum_compress(const W& w, uint8_t* out48) {
    using namespace wave;
    const fp X = w.get(REG_U), Y = w.get(REG_U + 1), Z = w.get(REG_U + 2);
    if (fp_is_zero(Z)) {
        if (w.lane == 0) g1_compress(out48, fp_zero(), fp_zero(), true);
        return;
    }
    const fp zi = w.inv(Z);
    if (w.lane == 0) g1_compress(out48, fp_mul(X, zi), fp_mul(Y, zi), false);
}

}  // namespace bls

