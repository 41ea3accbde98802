// Host build of the gfx950 BLS12-381 code (narwhal_amd/csrc/bls381.h, bls_verify.h) -- TEST
// INFRASTRUCTURE ONLY: tests/test_bls_hostemu.py runs these entry points on the CPU against the
// oracle (oracle/bls_oracle.c), so the device arithmetic is checked before it meets a GPU.
// Encodings as the oracle's: uncompressed affine big-endian (G1 x||y, G2 x.c1||x.c0||y.c1||y.c0),
// all-zero = identity; GT as 12 big-endian Fp in tower order.
#include <vector>

#define BLS_GROUP_HOST_EMU 1  // bls_group.h: the host form of the lane-group arithmetic
#include "../../narwhal_amd/csrc/bls_verify.h"

using namespace bls;

static void be_to_mont(fp& r, const uint8_t* b) {
    fp t;
    plain_from_be(t, b);
    r = fp_to_mont(t);
}
static void mont_to_be(uint8_t* b, const fp& a) { plain_to_be(b, fp_from_mont(a)); }

extern "C" {

void bh_pairing(const uint8_t* P, const uint8_t* Q, uint8_t* out) {
    fp px, py;
    fp2 qx, qy;
    be_to_mont(px, P);
    be_to_mont(py, P + 48);
    be_to_mont(qx.c1, Q);
    be_to_mont(qx.c0, Q + 48);
    be_to_mont(qy.c1, Q + 96);
    be_to_mont(qy.c0, Q + 144);
    const fp12 e = final_exp(miller_loop2(1, &px, &py, &qx, &qy));
    const fp* c[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                       &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
    for (int i = 0; i < 12; i++) mont_to_be(out + 48 * i, *c[i]);
}

void bh_hash_to_g1(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dl, uint8_t* out) {
    uint32_t rec[G1_REC_WORDS];
    h2c_record(msg, (uint32_t)n, dst, (uint32_t)dl, rec);
    if (rec[2 * NL]) {
        for (int i = 0; i < 96; i++) out[i] = 0;
        return;
    }
    mont_to_be(out, ld_fp(rec));
    mont_to_be(out + 48, ld_fp(rec + NL));
}

int bh_key_decode(const uint8_t* pk, uint8_t* out_xy) {
    uint32_t rec[G2_REC_WORDS];
    const int32_t st = key_decode(pk, rec);
    fp2 x, y;
    ld_g2(rec, x, y);
    mont_to_be(out_xy, x.c1);
    mont_to_be(out_xy + 48, x.c0);
    mont_to_be(out_xy + 96, y.c1);
    mont_to_be(out_xy + 144, y.c0);
    return st;
}

int bh_sig_decode(const uint8_t* sig, uint8_t* out_xy) {
    uint32_t rec[G1_REC_WORDS];
    const int32_t st = sig_decode(sig, rec);
    mont_to_be(out_xy, ld_fp(rec));
    mont_to_be(out_xy + 48, ld_fp(rec + NL));
    return st;
}

void bh_keygen(const uint8_t* sk, uint8_t* pk) {
    const jac<fp2> q = jac_mul_be(jac_from_affine(k_g2x(), k_g2y()), sk, 32);
    fp2 x = f2_zero(), y = f2_zero();
    if (!q.inf) g2_to_affine(x, y, q);
    g2_compress(pk, x, y, q.inf);
}

void bh_sign(const uint8_t* sk, const uint8_t* msg, size_t n, const uint8_t* dst, size_t dl, uint8_t* sig) {
    const jac<fp> h = hash_to_g1(msg, (uint32_t)n, dst, (uint32_t)dl);
    const jac<fp> s = jac_mul_be(h, sk, 32);
    fp x = fp_zero(), y = fp_zero();
    if (!s.inf) g1_to_affine(x, y, s);
    g1_compress(sig, x, y, s.inf);
}

// fast_aggregate_verify(sig, pks, msg) through the kernels' steps
int bh_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg, size_t n,
                             const uint8_t* dst, size_t dl) {
    uint32_t srec[G1_REC_WORDS], hrec[G1_REC_WORDS], arec[G2_REC_WORDS];
    int32_t st = sig_decode(sig, srec);
    if (st != ST_OK) return st;
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    uint32_t* krec = new uint32_t[G2_REC_WORDS * n_pks];
    int32_t* kst = new int32_t[n_pks];
    uint32_t* idx = new uint32_t[n_pks];
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec, kst, idx, (uint32_t)n_pks, arec);
    delete[] krec;
    delete[] kst;
    delete[] idx;
    if (st != ST_OK) return st;
    h2c_record(msg, (uint32_t)n, dst, (uint32_t)dl, hrec);
    return pairing_check(srec, hrec, arec) ? ST_OK : ST_VERIFY_FAIL;
}

// e(P, Q) through the group arithmetic (bls_group.h, host form): g_final_exp(g_miller(..)) in the
// tower order of bh_pairing, so the two must agree bit for bit
void bh_g_pairing(const uint8_t* P, const uint8_t* Q, uint8_t* out) {
    fp px, py;
    fp2 qx, qy;
    be_to_mont(px, P);
    be_to_mont(py, P + 48);
    be_to_mont(qx.c1, Q);
    be_to_mont(qx.c0, Q + 48);
    be_to_mont(qy.c1, Q + 96);
    be_to_mont(qy.c0, Q + 144);
    const GCtx g{};
    const fp12 e = g_gather(g, g_final_exp(g, g_miller<1>(g, &px, &py, &qx, &qy)));
    const fp* c[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                       &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
    for (int i = 0; i < 12; i++) mont_to_be(out + 48 * i, *c[i]);
}
// the group form of fast_aggregate_verify's pairing equation for one item (as k_bls_pair runs it)
int bh_g_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg, size_t n,
                               const uint8_t* dst, size_t dl) {
    uint32_t srec[G1_REC_WORDS], hrec[G1_REC_WORDS], arec[G2_REC_WORDS];
    int32_t st = sig_decode(sig, srec);
    if (st != ST_OK) return st;
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    uint32_t* krec = new uint32_t[G2_REC_WORDS * n_pks];
    int32_t* kst = new int32_t[n_pks];
    uint32_t* idx = new uint32_t[n_pks];
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec, kst, idx, (uint32_t)n_pks, arec);
    delete[] krec;
    delete[] kst;
    delete[] idx;
    if (st != ST_OK) return st;
    h2c_record(msg, (uint32_t)n, dst, (uint32_t)dl, hrec);
    return g_pairing_check(GCtx{}, srec, hrec, arec) ? ST_OK : ST_VERIFY_FAIL;
}

// the batch check over n items (item i: signature sig + 48 i, one key pk + 96 i, message msg + 32 i)
// exactly as the kernels stage it: points, the G1 tree, the Miller loops (items and (-S, g2)), the
// Fp12 tree, the final exponentiation.  1 accept, 0 reject, -1 if some item fails to decode.
int bh_rlc_batch(size_t n, const uint8_t* sigs, const uint8_t* pks, const uint8_t* msgs, const uint8_t* seed,
                 const uint8_t* dst, size_t dl) {
    const GCtx g{};
    std::vector<uint32_t> f(F12_REC_WORDS * (n + 1)), sj(G1J_REC_WORDS * n), pr(G1J_REC_WORDS * (n + 1)),
        ar(G2_REC_WORDS * (n + 1));
    for (size_t i = 0; i < n; i++) {
        uint32_t srec[G1_REC_WORDS], hrec[G1_REC_WORDS], krec[G2_REC_WORDS];
        const uint32_t idx = 0;
        int32_t kst = key_decode(pks + 96 * i, krec);
        if (sig_decode(sigs + 48 * i, srec) != ST_OK || kst != ST_OK ||
            apk_record(krec, &kst, &idx, 1, ar.data() + G2_REC_WORDS * i) != ST_OK)
            return -1;
        h2c_record(msgs + 32 * i, 32, dst, (uint32_t)dl, hrec);
        g_rlc_points(g, srec, hrec, rlc_scalar(seed, (uint32_t)i), pr.data() + G1J_REC_WORDS * i,
                     sj.data() + G1J_REC_WORDS * i);
    }
    for (size_t m = n; m > 1; m = (m + 1) / 2)
        for (size_t i = 0; i < m - (m + 1) / 2; i++)
            rlc_sfold(sj.data() + G1J_REC_WORDS * i, sj.data() + G1J_REC_WORDS * (i + (m + 1) / 2));
    rlc_sig_item(sj.data(), pr.data() + G1J_REC_WORDS * n, ar.data() + G2_REC_WORDS * n);
    for (size_t i = 0; i <= n; i++)
        g_rlc_ml(g, pr.data() + G1J_REC_WORDS * i, ar.data() + G2_REC_WORDS * i, f.data() + F12_REC_WORDS * i);
    for (size_t m = n + 1; m > 1; m = (m + 1) / 2)
        for (size_t i = 0; i < m - (m + 1) / 2; i++)
            g_rlc_ffold(g, f.data() + F12_REC_WORDS * i, f.data() + F12_REC_WORDS * (i + (m + 1) / 2));
    return g_rlc_final(g, f.data()) ? 1 : 0;
}

// ---- the wave engine (bls_wave.h) on the host: the same interpreter and stage tables -----------
// the device's layout: P << k below slot 0, then NSLOTS slots (the pairing kernels' NSLOTS_PAIR is
// a prefix of it; tests/test_bls_hostemu.py runs under AddressSanitizer too)
static wave::Wave host_wave() {
    static thread_local std::vector<uint32_t> wm(wave::WM_WORDS);
    wave::Wave w;
    w.wm = wm.data() + wave::KP_WORDS;
    return w;
}
static void f12_from_be(const uint8_t* in, uint32_t* slots) {
    for (int k = 0; k < 12; k++) {
        fp v;
        be_to_mont(v, in + 48 * k);
        st_fp(slots + NL * k, v);
    }
}
static void f12_to_be(const uint32_t* slots, uint8_t* out) {
    for (int k = 0; k < 12; k++) mont_to_be(out + 48 * k, ld_fp(slots + NL * k));
}
// op 0: F G (P_MUL_F_G), 1: cyclotomic square (P_CYC_SQR_F), 2: F^2 (P_SQR_F), 3: the final
// exponentiation; a, b: 12 big-endian Fp in tower order
void bh_w_f12_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
    const wave::Wave w = host_wave();
    wave::init_slots(w);
    f12_from_be(a, w.wm + NL * wave::REG_F);
    if (b) f12_from_be(b, w.wm + NL * wave::REG_G);
    if (op == 0) w.run(wave::P_MUL_F_G);
    else if (op == 1) w.run(wave::P_CYC_SQR_F);
    else if (op == 2) w.run(wave::P_SQR_F);
    else wave::final_exp(w);
    f12_to_be(w.wm + NL * wave::REG_F, out);
}
// fast_aggregate_verify with the pairing check on the (host-emulated) wave; lines: 1 = apk's line
// table precomputed by the lines programs (the cached-key path), 0 = computed in the loop
int bh_w_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg, size_t n,
                               const uint8_t* dst, size_t dl, int lines) {
    uint32_t srec[G1_REC_WORDS], hrec[G1_REC_WORDS], arec[G2_REC_WORDS];
    int32_t st = sig_decode(sig, srec);
    if (st != ST_OK) return st;
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    std::vector<uint32_t> krec(G2_REC_WORDS * n_pks), idx(n_pks);
    std::vector<int32_t> kst(n_pks);
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec.data() + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec.data(), kst.data(), idx.data(), (uint32_t)n_pks, arec);
    if (st != ST_OK) return st;
    h2c_record(msg, (uint32_t)n, dst, (uint32_t)dl, hrec);
    const wave::Wave w = host_wave();
    std::vector<uint32_t> tab;
    if (lines) {
        tab.resize((size_t)wave::NSTEPS * 6 * NL);
        w_key_lines(w, arec, tab.data());
    }
    return w_pairing_check(w, srec, hrec, arec, lines ? tab.data() : nullptr) ? ST_OK : ST_VERIFY_FAIL;
}

// H(msg) by the wave programs (homogeneous), returned affine like bh_hash_to_g1
void bh_w_hash_to_g1(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dl, uint8_t* out) {
    const wave::Wave w = host_wave();
    uint32_t rec[G1H_REC_WORDS];
    w_hash_to_g1(w, msg, (uint32_t)n, dst, (uint32_t)dl, rec);
    if (rec[3 * NL]) {
        for (int i = 0; i < 96; i++) out[i] = 0;
        return;
    }
    const fp zi = fp_inv(ld_fp(rec + 2 * NL));
    mont_to_be(out, fp_mul(ld_fp(rec), zi));
    mont_to_be(out + 48, fp_mul(ld_fp(rec + NL), zi));
}
// the signature's status with the G1 membership test on the wave (decode, then w_g1_in_group)
int bh_w_sig_status(const uint8_t* sig) {
    fp x, y;
    bool inf;
    int32_t st = g1_decompress(x, y, inf, sig);
    if (st != ST_OK || inf) return st;
    uint32_t rec[G1_REC_WORDS];
    st_g1(rec, x, y, false);
    return w_g1_in_group(host_wave(), rec) ? ST_OK : ST_NOT_IN_GROUP;
}
// fast_aggregate_verify with every step of the wave pipeline: signature decode + wave G1 check,
// keys, wave hash to G1 (homogeneous), wave pairing check
int bh_w2_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg, size_t n,
                                const uint8_t* dst, size_t dl) {
    int32_t st = bh_w_sig_status(sig);
    if (st != ST_OK) return st;
    uint32_t srec[G1_REC_WORDS], hrec[G1H_REC_WORDS], arec[G2_REC_WORDS];
    fp x, y;
    bool inf;
    g1_decompress(x, y, inf, sig);
    st_g1(srec, inf ? fp_zero() : x, inf ? fp_zero() : y, inf);
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    std::vector<uint32_t> krec(G2_REC_WORDS * n_pks), idx(n_pks);
    std::vector<int32_t> kst(n_pks);
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec.data() + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec.data(), kst.data(), idx.data(), (uint32_t)n_pks, arec);
    if (st != ST_OK) return st;
    const wave::Wave w = host_wave();
    w_hash_to_g1(w, msg, (uint32_t)n, dst, (uint32_t)dl, hrec);
    return w_pairing_check_h(w, srec, hrec, arec, nullptr) ? ST_OK : ST_VERIFY_FAIL;
}

// the same check with the cofactor clearing moved from H onto the key sum:
// e(H0, [h_eff] apk) for H0 = iso(SSWU(u0)) + iso(SSWU(u1)) (not cleared); mode 1 = computed lines,
// 2 = the line table of [h_eff] apk
int bh_w3_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg, size_t n,
                                const uint8_t* dst, size_t dl, int mode) {
    int32_t st = bh_w_sig_status(sig);
    if (st != ST_OK) return st;
    uint32_t srec[G1_REC_WORDS], hrec[G1H_REC_WORDS], arec[G2_REC_WORDS];
    fp x, y;
    bool inf;
    g1_decompress(x, y, inf, sig);
    st_g1(srec, inf ? fp_zero() : x, inf ? fp_zero() : y, inf);
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    std::vector<uint32_t> krec(G2_REC_WORDS * n_pks), idx(n_pks);
    std::vector<int32_t> kst(n_pks);
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec.data() + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec.data(), kst.data(), idx.data(), (uint32_t)n_pks, arec);
    if (st != ST_OK) return st;
    fp2 ax, ay;
    ld_g2(arec, ax, ay);
    const jac<fp2> hq = jac_mul64(jac_from_affine(ax, ay), BLS_H_EFF);
    g2_to_affine(ax, ay, hq);
    st_g2(arec, ax, ay, false);
    const wave::Wave w = host_wave();
    w_hash_to_g1(w, msg, (uint32_t)n, dst, (uint32_t)dl, hrec, false);
    std::vector<uint32_t> tab;
    if (mode == 2) {
        tab.resize((size_t)wave::NSTEPS * 6 * NL);
        w_key_lines(w, arec, tab.data());
    }
    return w_pairing_check_h(w, srec, hrec, arec, mode == 2 ? tab.data() : nullptr) ? ST_OK : ST_VERIFY_FAIL;
}

// the pairing check on a bank of exactly NSLOTS_PC slots (the packed kernel's k_blsw_pair_k bank),
// with a canary behind it: the pairing check's programs must address nothing past NSLOTS_PC.
// mode 1 = computed lines, 2 = the key's line table (precomputed on a full-size wave).  Returns
// the status, or -1000 when the canary was touched.
int bh_w_pc_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg, size_t n,
                                  const uint8_t* dst, size_t dl, int mode) {
    int32_t st = bh_w_sig_status(sig);
    if (st != ST_OK) return st;
    uint32_t srec[G1_REC_WORDS], hrec[G1H_REC_WORDS], arec[G2_REC_WORDS];
    fp x, y;
    bool inf;
    g1_decompress(x, y, inf, sig);
    st_g1(srec, inf ? fp_zero() : x, inf ? fp_zero() : y, inf);
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    std::vector<uint32_t> krec(G2_REC_WORDS * n_pks), idx(n_pks);
    std::vector<int32_t> kst(n_pks);
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec.data() + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec.data(), kst.data(), idx.data(), (uint32_t)n_pks, arec);
    if (st != ST_OK) return st;
    const wave::Wave full = host_wave();
    w_hash_to_g1(full, msg, (uint32_t)n, dst, (uint32_t)dl, hrec);
    std::vector<uint32_t> tab;
    if (mode == 2) {
        tab.resize((size_t)wave::NSTEPS * 6 * NL);
        w_key_lines(full, arec, tab.data());
    }
    constexpr uint32_t CANARY = 0xC0FFEE11u, CW = 4096;
    std::vector<uint32_t> bank(wave::WM_WORDS_PC + CW, CANARY);
    wave::Wave w;
    w.wm = bank.data() + wave::KP_WORDS;
    const bool ok = w_pairing_check_g(w, srec, hrec, true, arec, false, mode == 2 ? tab.data() : nullptr, true);
    for (uint32_t i = 0; i < CW; i++)
        if (bank[wave::WM_WORDS_PC + i] != CANARY) return -1000;
    return ok ? ST_OK : ST_VERIFY_FAIL;
}

// the packed kernel's flat script (wave::pairing_script, k_blsw_pair_k): the same set-up as
// bh_w_pc_fast_aggregate_verify, then the script's ops on the host wave -- RUN a program, LINES
// the step's lines into LA (g2's) and LB (the key's table, fixed mode), INV the inversion -- and
// F == 1.  mode 1 = computed lines, 2 = the key's line table.  Returns the status; *n_ops the
// script's length.
int bh_w_script_fast_aggregate_verify(const uint8_t* sig, size_t n_pks, const uint8_t* pks, const uint8_t* msg,
                                      size_t n, const uint8_t* dst, size_t dl, int mode, int* n_ops) {
    using namespace wave;
    int32_t st = bh_w_sig_status(sig);
    if (st != ST_OK) return st;
    uint32_t srec[G1_REC_WORDS], hrec[G1H_REC_WORDS], arec[G2_REC_WORDS];
    fp x, y;
    bool inf;
    g1_decompress(x, y, inf, sig);
    st_g1(srec, inf ? fp_zero() : x, inf ? fp_zero() : y, inf);
    if (n_pks == 0) return ST_AGGR_MISMATCH;
    std::vector<uint32_t> krec(G2_REC_WORDS * n_pks), idx(n_pks);
    std::vector<int32_t> kst(n_pks);
    for (size_t i = 0; i < n_pks; i++) {
        kst[i] = key_decode(pks + 96 * i, krec.data() + G2_REC_WORDS * i);
        idx[i] = (uint32_t)i;
    }
    st = apk_record(krec.data(), kst.data(), idx.data(), (uint32_t)n_pks, arec);
    if (st != ST_OK) return st;
    const Wave full = host_wave();
    w_hash_to_g1(full, msg, (uint32_t)n, dst, (uint32_t)dl, hrec);
    std::vector<uint32_t> tab;
    const bool fixed = mode == 2;
    if (fixed) {
        tab.resize((size_t)NSTEPS * 6 * NL);
        w_key_lines(full, arec, tab.data());
    }
    std::vector<uint32_t> bank(WM_WORDS_PC, 0);
    Wave w;
    w.wm = bank.data() + KP_WORDS;
    init_slots_pc(w);
    w.zero(REG_PA, 2);
    w.zero(REG_PB, 3);
    w.zero(REG_QB, 6);
    if (!srec[2 * NL]) {
        w.put_words(REG_PA, srec, 1);
        w.put_fp(REG_PA + 1, fp_neg(ld_fp(srec + NL)));
    }
    if (!hrec[3 * NL]) w.put_words(REG_PB, hrec, 3);
    else w.put_fp(REG_PB + 2, k_one());
    w.put_words(REG_QB, arec, 4);
    w.put_fp(REG_QB + 4, k_one());
    w.zero(REG_F, 12);
    w.put_fp(REG_F, k_one());
    w.copy_slots(REG_TB, REG_QB, 6);
    static SOp ops[SCRIPT_MAX];
    const int cnt = pairing_script(fixed, ops);
    *n_ops = cnt;
    for (int i = 0; i < cnt; i++) {
        const SOp& o = ops[i];
        if (sop_kind(o) == SOP_LINES) {
            w.put_words(REG_LA, &T_G2_LINES[o.a][0][0], 6);
            if (fixed) w.put_words(REG_LB, tab.data() + (size_t)o.a * 6 * NL, 6);
        } else if (sop_kind(o) == SOP_INV) {
            w.invert_slot((int)o.a, (int)o.b);
        } else {
            // next_run must name the next RUN op
            int j = i + 1;
            while (j < cnt && sop_kind(ops[j]) != SOP_RUN) j++;
            if (o.next_run != (j < cnt ? j : -1)) return -2000;
            w.run(Prog{o.a, (uint16_t)(o.b & 0xffffu), (uint16_t)(o.b >> 16)}, (int)(o.c & 0xffffu));
        }
    }
    return w.f_is_one() ? ST_OK : ST_VERIFY_FAIL;
}

// the variable-time inversion of the wave engine's final exponentiation (plain big-endian in / out)
void bh_fp_inv_vt(const uint8_t* a, uint8_t* out) {
    fp x;
    be_to_mont(x, a);
    mont_to_be(out, fp_inv_vt(x));
}
// the row form (fp_inv_wave's order of updates, one row after another)
void bh_fp_inv_rows(const uint8_t* a, uint8_t* out) {
    fp x;
    be_to_mont(x, a);
    mont_to_be(out, inv_rows(x));
}

// AggregateAuthenticator::aggregate as the device runs it: statuses in list order (decode, then
// the wave G1 check), the records summed 16 at a time by the g1_sum programs into partial sums, the partials
// summed the same way, U compressed (first = 0: records straight; first = 1: through a reversed
// position list, as the verified-signature ring is read)
int bh_w_aggregate(size_t n, const uint8_t* sigs, uint8_t* out48, int through_idx) {
    if (n == 0) return ST_AGGR_MISMATCH;
    std::vector<uint32_t> rec(G1_REC_WORDS * n), pos(n);
    for (size_t i = 0; i < n; i++) {
        const int32_t st = bh_w_sig_status(sigs + 48 * i);
        if (st != ST_OK) return st;
        fp x, y;
        bool inf;
        g1_decompress(x, y, inf, sigs + 48 * i);
        const size_t at = through_idx ? n - 1 - i : i;  // record i stored at position `at`
        st_g1(rec.data() + G1_REC_WORDS * at, inf ? fp_zero() : x, inf ? fp_zero() : y, inf);
        pos[i] = (uint32_t)at;
    }
    const wave::Wave w = host_wave();
    const uint32_t* src = rec.data();
    const uint32_t* idx = through_idx ? pos.data() : nullptr;
    int hom = 0;
    size_t m = n;
    std::vector<uint32_t> part;
    while (m > (size_t)wave::G1SUM_N) {
        const size_t per = g1_sum_per((uint32_t)m), nb = (m + per - 1) / per;
        std::vector<uint32_t> nxt(G1P_WORDS * nb);
        for (size_t b = 0; b < nb; b++) {
            const uint32_t cnt = (uint32_t)(m - b * per < per ? m - b * per : per);
            wave::init_slots(w);
            w_g1_sum_put(w, src, idx, hom, (uint32_t)(b * per), (uint32_t)m, g1_sum_width(cnt));
            w.run(g1_sum_prog(cnt));
            w.get_words(wave::REG_U, nxt.data() + G1P_WORDS * b, 3);
        }
        part.swap(nxt);
        src = part.data();
        idx = nullptr;
        hom = 1;
        m = nb;
    }
    wave::init_slots(w);
    w_g1_sum_put(w, src, idx, hom, 0, (uint32_t)m, g1_sum_width((uint32_t)m));
    w.run(g1_sum_prog((uint32_t)m));
    w_g1_sum_compress(w, out48);
    return ST_OK;
}

}  // extern "C"

