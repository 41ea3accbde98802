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

}  // extern "C"
