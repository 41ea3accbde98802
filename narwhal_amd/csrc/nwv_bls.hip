// nwv_bls.hip -- BLS12-381 min_sig verification engine on gfx950: the
// kernels over bls_verify.h and the C ABI of include/nwv_bls.h.
//
// A call stages its inputs in one pinned arena and one H2D copy, then runs on three streams
//   k_bls_keys_fill  one lane per key the device's key cache has not seen: decode + G2 membership
//                    (psi(Q) = [x] Q), into the cache (fastcrypto validates a key once, at
//                    deserialization); then k_bls_apk_g, one 8-lane group per item: the sum of the
//                    item's keys (eight partial sums and a tree), its first bad key's status
//   k_bls_sigs       one lane per item: decode + G1 membership (phi(P) = [-x^2] P)
//   k_bls_h2c_g      one 8-lane group per item: H(msg) (RFC 9380 hash_to_curve G1), the two
//                    field elements mapped side by side
// joined by k_bls_status (the statuses in the oracle's order), then
//   the pairing check, by default as ONE batch check over the call (bls_verify.h, kernels below:
//     [r_i] H_i and [r_i] sig_i per item, S = sum [r_i] sig_i, every item's Miller loop and that
//     of (-S, g2) in one grid, a product tree, one final exponentiation)
//   and only when that rejects (or under NWV_FLAG_BLS_PER_ITEM)
//     k_bls_pair   one lane per item: e(-sig, g2) e(H, apk) == 1 (two-pair Miller loop + final exp)
// and copies the per-item statuses back.  The Miller loops are the hot part: Fp products on VALU
// v_mad_u64_u32 (bls381.h), no MFMA (no dense contraction).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/nwv.h"
#include "../../include/nwv_bls.h"
#include "bls_verify.h"
#include "bls_shard.h"
#include "stage_args.h"

using namespace bls;
using nwv::bls_for_ranges;
using nwv::bls_shard_ranges;

__attribute__((visibility("hidden"))) int nwv_internal_set_err(int code, const char* msg);
extern "C" {  // defined in nwv_host.hip's extern "C" section
__attribute__((visibility("hidden"))) uint32_t nwv_internal_ctx_flags(const nwv_ctx* ctx);
__attribute__((visibility("hidden"))) void nwv_internal_fill_seed(const uint8_t* seed32, uint8_t out[32]);
}

// ------------------------------------------------------------------------------ kernels
#define BLS_LANES 64
#define BLS_IDX() const uint32_t i = blockIdx.x * BLS_LANES + threadIdx.x; \
    if (i >= n) return

// decode + check keys: key j of the list goes to record slot slot[j] (the committee key cache at
// registration, or a call's scratch table for keys the cache does not hold)
__global__ __launch_bounds__(BLS_LANES) void k_bls_keys_fill(uint32_t n, const uint8_t* pk, const uint32_t* slot,
                                                             uint32_t* rec, int32_t* st) {
    BLS_IDX();
    const uint32_t k = slot[i];
    st[k] = key_decode(pk + 96 * (size_t)i, rec + (size_t)G2_REC_WORDS * k);
}
// copy validated records into the key cache: record src[j] of `from` -> slot dst[j] of `to`
__global__ __launch_bounds__(BLS_LANES) void k_bls_rec_copy(uint32_t n, const uint32_t* src, const uint32_t* dst,
                                                            const uint32_t* from, uint32_t* to, int32_t* to_st) {
    const uint32_t t = blockIdx.x * BLS_LANES + threadIdx.x;
    const uint32_t i = t / G2_REC_WORDS, w = t % G2_REC_WORDS;
    if (i >= n) return;
    to[(size_t)G2_REC_WORDS * dst[i] + w] = from[(size_t)G2_REC_WORDS * src[i] + w];
    if (w == 0) to_st[dst[i]] = ST_OK;
}
// A call's key table: index k < KC_CAP names slot k of the device's key cache, k >= KC_CAP entry
// k - KC_CAP of the call's scratch table (keys the cache does not hold, decoded by this call)
constexpr uint32_t KC_CAP = 65536;
constexpr uint32_t SC_CAP = 65536;  // the verified-signature ring (BlsSigCache)
struct KeyTab {
    const uint32_t* rc;
    const int32_t* sc;
    const uint32_t* rs;
    const int32_t* ss;
    const uint32_t* lines;  // cached keys' Miller-loop line tables (KL_WORDS per slot), or null
    const uint32_t* hrc;    // cached keys' [h_eff] pk records (G2_REC_WORDS per slot), or null
};
// words of a registered key's line table: (l0, l1, l4) of every Miller-loop step (w_key_lines)
constexpr size_t KL_WORDS = (size_t)wave::NSTEPS * 6 * wave::SW;
__device__ inline const uint32_t* key_rec(const KeyTab& t, uint32_t k) {
    return k < KC_CAP ? t.rc + (size_t)G2_REC_WORDS * k : t.rs + (size_t)G2_REC_WORDS * (k - KC_CAP);
}
__device__ inline int32_t key_st(const KeyTab& t, uint32_t k) { return k < KC_CAP ? t.sc[k] : t.ss[k - KC_CAP]; }
__global__ __launch_bounds__(BLS_LANES) void k_bls_sigs(uint32_t n, const uint8_t* sig, uint32_t* rec, int32_t* st) {
    BLS_IDX();
    st[i] = sig_decode(sig + 48 * (size_t)i, rec + (size_t)G1_REC_WORDS * i);
}
// the pairing kernels run one item per GROUP of 8 lanes (bls_group.h): 8 items per 64-lane block
#define BLS_GIDX()                                                                  \
    __shared__ uint32_t g_lds[(BLS_LANES / GRP) * GX_WORDS];                       \
    const GCtx g = g_ctx(g_lds);                                                    \
    const uint32_t i = blockIdx.x * (BLS_LANES / GRP) + threadIdx.x / GRP;          \
    if (i >= n) return

// the key sum of item i over a group: lane s adds the item's keys s, s + 8, ... (apk_record's
// formulas), the eight partial sums meet in a three-level tree through the group's LDS area, and
// the status is that of the item's FIRST bad key in list order (apk_record's), else identity ->
// PK_INFINITY.  st_apk[i] = the item's key status (the signature's status is combined later).
constexpr int G2J_WORDS = 6 * NL + 1;  // Jacobian X, Y, Z (Fp2 each), identity flag
__device__ void st_g2j(uint32_t* o, const jac<fp2>& p) {
    st_f2(o, p.x);
    st_f2(o + F2W, p.y);
    st_f2(o + 2 * F2W, p.z);
    o[3 * F2W] = p.inf ? 1u : 0u;
}
__device__ jac<fp2> ld_g2j(const uint32_t* o) {
    jac<fp2> p;
    p.x = ld_f2(o);
    p.y = ld_f2(o + F2W);
    p.z = ld_f2(o + 2 * F2W);
    p.inf = o[3 * F2W] != 0;
    return p;
}
static_assert(4 * G2J_WORDS + 8 <= GX_WORDS, "the tree's first level fits a group's LDS area");
__global__ __launch_bounds__(BLS_LANES) void k_bls_apk_g(uint32_t n, KeyTab kt, const uint32_t* pk_off,
                                                         const uint32_t* pk_cnt, const uint32_t* pk_idx, uint32_t* rec,
                                                         int32_t* st_apk) {
    BLS_GIDX();
    const uint32_t cnt = pk_cnt[i];
    const uint32_t* idx = pk_idx + pk_off[i];
    uint32_t* out = rec + (size_t)G2_REC_WORDS * i;
    if (cnt == 1) {  // one key (Verifier::verify): its validated record is the sum, no inversion
        if (g.slot < G2_REC_WORDS) {
            const uint32_t k = idx[0];
            const int32_t ks = key_st(kt, k);
            const uint32_t* kr = key_rec(kt, k);
            for (int w = g.slot; w < G2_REC_WORDS; w += GRP) out[w] = ks == ST_OK ? kr[w] : (w == 4 * NL ? 1u : 0u);
            if (g.slot == 0) st_apk[i] = ks;
        }
        return;
    }
    jac<fp2> acc;
    acc.inf = true;
    acc.x = acc.y = acc.z = f2_zero();
    uint32_t first_bad = 0xffffffffu;
    for (uint32_t j = (uint32_t)g.slot; j < cnt; j += GRP) {
        const uint32_t k = idx[j];
        if (key_st(kt, k) != ST_OK) {
            first_bad = j;
            break;
        }
        fp2 x, y;
        ld_g2(key_rec(kt, k), x, y);
        acc = jac_add(acc, jac_from_affine(x, y));
    }
    // the group's first bad position, and the tree over the partial sums
    uint32_t* xa = g.xa;
    g_sync();
    xa[4 * G2J_WORDS + g.slot] = first_bad;
#pragma unroll 1
    for (int h = GRP / 2; h >= 1; h /= 2) {
        g_sync();
        if (g.slot >= h && g.slot < 2 * h) st_g2j(xa + (g.slot - h) * G2J_WORDS, acc);
        g_sync();
        if (g.slot < h) acc = jac_add(acc, ld_g2j(xa + g.slot * G2J_WORDS));
    }
    g_sync();
    uint32_t fb = 0xffffffffu;
    for (int s2 = 0; s2 < GRP; s2++) fb = min(fb, xa[4 * G2J_WORDS + s2]);
    if (g.slot != 0) return;
    int32_t status;
    fp2 x = f2_zero(), y = f2_zero();
    bool inf = true;
    if (cnt == 0) {
        status = ST_AGGR_MISMATCH;
    } else if (fb != 0xffffffffu) {
        status = key_st(kt, idx[fb]);
    } else {
        if (!acc.inf) g2_to_affine(x, y, acc);
        inf = acc.inf;
        status = acc.inf ? ST_PK_INFINITY : ST_OK;
    }
    if (status != ST_OK) {
        x = y = f2_zero();
        inf = true;
    }
    st_g2(out, x, y, inf);
    st_apk[i] = status;
}
// H(msg_i) on a group: lanes 0-3 map hash_to_field's u_0, lanes 4-7 u_1 (side by side), lane 4
// hands its point to lane 0 through the group's LDS area, lane 0 adds and clears the cofactor
// (kmode[i] = 1: item i's cofactor clearing is on its key side -- H0 = the maps' sum, see
// k_bls_key_heff; kmode may be null)
__global__ __launch_bounds__(BLS_LANES) void k_bls_h2c_g(uint32_t n, const uint8_t* msg, const uint64_t* off,
                                                         const uint32_t* len, const uint8_t* dst, uint32_t dl,
                                                         uint32_t* rec, const uint32_t* kmode) {
    BLS_GIDX();
    const jac<fp> q = h2c_map(msg + off[i], len[i], dst, dl, (g.slot & 4) ? 1 : 0);
    g_sync();
    if (g.slot == 4) st_g1j(g.xa, q);
    g_sync();
    const jac<fp> q1 = ld_g1j(g.xa);
    if (g.slot != 0) return;
    const jac<fp> h0 = jac_add(q, q1);
    const jac<fp> h = kmode && kmode[i] ? h0 : jac_mul64(h0, BLS_H_EFF);
    fp x = fp_zero(), y = fp_zero();
    if (!h.inf) g1_to_affine_vt(x, y, h);
    st_g1(rec + (size_t)G1_REC_WORDS * i, x, y, h.inf);
}
// The same on a lane pair: lane 2 j maps u_0 and lane 2 j + 1 u_1 of item 32 b + j; the odd lane
// hands its point over through LDS.  32 items a wave instead of 8: a 16,384-item call is 512 waves
// (one per SIMD at most) instead of 2,048 (two per SIMD, six of every group's eight lanes
// repeating the pair's work), so each lane's dependent chain runs with its SIMD to itself.
constexpr int G1J_WORDS = 3 * NL + 1;
__global__ __launch_bounds__(BLS_LANES) void k_bls_h2c_2(uint32_t n, const uint8_t* msg, const uint64_t* off,
                                                         const uint32_t* len, const uint8_t* dst, uint32_t dl,
                                                         uint32_t* rec, const uint32_t* kmode) {
    __shared__ uint32_t xa[(BLS_LANES / 2) * G1J_WORDS];
    const int pr = (int)threadIdx.x >> 1, u = (int)threadIdx.x & 1;
    const uint32_t i = blockIdx.x * (BLS_LANES / 2) + (uint32_t)pr;
    jac<fp> q;
    if (i < n) {
        q = h2c_map(msg + off[i], len[i], dst, dl, u);
        if (u) st_g1j(xa + G1J_WORDS * pr, q);
    }
    __syncthreads();
    if (i >= n || u) return;
    const jac<fp> q1 = ld_g1j(xa + G1J_WORDS * pr);
    const jac<fp> h0 = jac_add(q, q1);
    const jac<fp> h = kmode && kmode[i] ? h0 : jac_mul64(h0, BLS_H_EFF);
    fp x = fp_zero(), y = fp_zero();
    if (!h.inf) g1_to_affine_vt(x, y, h);
    st_g1(rec + (size_t)G1_REC_WORDS * i, x, y, h.inf);
}
// the item's status in the oracle's order: the signature's, then the keys'
__global__ __launch_bounds__(BLS_LANES) void k_bls_status(uint32_t n, const int32_t* st_sig, const int32_t* st_apk,
                                                          int32_t* st) {
    BLS_IDX();
    st[i] = st_sig[i] != ST_OK ? st_sig[i] : st_apk[i];
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_pair(uint32_t n, const uint32_t* sig_rec, const uint32_t* h_rec,
                                                        const uint32_t* apk_rec, int32_t* st) {
    BLS_GIDX();
    if (st[i] != ST_OK) return;  // uniform over the group
    const bool ok = g_pairing_check(g, sig_rec + (size_t)G1_REC_WORDS * i, h_rec + (size_t)G1_REC_WORDS * i,
                                    apk_rec + (size_t)G2_REC_WORDS * i);
    g_sync();
    if (g.slot == 0) st[i] = ok ? ST_OK : ST_VERIFY_FAIL;
}
// the batch check (bls_verify.h), in stages:
//   k_bls_rlc_pts   one group per item: P_i = [r_i] H_i, s_i = [r_i] sig_i (Jacobian)
//   k_bls_sfold     ceil(log2 n) levels of G1 sums: S = sum s_i
//   k_bls_sig_item  one lane: (-S, g2) as item n
//   k_bls_rlc_ml    one group per item and one more: the Miller loops of (P_i, apk_i) and (-S, g2)
//   k_bls_ffold     ceil(log2 (n + 1)) levels of group Fp12 products
//   k_bls_final     one group: the final exponentiation, == 1
__global__ __launch_bounds__(BLS_LANES) void k_bls_rlc_pts(uint32_t n, const uint32_t* sig_rec, const uint32_t* h_rec,
                                                           const int32_t* st, const uint8_t* seed, uint32_t* prec,
                                                           uint32_t* srec) {
    BLS_GIDX();
    uint32_t* p = prec + (size_t)G1J_REC_WORDS * i;
    uint32_t* s = srec + (size_t)G1J_REC_WORDS * i;
    if (st[i] != ST_OK) {
        g_rlc_neutral(g, p, s);
        return;
    }
    g_rlc_points(g, sig_rec + (size_t)G1_REC_WORDS * i, h_rec + (size_t)G1_REC_WORDS * i, rlc_scalar(seed, i), p, s);
}
// one level of a tree over m entries: entry j <- entry j (+) entry j + h, h = ceil(m / 2), j < m - h
__global__ __launch_bounds__(BLS_LANES) void k_bls_sfold(uint32_t m, uint32_t* srec) {
    const uint32_t h = (m + 1) / 2;
    const uint32_t n = m - h;
    BLS_IDX();
    rlc_sfold(srec + (size_t)G1J_REC_WORDS * i, srec + (size_t)G1J_REC_WORDS * (i + h));
}
// -S (affine) and g2 as item n of the Miller-loop grid (srec[0] = S after the G1 tree)
__global__ void k_bls_sig_item(uint32_t n, const uint32_t* srec, uint32_t* prec, uint32_t* apk_rec) {
    if (blockIdx.x || threadIdx.x) return;
    rlc_sig_item(srec, prec + (size_t)G1J_REC_WORDS * n, apk_rec + (size_t)G2_REC_WORDS * n);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_rlc_ml(uint32_t n, const uint32_t* prec, const uint32_t* apk_rec,
                                                          uint32_t* frec) {
    BLS_GIDX();
    g_rlc_ml(g, prec + (size_t)G1J_REC_WORDS * i, apk_rec + (size_t)G2_REC_WORDS * i, frec + (size_t)F12_REC_WORDS * i);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_ffold(uint32_t m, uint32_t* frec) {
    const uint32_t h = (m + 1) / 2;
    const uint32_t n = m - h;
    BLS_GIDX();
    g_rlc_ffold(g, frec + (size_t)F12_REC_WORDS * i, frec + (size_t)F12_REC_WORDS * (i + h));
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_final(const uint32_t* frec, int32_t* ok) {
    const uint32_t n = 1;
    BLS_GIDX();
    const bool r = g_rlc_final(g, frec);
    g_sync();
    if (g.slot == 0) *ok = r ? 1 : 0;
}
// st[i] <- the decode status when it is a failure, else the G1 check's
__global__ __launch_bounds__(BLS_LANES) void k_bls_st_join(uint32_t n, const int32_t* dec, int32_t* st) {
    BLS_IDX();
    if (dec[i] != ST_OK) st[i] = dec[i];
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_keygen(uint32_t n, const uint8_t* sk, uint8_t* pk) {
    BLS_IDX();
    const jac<fp2> q = jac_mul_be(jac_from_affine(k_g2x(), k_g2y()), sk + 32 * (size_t)i, 32);
    fp2 x = f2_zero(), y = f2_zero();
    if (!q.inf) g2_to_affine(x, y, q);
    g2_compress(pk + 96 * (size_t)i, x, y, q.inf);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_sign(uint32_t n, const uint8_t* sk, const uint8_t* msg,
                                                        const uint64_t* off, const uint32_t* len, const uint8_t* dst,
                                                        uint32_t dl, uint8_t* sig) {
    BLS_IDX();
    const jac<fp> s = jac_mul_be(hash_to_g1(msg + off[i], len[i], dst, dl), sk + 32 * (size_t)i, 32);
    fp x = fp_zero(), y = fp_zero();
    if (!s.inf) g1_to_affine(x, y, s);
    g1_compress(sig + 48 * (size_t)i, x, y, s.inf);
}
__device__ void be_to_mont(fp& r, const uint8_t* b) {
    fp t;
    plain_from_be(t, b);
    r = fp_to_mont(t);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_h2c_out(uint32_t n, const uint8_t* msg, const uint64_t* off,
                                                           const uint32_t* len, const uint8_t* dst, uint32_t dl,
                                                           uint8_t* out) {
    BLS_IDX();
    uint32_t rec[G1_REC_WORDS];
    h2c_record(msg + off[i], len[i], dst, dl, rec);
    uint8_t* o = out + 96 * (size_t)i;
    if (rec[2 * NL]) {
        for (int k = 0; k < 96; k++) o[k] = 0;
        return;
    }
    plain_to_be(o, fp_from_mont(ld_fp(rec)));
    plain_to_be(o + 48, fp_from_mont(ld_fp(rec + NL)));
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_pairing_raw(uint32_t n, const uint8_t* P, const uint8_t* Q,
                                                               uint8_t* out) {
    BLS_IDX();
    const uint8_t* p = P + 96 * (size_t)i;
    const uint8_t* q = Q + 192 * (size_t)i;
    uint32_t zp = 0, zq = 0;
    for (int k = 0; k < 96; k++) zp |= p[k];
    for (int k = 0; k < 192; k++) zq |= q[k];
    fp12 e = f12_one();
    if (zp && zq) {
        fp px, py;
        fp2 qx, qy;
        be_to_mont(px, p);
        be_to_mont(py, p + 48);
        be_to_mont(qx.c1, q);
        be_to_mont(qx.c0, q + 48);
        be_to_mont(qy.c1, q + 96);
        be_to_mont(qy.c0, q + 144);
        e = final_exp(miller_loop2(1, &px, &py, &qx, &qy));
    }
    const fp* c[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                       &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
    uint8_t* o = out + 576 * (size_t)i;
    for (int k = 0; k < 12; k++) plain_to_be(o + 48 * k, fp_from_mont(*c[k]));
}

// ---- the wave engine (bls_wave.h): one 64-lane wave per item ------------------------------------
// a wave's LDS for programs of up to NS slots: wm points at slot 0 (P << k sits below it)
#define BLSW_LDS(NS)                                            \
    __shared__ uint32_t wm_lds[wave::KP_WORDS + wave::SW * (NS)]; \
    uint32_t* const wm = wm_lds + wave::KP_WORDS
#define BLSW_IDX()                    \
    BLSW_LDS(wave::NSLOTS_PAIR);      \
    const uint32_t i = blockIdx.x;    \
    if (i >= n) return
// H(msg_i), homogeneous
__device__ __forceinline__ void blsw_h2c_item(uint32_t* wm, uint32_t i, const uint8_t* msg, const uint64_t* off,
                                              const uint32_t* len, const uint8_t* dst, uint32_t dl, uint32_t* hrec,
                                              const uint32_t* kmode) {
    const wave::Wave w{wm, (int)threadIdx.x};
    w_hash_to_g1(w, msg + off[i], len[i], dst, dl, hrec + (size_t)G1H_REC_WORDS * i, !(kmode && kmode[i]));
}
// signature decode only (one lane per item); the G1 check runs beside the pairing (k_blsw_pair_sub)
__global__ __launch_bounds__(BLS_LANES) void k_blsw_sigdec(uint32_t n, const uint8_t* sig, uint32_t* rec, int32_t* st) {
    BLS_IDX();
    fp x, y;
    bool inf;
    const int32_t s = g1_decompress(x, y, inf, sig + 48 * (size_t)i);
    if (s != ST_OK || inf) x = y = fp_zero();
    st_g1(rec + (size_t)G1_REC_WORDS * i, x, y, s == ST_OK && inf);
    st[i] = s;
}
__device__ __forceinline__ void blsw_sub_item(uint32_t* wm, uint32_t i, const uint32_t* rec, const int32_t* st_dec,
                                              int32_t* st_sub) {
    const wave::Wave w{wm, (int)threadIdx.x};
    const uint32_t* r = rec + (size_t)G1_REC_WORDS * i;
    int32_t s = ST_OK;
    if (st_dec[i] == ST_OK && !r[2 * NL]) s = w_g1_in_group(w, r) ? ST_OK : ST_NOT_IN_GROUP;
    if (threadIdx.x == 0) st_sub[i] = s;
}
__global__ __launch_bounds__(64) void k_blsw_sub(uint32_t n, const uint32_t* rec, const int32_t* st_dec, int32_t* st_sub) {
    BLSW_IDX();
    blsw_sub_item(wm, i, rec, st_dec, st_sub);
}
// e(-sig, g2) e(H, apk) == 1 for every item whose signature decoded and whose keys are valid
// (run beside the signature's G1 check: the status join puts that check first)
// H: homogeneous records (k_blsw_pre) or affine ones (k_bls_h2c_g, h_hom = 0); apk: Jacobian
// records (k_blsw_apk)
// (a one-key item whose key is in the cache takes the key's precomputed line table: the Miller
// loop then only evaluates lines, no G2 arithmetic)
__device__ __forceinline__ void blsw_pair_item(uint32_t* wm, uint32_t i, const uint32_t* srec, const int32_t* st_dec,
                                               const uint32_t* hrec, int h_hom, const uint32_t* arec,
                                               const int32_t* st_apk, const KeyTab& kt, const uint32_t* pk_off,
                                               const uint32_t* pk_cnt, const uint32_t* pk_idx, const uint32_t* kmode,
                                               int32_t* st_pair) {
    const wave::Wave w{wm, (int)threadIdx.x};
    int32_t s = ST_VERIFY_FAIL;
    if (st_dec[i] == ST_OK && st_apk[i] == ST_OK) {
        const uint32_t* ql = nullptr;
        if (kt.lines && kmode && kmode[i] && pk_cnt[i] == 1) ql = kt.lines + KL_WORDS * pk_idx[pk_off[i]];
        s = w_pairing_check_g(w, srec + (size_t)G1_REC_WORDS * i,
                              hrec + (size_t)(h_hom ? G1H_REC_WORDS : G1_REC_WORDS) * i, h_hom != 0,
                              arec + (size_t)G2J_WORDS * i, true, ql)
                ? ST_OK
                : ST_VERIFY_FAIL;
    }
    if (threadIdx.x == 0) st_pair[i] = s;
}
// The throughput form: up to BLS_PACK_MAX items per wave (wave::WaveK: each item's slots in its
// own LDS bank, the narrow stages of every item in one pass).  e(-sig, g2) e(H, apk) == 1 for each
// item as blsw_pair_item; an item whose signature or keys failed gets VERIFY_FAIL whatever its bank
// computed.  Precomputed key lines are used only when every item of the wave has them (the Miller
// loop's program is one for the wave).
//
// The whole check is one loop over the flat script of wave::pairing_script (g_pair_script, one per
// line mode): the stage loop below is the kernel's only copy of the interpreter and the loop makes
// no calls, so no callee-saved registers go through scratch (round 5's out-of-line wave_run_k
// wrote ~616 KB of scratch per item).  The banks share one P << k table at the front of the LDS
// (9.6 KB a bank instead of 10.5 KB).
constexpr int BLS_PACK_MAX = 4;
__device__ wave::SOp g_pair_script[2][wave::SCRIPT_MAX];  // [fixed key lines]
__device__ int g_pair_script_n[2];
// two waves per SIMD (<= 256 registers: at most 4 terms' LDS reads in flight, NWV_BLS_PAIR_TERMS)
// with three items a wave (NWV_BLS_PACK: 3 x 6.5 KB banks -- registers never live together share
// slots, tools/gen_bls_wave.py PC_ALIAS -- + the shared 0.9 KB table = 8 waves per CU): 16,384
// checks 23.5 -> 16.0 ms against one wave per SIMD with three 10.5 KB banks
// (profiles/round6_bls_pair_sweep.txt)
#ifndef NWV_BLS_PAIR_WAVES
#define NWV_BLS_PAIR_WAVES 2
#endif
#ifndef NWV_BLS_PAIR_TERMS
#define NWV_BLS_PAIR_TERMS 4
#endif
// x / d and x % d for 0 <= x <= 64 and a wave-uniform 1 <= d <= 64 without a division sequence:
// x ceil(2^16 / d) >> 16 is exact there (the error x (ceil(2^16/d) - 2^16/d) / 2^16 < 1/1024 < 1/d)
__constant__ const uint32_t k_div_magic[65] = {0, 65536, 32768, 21846, 16384, 13108, 10923, 9363, 8192, 7282, 6554, 5958, 5462, 5042, 4682, 4370, 4096, 3856, 3641, 3450, 3277, 3121, 2979, 2850, 2731, 2622, 2521, 2428, 2341, 2260, 2185, 2115, 2048, 1986, 1928, 1873, 1821, 1772, 1725, 1681, 1639, 1599, 1561, 1525, 1490, 1457, 1425, 1395, 1366, 1338, 1311, 1286, 1261, 1237, 1214, 1192, 1171, 1150, 1130, 1111, 1093, 1075, 1058, 1041, 1024};  // ceil(2^16 / d)
__device__ __forceinline__ int lane_div(int x, int d) {
    const uint32_t m = k_div_magic[__builtin_amdgcn_readfirstlane(d)];
    return (int)(((uint32_t)x * m) >> 16);
}
__device__ __forceinline__ int lane_mod(int x, int d) { return x - lane_div(x, d) * d; }
// items [i0, i0 + k) on this wave: lds_k = the P << k table, then k banks; G: term reads in flight
template <int G>
__device__ __forceinline__ void pair_flat(uint32_t* lds_k, uint32_t i0, int k, const uint32_t* srec,
                                          const int32_t* st_dec, const uint32_t* hrec, int h_hom,
                                          const uint32_t* arec, const int32_t* st_apk, const KeyTab& kt,
                                          const uint32_t* pk_off, const uint32_t* pk_cnt, const uint32_t* pk_idx,
                                          const uint32_t* kmode, int32_t* st_pair) {
    using namespace wave;
    const int lane = (int)threadIdx.x;
    constexpr uint32_t bankw = (uint32_t)(SW * NSLOTS_PC);
    const WaveK w{lds_k + KP_WORDS, bankw, k, lane};
    const wword* kpt = (const wword*)lds_k;  // the shared P << k table
    const uint32_t* sig[BLS_PACK_MAX];
    const uint32_t* hr[BLS_PACK_MAX];
    const uint32_t* ql[BLS_PACK_MAX];
    bool fixed = true;
    for (int j = 0; j < k; j++) {
        const uint32_t i = i0 + j;
        sig[j] = srec + (size_t)G1_REC_WORDS * i;
        hr[j] = hrec + (size_t)(h_hom ? G1H_REC_WORDS : G1_REC_WORDS) * i;
        ql[j] = (kt.lines && kmode && kmode[i] && pk_cnt[i] == 1) ? kt.lines + KL_WORDS * pk_idx[pk_off[i]] : nullptr;
        fixed = fixed && ql[j] != nullptr;
    }
    // P << k once, then every bank: slot 0 = 0, the pairing check's constants at slots 1..
    for (int t = lane; t < KP_WORDS; t += 64) lds_k[t] = (&T_KP[0][0])[t];
    for (int j = 0; j < k; j++) {
        if (lane < SW) w.bk(j)[lane] = 0u;
        for (int t = lane; t < SW * NCONSTS_PC; t += 64) w.bk(j)[SW + t] = (&T_CONSTS[0][0])[t];
    }
    w.zero(REG_PA, 2);
    w.zero(REG_PB, 3);
    w.zero(REG_QB, 6);
    w.sync();
    for (int j = 0; j < k; j++) {
        const uint32_t i = i0 + j;
        if (!sig[j][2 * NL]) {
            w.put_words(j, REG_PA, sig[j], 1);
            w.put_fp(j, REG_PA + 1, fp_neg(ld_fp(sig[j] + NL)));
        }
        const bool h_inf = hr[j][(h_hom ? 3 : 2) * NL] != 0;
        if (!h_inf) w.put_words(j, REG_PB, hr[j], h_hom ? 3 : 2);
        if (h_inf || !h_hom) w.put_fp(j, REG_PB + 2, k_one());
        w.put_words(j, REG_QB, arec + (size_t)G2J_WORDS * i, 6);
    }
    w.sync();
    // wave::pairing_check's set-up over the k banks
    w.zero(REG_F, 12);
    w.sync();
    w.put_fp(-1, REG_F, k_one());
    w.copy_slots(REG_TB, REG_QB, 6);
    w.sync();
    constexpr int LW = 6 * SW;  // words of a step's line
    // the next step's lines load while this step runs: g2's (every bank) and each item's key lines
    uint32_t la0 = 0, la1 = 0, lb0[BLS_PACK_MAX], lb1[BLS_PACK_MAX];
    auto fetch = [&](int st) {
        const uint32_t* g = &T_G2_LINES[st][0][0];
        la0 = lane < LW ? g[lane] : 0u;
        la1 = lane + 64 < LW ? g[lane + 64] : 0u;
        for (int j = 0; j < BLS_PACK_MAX; j++) {
            lb0[j] = 0u;
            lb1[j] = 0u;
            if (j < k && fixed) {
                const uint32_t* q = ql[j] + (size_t)st * LW;
                lb0[j] = lane < LW ? q[lane] : 0u;
                lb1[j] = lane + 64 < LW ? q[lane + 64] : 0u;
            }
        }
    };
    fetch(0);
    const SOp* script = g_pair_script[fixed ? 1 : 0];
    const int nops = g_pair_script_n[fixed ? 1 : 0];
    auto first_rec = [&](const SOp& o) { return load_rec(T_DATA + o.a + (uint32_t)lane_mod(lane, (int)(o.b >> 16)) * REC); };
    Rec cur = first_rec(script[0].c >> 16 == SOP_RUN ? script[0] : script[script[0].next_run]);
    int step = 0;
#pragma unroll 1
    for (int oi = 0; oi < nops; oi++) {
        const SOp op = script[oi];
        const uint32_t kind = op.c >> 16;
        if (kind == SOP_LINES) {
            for (int j = 0; j < k; j++) {
                uint32_t* b = w.bk(j);
                if (lane < LW) b[SW * REG_LA + lane] = la0;
                if (lane + 64 < LW) b[SW * REG_LA + lane + 64] = la1;
                if (fixed) {
                    if (lane < LW) b[SW * REG_LB + lane] = lb0[j];
                    if (lane + 64 < LW) b[SW * REG_LB + lane + 64] = lb1[j];
                }
            }
            w.sync();
            if (step + 1 < NSTEPS) fetch(step + 1);
            step++;
            continue;
        }
        if (kind == SOP_INV) {
            w.invert_slot((int)op.a, (int)op.b);
            w.sync();
            continue;
        }
        // RUN: the program's stages, `reps` times over (wave_run_k's loop, inline: the one copy)
        const uint16_t* base0 = T_DATA + op.a;
        const uint16_t* base = base0;
        const int np = (int)(op.b & 0xffffu), nl0 = (int)(op.b >> 16), total = np * (int)(op.c & 0xffffu);
        int nl = nl0;
#pragma unroll 1
        for (int t = 0, s = 0; t < total; t++) {
            Hdr h = rec_hdr(cur);
            h.nap = __builtin_amdgcn_readfirstlane(h.nap);
            h.nan = __builtin_amdgcn_readfirstlane(h.nan);
            h.nbp = __builtin_amdgcn_readfirstlane(h.nbp);
            h.nbn = __builtin_amdgcn_readfirstlane(h.nbn);
            const bool wrap = s + 1 == np;
            const int nl_next = wrap ? nl0 : __builtin_amdgcn_readfirstlane(h.nl_next);
            const uint16_t* nbase = wrap ? base0 : base + (uint32_t)nl * REC;
            // the next stage's record, or the next RUN op's first one (records are static data)
            Rec nxt = cur;
            if (t + 1 < total) nxt = load_rec(nbase + (uint32_t)lane_mod(lane, nl_next) * REC);
            else if (op.next_run >= 0) nxt = first_rec(script[op.next_run]);
            const int ipp = lane_div(64, nl), first = lane_div(lane, nl);
            if (first < ipp) {
                const uint32_t dst = rec_u16(cur, 0);
#pragma unroll 1
                for (int item = first; item < k; item += ipp) {
                    wword* wm = (wword*)w.bk(item);
                    const fp v = lane_value<G>(wm, kpt, h, cur);
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
    const uint32_t ok = w.f_is_one_mask();
    if (lane == 0)
        for (int j = 0; j < k; j++) {
            const uint32_t i = i0 + j;
            st_pair[i] = (st_dec[i] == ST_OK && st_apk[i] == ST_OK && ((ok >> j) & 1u)) ? ST_OK : ST_VERIFY_FAIL;
        }
}
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NWV_BLS_PAIR_WAVES))) void k_blsw_pair_k(
    uint32_t n, uint32_t kper, const uint32_t* srec, const int32_t* st_dec, const uint32_t* hrec, int h_hom,
    const uint32_t* arec, const int32_t* st_apk, KeyTab kt, const uint32_t* pk_off, const uint32_t* pk_cnt,
    const uint32_t* pk_idx, const uint32_t* kmode, int32_t* st_pair) {
    extern __shared__ uint32_t lds_k[];
    const uint32_t i0 = blockIdx.x * kper;
    if (i0 >= n) return;
    pair_flat<NWV_BLS_PAIR_TERMS>(lds_k, i0, (int)(n - i0 < kper ? n - i0 : kper), srec, st_dec, hrec, h_hom, arec,
                                  st_apk, kt, pk_off, pk_cnt, pk_idx, kmode, st_pair);
}
// the flat scripts into g_pair_script on the calling thread's device, once per device
static int ensure_pair_script() {
    static std::mutex mu;
    static bool done[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return nwv_internal_set_err(NWV_ERR_HIP, "pair script: no device");
    std::lock_guard<std::mutex> g(mu);
    if (done[dev]) return NWV_OK;
    static wave::SOp ops[2][wave::SCRIPT_MAX];
    int cnt[2];
    for (int f = 0; f < 2; f++) cnt[f] = wave::pairing_script(f != 0, ops[f]);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pair_script), ops, sizeof(ops)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_pair_script_n), cnt, sizeof(cnt)) != hipSuccess)
        return nwv_internal_set_err(NWV_ERR_HIP, "pair script copy");
    done[dev] = true;
    return NWV_OK;
}
__global__ __launch_bounds__(64) void k_blsw_pair(uint32_t n, const uint32_t* srec, const int32_t* st_dec,
                                                  const uint32_t* hrec, int h_hom, const uint32_t* arec,
                                                  const int32_t* st_apk, KeyTab kt, const uint32_t* pk_off,
                                                  const uint32_t* pk_cnt, const uint32_t* pk_idx, const uint32_t* kmode,
                                                  int32_t* st_pair) {
    BLSW_LDS(wave::NSLOTS_PAIR2);  // the two-step Miller-loop programs (a key's line table)
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    blsw_pair_item(wm, i, srec, st_dec, hrec, h_hom, arec, st_apk, kt, pk_off, pk_cnt, pk_idx, kmode, st_pair);
}
// the pairing checks (blocks [0, n)) and the signatures' G1 checks (blocks [n, 2n)) as one launch:
// independent waves, so the launch takes as long as the slower of the two per item
__global__ __launch_bounds__(64) void k_blsw_pair_sub(uint32_t n, const uint32_t* srec, const int32_t* st_dec,
                                                      const uint32_t* hrec, int h_hom, const uint32_t* arec,
                                                      const int32_t* st_apk, KeyTab kt, const uint32_t* pk_off,
                                                      const uint32_t* pk_cnt, const uint32_t* pk_idx,
                                                      const uint32_t* kmode, int32_t* st_pair, int32_t* st_sub) {
    BLSW_LDS(wave::NSLOTS_PAIR2);
    const uint32_t b = blockIdx.x;
    if (b < n)
        blsw_pair_item(wm, b, srec, st_dec, hrec, h_hom, arec, st_apk, kt, pk_off, pk_cnt, pk_idx, kmode, st_pair);
    else if (b < 2 * n)
        blsw_sub_item(wm, b - n, srec, st_dec, st_sub);
}
// the same with the pairing on the flat script (pair_flat, one item on the wave); NWV_BLS_SUB_FLAT=1
__global__ __launch_bounds__(64) void k_blsw_pair_sub_f(uint32_t n, const uint32_t* srec, const int32_t* st_dec,
                                                        const uint32_t* hrec, int h_hom, const uint32_t* arec,
                                                        const int32_t* st_apk, KeyTab kt, const uint32_t* pk_off,
                                                        const uint32_t* pk_cnt, const uint32_t* pk_idx,
                                                        const uint32_t* kmode, int32_t* st_pair, int32_t* st_sub) {
    BLSW_LDS(wave::NSLOTS_PAIR2);
    const uint32_t b = blockIdx.x;
    if (b < n)
        pair_flat<8>(wm_lds, b, 1, srec, st_dec, hrec, h_hom, arec, st_apk, kt, pk_off, pk_cnt, pk_idx, kmode, st_pair);
    else if (b < 2 * n)
        blsw_sub_item(wm, b - n, srec, st_dec, st_sub);
}
// [h_eff] pk of newly registered keys (lane per key, affine records): the hash's cofactor clearing
// moves onto the key side -- e(H0, [h_eff] pk) = e([h_eff] H0, pk) for H0 in E(Fp), as the
// reduced pairing sees only H0's G1 component (tests/test_bls_hostemu.py
// test_wave_cofactor_on_key_side) -- so a cached key's item skips the 64-bit G1 chain on H
__global__ __launch_bounds__(BLS_LANES) void k_bls_key_heff(uint32_t n, const uint32_t* slots, const uint32_t* rc,
                                                            uint32_t* hrc) {
    BLS_IDX();
    const uint32_t k = slots[i];
    fp2 x, y;
    ld_g2(rc + (size_t)G2_REC_WORDS * k, x, y);
    g2_to_affine_vt(x, y, jac_mul64(jac_from_affine(x, y), BLS_H_EFF));
    st_g2(hrc + (size_t)G2_REC_WORDS * k, x, y, false);
}
// the line tables of newly registered keys (of their [h_eff] pk): one wave per key (slots[i] = its
// cache slot)
__global__ __launch_bounds__(64) void k_blsw_key_lines(uint32_t n, const uint32_t* slots, const uint32_t* rc,
                                                       uint32_t* lines) {
    BLSW_IDX();
    const uint32_t k = slots[i];
    const wave::Wave w{wm, (int)threadIdx.x};
    w_key_lines(w, rc + (size_t)G2_REC_WORDS * k, lines + KL_WORDS * k);
}
// the key sum of item i on a wave: lane j adds the item's keys j, j + 64, ... (Jacobian, jac_add:
// exact in every case), then a six-level tree through LDS.  The status is that of the item's first
// bad key in list order (else AGGR_MISMATCH for an empty list, PK_INFINITY for an identity sum).
// The sum stays Jacobian (G2J_WORDS record: the Miller-loop programs take a Jacobian Q), so there
// is no inversion; a one-key item copies its validated record with Z = 1.
__device__ __forceinline__ void blsw_apk_item(uint32_t* xa, uint32_t i, const KeyTab& kt, const uint32_t* pk_off,
                                              const uint32_t* pk_cnt, const uint32_t* pk_idx, const uint32_t* kmode,
                                              uint32_t* rec, int32_t* st_apk) {
    const int lane = (int)threadIdx.x;
    const uint32_t cnt = pk_cnt[i];
    const uint32_t* idx = pk_idx + pk_off[i];
    uint32_t* out = rec + (size_t)G2J_WORDS * i;
    // key-side items (every key cached) sum the keys' [h_eff] pk records
    KeyTab kq = kt;
    if (kmode && kmode[i]) kq.rc = kt.hrc;
    if (cnt == 1) {
        const uint32_t k = idx[0];
        const int32_t ks = key_st(kq, k);
        const uint32_t* kr = key_rec(kq, k);
        const fp one = k_one();
        for (int wd = lane; wd < G2J_WORDS; wd += 64) {
            uint32_t v = 0;
            if (wd < 4 * NL) v = ks == ST_OK ? kr[wd] : 0u;
            else if (wd < 5 * NL) v = one.l[wd - 4 * NL];
            else if (wd == 6 * NL) v = ks == ST_OK ? 0u : 1u;
            out[wd] = v;
        }
        if (lane == 0) st_apk[i] = ks;
        return;
    }
    jac<fp2> acc;
    acc.inf = true;
    acc.x = acc.y = acc.z = f2_zero();
    uint32_t first_bad = 0xffffffffu;
    for (uint32_t j = (uint32_t)lane; j < cnt; j += 64) {
        const uint32_t k = idx[j];
        if (key_st(kq, k) != ST_OK) {
            first_bad = j;
            break;
        }
        fp2 x, y;
        ld_g2(key_rec(kq, k), x, y);
        acc = jac_add(acc, jac_from_affine(x, y));
    }
    for (int m = 32; m >= 1; m >>= 1) first_bad = min(first_bad, (uint32_t)__shfl_xor((int)first_bad, m));
#pragma unroll 1
    for (int h = 32; h >= 1; h >>= 1) {
        __syncthreads();
        if (lane >= h && lane < 2 * h) st_g2j(xa + (lane - h) * G2J_WORDS, acc);
        __syncthreads();
        if (lane < h) acc = jac_add(acc, ld_g2j(xa + lane * G2J_WORDS));
    }
    if (lane != 0) return;
    int32_t status = ST_OK;
    if (cnt == 0) status = ST_AGGR_MISMATCH;
    else if (first_bad != 0xffffffffu) status = key_st(kq, idx[first_bad]);
    else if (acc.inf) status = ST_PK_INFINITY;
    if (status != ST_OK) {
        acc.inf = true;
        acc.x = acc.y = acc.z = f2_zero();
    }
    st_g2j(out, acc);
    st_apk[i] = status;
}
__global__ __launch_bounds__(64) void k_blsw_apk(uint32_t n, KeyTab kt, const uint32_t* pk_off, const uint32_t* pk_cnt,
                                                 const uint32_t* pk_idx, const uint32_t* kmode, uint32_t* rec,
                                                 int32_t* st_apk) {
    __shared__ uint32_t xa[32 * G2J_WORDS];
    if (blockIdx.x >= n) return;
    blsw_apk_item(xa, blockIdx.x, kt, pk_off, pk_cnt, pk_idx, kmode, rec, st_apk);
}
// hash to G1 (blocks [0, n)) and the key sums (blocks [n, 2n)) as one launch (one stream per
// call side): independent waves, the LDS of the larger of the two
__global__ __launch_bounds__(64) void k_blsw_pre(uint32_t n, const uint8_t* msg, const uint64_t* off,
                                                 const uint32_t* len, const uint8_t* dst, uint32_t dl, uint32_t* hrec,
                                                 KeyTab kt, const uint32_t* pk_off, const uint32_t* pk_cnt,
                                                 const uint32_t* pk_idx, const uint32_t* kmode, uint32_t* arec,
                                                 int32_t* st_apk) {
    constexpr int LW = wave::WM_WORDS > 32 * G2J_WORDS ? wave::WM_WORDS : 32 * G2J_WORDS;
    __shared__ uint32_t lds[LW];
    const uint32_t b = blockIdx.x;
    if (b < n)
        blsw_h2c_item(lds + wave::KP_WORDS, b, msg, off, len, dst, dl, hrec, kmode);
    else if (b < 2 * n)
        blsw_apk_item(lds, b - n, kt, pk_off, pk_cnt, pk_idx, kmode, arec, st_apk);
}

// AggregateAuthenticator::aggregate (types/src/primary.rs:476-477) on the wave engine: a wave adds
// up to 16 points with the smallest g1_sum program that holds them (2, 4, 8, 16 inputs: one level
// of complete additions, about three stages, per doubling).  The inputs (w_g1_sum_put's forms:
// affine records, optionally through a list of positions, or partial sums) are fetched in one
// batch -- every lane issues all its loads before any is stored -- rather than point by point.
// points [first, first + k) of the input (k <= G1SUM_N; those at or past m are the identity)
__device__ __forceinline__ void blsw_sum_load(uint32_t* wm, const uint32_t* in, const uint32_t* idx, int hom,
                                              uint32_t first, uint32_t m, uint32_t k) {
    using namespace wave;
    const int lane = (int)threadIdx.x;
    constexpr int PW = 3 * NL, T = (G1SUM_N * PW + 63) / 64;
    static_assert(T <= 32, "one mask bit per word");
    const int tot = (int)k * PW;
    init_slots(Wave{wm, lane});
    uint32_t v[T], one_at = 0;
#pragma unroll
    for (int t = 0; t < T; t++) {
        const int wd = lane + 64 * t, q = wd / PW, c = (wd % PW) / NL, l = wd % NL;
        const uint32_t j = first + (uint32_t)q;
        uint32_t x = 0;
        bool one = false;
        if (wd < tot) {
            if (j >= m) {
                one = c == 1;  // the identity (0 : 1 : 0)
            } else if (hom) {
                x = in[(size_t)PW * j + (wd % PW)];
            } else {
                const uint32_t* r = in + (size_t)G1_REC_WORDS * (idx ? idx[j] : j);
                if (r[2 * NL]) one = c == 1;
                else if (c < 2) x = r[c * NL + l];
                else one = true;
            }
        }
        v[t] = x;
        one_at |= (one ? 1u : 0u) << t;
    }
#pragma unroll
    for (int t = 0; t < T; t++) {
        const int wd = lane + 64 * t;
        if (wd < tot)
            wm[SW * g1sum_slot(wd / PW) + (wd % PW)] = (one_at >> t) & 1u ? wm[SW * SLOT_ONE + wd % NL] : v[t];
    }
    wsync();
}
// block b: points [b per, b per + per) (per <= G1SUM_N) -> partial sum b
__global__ __launch_bounds__(64) void k_blsw_g1_sum(uint32_t m, const uint32_t* in, const uint32_t* idx, int hom,
                                                    uint32_t* part, uint32_t per) {
    BLSW_LDS(wave::NSLOTS);
    const uint32_t first = blockIdx.x * per;
    if (first >= m) return;
    const uint32_t cnt = min(per, m - first);
    blsw_sum_load(wm, in, idx, hom, first, m, g1_sum_width(cnt));
    const wave::Wave w{wm, (int)threadIdx.x};
    w.run(g1_sum_prog(cnt));
    w.get_words(wave::REG_U, part + (size_t)G1P_WORDS * blockIdx.x, 3);
}
// the last level (m <= G1SUM_N inputs, one block): the first bad status of the n_st items in list
// order (st: null when every item is known good), else the compressed sum
__global__ __launch_bounds__(64) void k_blsw_g1_sum_fin(uint32_t m, const uint32_t* in, const uint32_t* idx, int hom,
                                                        uint32_t n_st, const int32_t* st, uint8_t* out48,
                                                        int32_t* out_st) {
    BLSW_LDS(wave::NSLOTS);
    const int lane = (int)threadIdx.x;
    if (blockIdx.x) return;
    if (st) {
        uint32_t bad = 0xffffffffu;
        for (uint32_t k = (uint32_t)lane; k < n_st; k += 64)
            if (st[k] != ST_OK) {
                bad = k;
                break;
            }
        for (int o = 32; o >= 1; o >>= 1) bad = min(bad, (uint32_t)__shfl_xor((int)bad, o));
        if (bad != 0xffffffffu) {
            if (lane == 0) *out_st = st[bad];
            return;
        }
    }
    blsw_sum_load(wm, in, idx, hom, 0, m, g1_sum_width(m));
    const wave::Wave w{wm, lane};
    w.run(g1_sum_prog(m));
    w_g1_sum_compress(w, out48);
    if (lane == 0) *out_st = ST_OK;
}

// the oracle's order: signature decode, its G1 check, the keys, the pairing equation
// (sc_rec: a verified signature's record is also kept in the signature ring, at slot sc_slot[i])
__global__ __launch_bounds__(BLS_LANES) void k_blsw_status(uint32_t n, const int32_t* dec, const int32_t* sub,
                                                           const int32_t* apk, const int32_t* pair, int32_t* st,
                                                           const uint32_t* srec, uint32_t* sc_rec, const uint32_t* sc_slot) {
    BLS_IDX();
    const int32_t s = dec[i] != ST_OK ? dec[i] : sub[i] != ST_OK ? sub[i] : apk[i] != ST_OK ? apk[i] : pair[i];
    st[i] = s;
    if (sc_rec && s == ST_OK) {
        uint32_t* d = sc_rec + (size_t)G1_REC_WORDS * sc_slot[i];
        const uint32_t* r = srec + (size_t)G1_REC_WORDS * i;
        for (int k = 0; k < G1_REC_WORDS; k++) d[k] = r[k];
    }
}

// ------------------------------------------------------------------------------- host side
namespace {

#define BLS_HIP(x)                                                                  \
    do {                                                                            \
        const hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) return nwv_internal_set_err(NWV_ERR_HIP, hipGetErrorString(e_)); \
    } while (0)

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return NWV_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, n) != hipSuccess) return nwv_internal_set_err(NWV_ERR_OOM, "hipMalloc (bls)");
        cap = n;
        return NWV_OK;
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return NWV_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess)
            return nwv_internal_set_err(NWV_ERR_OOM, "hipHostMalloc (bls)");
        cap = n;
        return NWV_OK;
    }
    ~HBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// The committee key cache of a device.  fastcrypto validates a BLS public key once, when it is
// deserialized; here nwv_bls_keycache_register (epoch start: the committee's keys) decodes and
// subgroup-checks keys once and keeps the records of the VALID ones.  Verification calls only look
// keys up: a key the cache does not hold (a stray key, a single verify by an outsider, an invalid
// key) is decoded into the call's own scratch table and never takes a slot.  Slots are published
// only after the fill kernel has completed; reset (epoch change) waits for calls in flight, which
// hold the lock shared while their kernels read the records.
struct BlsKeyCache {
    std::shared_mutex mu;
    DBuf rec, st;  // KC_CAP x G2_REC_WORDS u32 records, KC_CAP int32 statuses
    DBuf hrec;     // KC_CAP x G2_REC_WORDS: [h_eff] pk of each slot
    DBuf lines;    // line tables of slots [0, used): KL_WORDS u32 each (grown as keys register)
    uint32_t lines_slots = 0;
    std::unordered_map<std::string, uint32_t> slot;
    uint32_t used = 0;
};

// One call in flight: its streams, staging arena and scratch.  A device keeps a pool of these, so
// concurrent callers run their pipelines side by side instead of queueing on one device lock.
struct BlsLane {
    hipStream_t stream = nullptr;              // H2D, signatures, pairing check, D2H
    hipStream_t side[2] = {nullptr, nullptr};  // keys + key sums (+ hash to G1 on small wave calls); hash to G1
    HBuf stage;
    DBuf in, work;
    // [0,1] keys, [1,2] key sums (side 0); [3,4] signatures (main); [5,6] hash to G1 (side 1; side
    // 0 on small wave calls); [7,8] pairing check (main); [9] inputs resident, [10] side 0 done,
    // [11] side 1 done.  side[1] is created by the first call that needs it: a lane of small wave
    // calls holds two streams, so eight lanes map one to one onto 16 hardware queues
    hipEvent_t ev[12] = {};
    // ordering only (no timestamps): [0] inputs resident, [1] signatures decoded (small wave calls)
    hipEvent_t sev[2] = {};
    ~BlsLane() {
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : sev)
            if (e) (void)hipEventDestroy(e);
        for (auto& t : side)
            if (t) (void)hipStreamDestroy(t);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// Signatures that passed a wave-path verify call of up to wave_max items, kept decoded (affine G1
// records) by their 48 bytes: AggregateAuthenticator::aggregate over votes the Core has already
// verified (primary/src/aggregators.rs VotesAggregator::append -> types/src/primary.rs:476) then
// sums kept records instead of decoding and G1-checking each signature again.  A ring of SC_CAP
// records: a verify call reserves n slots (unmapping what they held) under the unique lock before
// its kernels run, k_blsw_status writes the verified records into them, and the call maps them
// after its stream synchronises.  A reserved slot stays `busy` until its call maps or releases
// it, and the cursor steps over busy slots, so no two calls in flight ever write one slot.  An
// aggregate holds the shared lock from its lookups until its stream synchronises, so no slot it
// reads is reserved while its kernels run.
struct Sig48 {
    uint8_t b[48];
    bool operator==(const Sig48& o) const { return std::memcmp(b, o.b, 48) == 0; }
};
struct Sig48Hash {
    size_t operator()(const Sig48& s) const {  // the x coordinate's low 64 bits (big-endian bytes 40..47)
        uint64_t h;
        std::memcpy(&h, s.b + 40, 8);
        return (size_t)(h * 0x9e3779b97f4a7c15ull);
    }
};
struct BlsSigCache {
    std::shared_mutex mu;
    DBuf rec;  // SC_CAP x G1_REC_WORDS
    std::unordered_map<Sig48, uint32_t, Sig48Hash> slot;
    std::vector<Sig48> key;     // the signature slot s holds (when held[s])
    std::vector<uint8_t> held;  // slot s is mapped
    std::vector<uint8_t> busy;  // reserved by a call still in flight
    uint32_t next = 0;
    // n free slots from the ring's cursor (busy ones skipped: at most kMaxLanes x 1,024 are),
    // unmapped and marked busy -> out
    int reserve(size_t n, std::vector<uint32_t>& out) {
        std::unique_lock<std::shared_mutex> lk(mu);
        if (!rec.p) {
            int rc = rec.ensure((size_t)4 * G1_REC_WORDS * SC_CAP);
            if (rc) return rc;
            key.resize(SC_CAP);
            held.assign(SC_CAP, 0);
            busy.assign(SC_CAP, 0);
            slot.reserve(SC_CAP);
        }
        out.clear();
        for (size_t i = 0; i < n; i++) {
            uint32_t t = next, seen = 0;
            while (busy[t] && ++seen < SC_CAP) t = (t + 1) % SC_CAP;
            if (busy[t]) {  // only after failed calls abandoned their slots (SigSlots)
                for (uint32_t u : out) busy[u] = 0;
                out.clear();
                return nwv_internal_set_err(NWV_ERR_HIP, "bls signature ring: no free slot");
            }
            if (held[t]) {
                auto it = slot.find(key[t]);
                if (it != slot.end() && it->second == t) slot.erase(it);
                held[t] = 0;
            }
            busy[t] = 1;
            out.push_back(t);
            next = (t + 1) % SC_CAP;
        }
        return NWV_OK;
    }
    // the call's verified signatures (status OK) mapped to their slots (status null: the call
    // failed, its slots are only released)
    void publish(size_t n, const uint8_t* sigs, const int32_t* status, const std::vector<uint32_t>& slots) {
        std::unique_lock<std::shared_mutex> lk(mu);
        for (size_t i = 0; i < slots.size() && i < n; i++) {
            const uint32_t t = slots[i];
            busy[t] = 0;
            if (!status || status[i] != ST_OK) continue;
            std::memcpy(key[t].b, sigs + 48 * i, 48);
            held[t] = 1;
            slot[key[t]] = t;
        }
    }
};
// a call's reserved ring slots, released unless the call publishes them.  A call that fails
// after its kernels were queued may still have k_blsw_status writing into them: the release
// first waits for the call's stream, and if that wait fails too the slots stay busy (abandoned)
// so no other call can ever map a slot a late write may still land in.
struct SigSlots {
    BlsSigCache* sc = nullptr;
    std::vector<uint32_t> slots;
    size_t n = 0;
    hipStream_t stream = nullptr;  // the stream k_blsw_status writes the slots on
    ~SigSlots() {
        if (!sc) return;
        if (stream && hipStreamSynchronize(stream) != hipSuccess) return;  // abandoned, see above
        sc->publish(n, nullptr, nullptr, slots);
    }
};

constexpr size_t kMaxLanes = 8;

struct BlsDev {
    int ordinal = -1;
    uint32_t flags = 0;  // the context's nwv_init flags
    BlsKeyCache kc;
    BlsSigCache sc;
    std::mutex pool_mu;
    std::condition_variable pool_cv;
    std::vector<std::unique_ptr<BlsLane>> lanes;
    std::vector<BlsLane*> idle;
    std::mutex stat_mu;  // the last completed verify_many call's stage times and path
    double last_ms[5] = {0, 0, 0, 0, 0};
    int last_path = 0;
    uint64_t last_keys[2] = {0, 0};  // key-list entries found in the cache, distinct keys decoded
};
// the BLS engine's state of one context: one BlsDev per device of the context (nwv_init with
// several devices shards nwv_bls_verify_many by item index, bls_shard.h).  Diagnostic / test hook:
// env NWV_BLS_DEVICE_REPLICAS=r gives every device r independent BlsDev shards (own key cache,
// ring and lanes), so the split, the per-shard key registration and the status merge run on a
// one-GPU box too.
struct BlsCtx {
    std::vector<BlsDev*> devs;
};
std::mutex g_mu;
std::unordered_map<nwv_ctx*, BlsCtx*> g_devs;

int ctx_of(nwv_ctx* ctx, BlsCtx** out) {
    if (!ctx) return nwv_internal_set_err(NWV_ERR_ARG, "null context");
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_devs.find(ctx);
    if (it != g_devs.end()) {
        *out = it->second;
        return NWV_OK;
    }
    const int nd = nwv_device_count(ctx);
    if (nd <= 0 || nwv_device_ordinal(ctx, 0) < 0) return nwv_internal_set_err(NWV_ERR_NODEV, "context has no device");
    static const int replicas = [] {
        const char* e = std::getenv("NWV_BLS_DEVICE_REPLICAS");
        const int r = e ? std::atoi(e) : 1;
        return r < 1 ? 1 : (r > 8 ? 8 : r);
    }();
    auto* c = new BlsCtx;
    for (int k = 0; k < nd; k++)
        for (int r = 0; r < replicas; r++) {
            auto* d = new BlsDev;
            d->ordinal = nwv_device_ordinal(ctx, k);
            d->flags = nwv_internal_ctx_flags(ctx);
            c->devs.push_back(d);
        }
    g_devs[ctx] = c;
    *out = c;
    return NWV_OK;
}

// the context's first device (single-device entry points: aggregate, keygen, sign, hash, pairing)
int dev_of(nwv_ctx* ctx, BlsDev** out) {
    BlsCtx* c;
    int rc = ctx_of(ctx, &c);
    if (rc) return rc;
    *out = c->devs[0];
    return NWV_OK;
}

// fn(dev) on every device of the context (one host thread each), first nonzero rc in device order
template <class Fn>
int on_all_devices(BlsCtx& c, Fn fn) {
    std::vector<std::pair<size_t, size_t>> r;
    for (size_t k = 0; k < c.devs.size(); k++) r.push_back({k, k + 1});
    std::vector<std::string> err(c.devs.size());
    const int rc = bls_for_ranges(r, [&](size_t k, size_t, size_t) {
        const int e = fn(*c.devs[k]);
        if (e) err[k] = nwv_last_error();
        return e;
    });
    if (rc)
        for (size_t k = 0; k < err.size(); k++)
            if (!err[k].empty()) return nwv_internal_set_err(rc, err[k].c_str());
    return rc;
}

// a lane of the device's pool for the duration of one call (created on demand, at most kMaxLanes)
class LaneLease {
  public:
    explicit LaneLease(BlsDev& d) : d_(d) {
        std::unique_lock<std::mutex> g(d.pool_mu);
        for (;;) {
            if (!d.idle.empty()) {
                lane_ = d.idle.back();
                d.idle.pop_back();
                break;
            }
            if (d.lanes.size() < kMaxLanes) {
                auto l = std::make_unique<BlsLane>();
                if (hipSetDevice(d.ordinal) != hipSuccess ||
                    hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking) != hipSuccess ||
                    hipStreamCreateWithFlags(&l->side[0], hipStreamNonBlocking) != hipSuccess) {
                    rc_ = nwv_internal_set_err(NWV_ERR_HIP, "bls stream");
                    return;
                }
                for (auto& e : l->ev)
                    if (hipEventCreate(&e) != hipSuccess) {
                        rc_ = nwv_internal_set_err(NWV_ERR_HIP, "bls event");
                        return;
                    }
                for (auto& e : l->sev)
                    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                        rc_ = nwv_internal_set_err(NWV_ERR_HIP, "bls event");
                        return;
                    }
                lane_ = l.get();
                d.lanes.push_back(std::move(l));
                break;
            }
            d.pool_cv.wait(g);
        }
        if (hipSetDevice(d.ordinal) != hipSuccess) rc_ = nwv_internal_set_err(NWV_ERR_HIP, "hipSetDevice (bls)");
    }
    ~LaneLease() {
        if (!lane_) return;
        std::lock_guard<std::mutex> g(d_.pool_mu);
        d_.idle.push_back(lane_);
        d_.pool_cv.notify_one();
    }
    int rc() const { return rc_; }
    BlsLane& operator*() { return *lane_; }
    BlsLane* operator->() { return lane_; }

  private:
    BlsDev& d_;
    BlsLane* lane_ = nullptr;
    int rc_ = NWV_OK;
};

// an arena of sections placed 256-byte aligned, filled on the host, copied with one H2D
struct Arena {
    std::vector<std::pair<const void*, size_t>> parts;
    std::vector<size_t> offs;
    size_t total = 0;
    size_t add(const void* p, size_t n) {
        const size_t o = total;
        parts.push_back({p, n});
        offs.push_back(o);
        total += (n + 255) & ~(size_t)255;
        return o;
    }
};

constexpr int kBlocks(size_t n) { return (int)((n + BLS_LANES - 1) / BLS_LANES); }
// blocks of the group kernels: 8 items per 64-lane block
constexpr int gBlocks(size_t n) { return (int)((n + BLS_LANES / GRP - 1) / (BLS_LANES / GRP)); }
size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Key registration: the keys the cache does not hold are decoded and subgroup-checked into a
// scratch table, then (after the stream has completed) the valid ones are copied into fresh
// slots and published.  Invalid keys take no slot; a failure publishes nothing.
int keycache_register(BlsDev& d, size_t n_keys, const uint8_t* keys) {
    if (d.flags & NWV_FLAG_NO_KEYCACHE) return NWV_OK;
    {  // fast path: every key already held
        std::shared_lock<std::shared_mutex> g(d.kc.mu);
        bool all = d.kc.rec.p != nullptr;
        for (size_t j = 0; j < n_keys && all; j++)
            all = d.kc.slot.count(std::string(reinterpret_cast<const char*>(keys + 96 * j), 96)) != 0;
        if (all) return NWV_OK;
    }
    LaneLease lane(d);
    if (lane.rc()) return lane.rc();
    std::unique_lock<std::shared_mutex> g(d.kc.mu);
    int rc;
    if ((rc = d.kc.rec.ensure((size_t)4 * G2_REC_WORDS * KC_CAP)) || (rc = d.kc.st.ensure((size_t)4 * KC_CAP)) ||
        (rc = d.kc.hrec.ensure((size_t)4 * G2_REC_WORDS * KC_CAP)))
        return rc;
    std::vector<std::string> fresh;
    std::vector<uint8_t> fk;
    std::unordered_map<std::string, uint32_t> seen;
    for (size_t j = 0; j < n_keys; j++) {
        std::string kb(reinterpret_cast<const char*>(keys + 96 * j), 96);
        if (d.kc.slot.count(kb) || seen.count(kb)) continue;
        seen.emplace(kb, (uint32_t)fresh.size());
        fresh.push_back(kb);
        fk.insert(fk.end(), keys + 96 * j, keys + 96 * (j + 1));
    }
    const size_t m = fresh.size();
    if (m == 0) return NWV_OK;
    // scratch: keys, identity slot list, records, statuses; then the copy lists
    const size_t o_keys = 0, o_slot = al256(96 * m), o_rec = al256(o_slot + 4 * m),
                 o_st = al256(o_rec + 4 * G2_REC_WORDS * m), o_src = al256(o_st + 4 * m), o_dst = al256(o_src + 4 * m),
                 o_end = o_dst + 4 * m;
    if ((rc = lane->work.ensure(o_end)) || (rc = lane->stage.ensure(o_end))) return rc;
    uint8_t* w = static_cast<uint8_t*>(lane->work.p);
    uint8_t* h = static_cast<uint8_t*>(lane->stage.p);
    std::memcpy(h + o_keys, fk.data(), 96 * m);
    auto* hs = reinterpret_cast<uint32_t*>(h + o_slot);
    for (size_t j = 0; j < m; j++) hs[j] = (uint32_t)j;
    BLS_HIP(hipMemcpyAsync(w, h, o_rec, hipMemcpyHostToDevice, lane->stream));
    hipLaunchKernelGGL(k_bls_keys_fill, dim3(kBlocks(m)), dim3(BLS_LANES), 0, lane->stream, (uint32_t)m, w + o_keys,
                       reinterpret_cast<const uint32_t*>(w + o_slot), reinterpret_cast<uint32_t*>(w + o_rec),
                       reinterpret_cast<int32_t*>(w + o_st));
    BLS_HIP(hipGetLastError());
    BLS_HIP(hipMemcpyAsync(h + o_st, w + o_st, 4 * m, hipMemcpyDeviceToHost, lane->stream));
    BLS_HIP(hipStreamSynchronize(lane->stream));
    const auto* kst = reinterpret_cast<const int32_t*>(h + o_st);
    auto* src = reinterpret_cast<uint32_t*>(h + o_src);
    auto* dst = reinterpret_cast<uint32_t*>(h + o_dst);
    size_t nv = 0;
    for (size_t j = 0; j < m && d.kc.used + nv < KC_CAP; j++)
        if (kst[j] == ST_OK) {
            src[nv] = (uint32_t)j;
            dst[nv] = d.kc.used + (uint32_t)nv;
            nv++;
        }
    if (nv == 0) return NWV_OK;
    BLS_HIP(hipMemcpyAsync(w + o_src, h + o_src, o_end - o_src, hipMemcpyHostToDevice, lane->stream));
    hipLaunchKernelGGL(k_bls_rec_copy, dim3(kBlocks(nv * G2_REC_WORDS)), dim3(BLS_LANES), 0, lane->stream,
                       (uint32_t)nv, reinterpret_cast<const uint32_t*>(w + o_src),
                       reinterpret_cast<const uint32_t*>(w + o_dst), reinterpret_cast<const uint32_t*>(w + o_rec),
                       static_cast<uint32_t*>(d.kc.rec.p), static_cast<int32_t*>(d.kc.st.p));
    BLS_HIP(hipGetLastError());
    // the new slots' Miller-loop line tables (the table grows by whole copies: registration is rare)
    const uint32_t need = d.kc.used + (uint32_t)nv;
    if (need > d.kc.lines_slots) {
        uint32_t cap = std::max<uint32_t>(need, std::max<uint32_t>(2 * d.kc.lines_slots, 256u));
        cap = std::min<uint32_t>(cap, (uint32_t)KC_CAP);
        DBuf nb;
        if ((rc = nb.ensure(4 * KL_WORDS * cap))) return rc;
        if (d.kc.used)
            BLS_HIP(hipMemcpyAsync(nb.p, d.kc.lines.p, 4 * KL_WORDS * d.kc.used, hipMemcpyDeviceToDevice,
                                   lane->stream));
        BLS_HIP(hipStreamSynchronize(lane->stream));
        std::swap(d.kc.lines.p, nb.p);
        std::swap(d.kc.lines.cap, nb.cap);
        d.kc.lines_slots = cap;
    }
    hipLaunchKernelGGL(k_bls_key_heff, dim3(kBlocks(nv)), dim3(BLS_LANES), 0, lane->stream, (uint32_t)nv,
                       reinterpret_cast<const uint32_t*>(w + o_dst), static_cast<const uint32_t*>(d.kc.rec.p),
                       static_cast<uint32_t*>(d.kc.hrec.p));
    hipLaunchKernelGGL(k_blsw_key_lines, dim3((unsigned)nv), dim3(64), 0, lane->stream, (uint32_t)nv,
                       reinterpret_cast<const uint32_t*>(w + o_dst), static_cast<const uint32_t*>(d.kc.hrec.p),
                       static_cast<uint32_t*>(d.kc.lines.p));
    BLS_HIP(hipGetLastError());
    BLS_HIP(hipStreamSynchronize(lane->stream));
    for (size_t k = 0; k < nv; k++) d.kc.slot.emplace(fresh[src[k]], dst[k]);  // published after the copy
    d.kc.used += (uint32_t)nv;
    return NWV_OK;
}

// the whole verify_many pipeline on one lane of a device: after one H2D copy, three streams --
//   side 0: the call's keys the cache does not hold, decoded into the scratch table
//           (k_bls_keys_fill), then the key sums (k_bls_apk_g)
//   main  : signature decode + G1 checks (k_bls_sigs)
//   side 1: hash to G1 (k_bls_h2c_g)
// -- then, joined on the main stream, the statuses in the oracle's order and the pairing check
int verify_on(BlsDev& d, size_t n_keys, const uint8_t* keys, size_t n, const uint8_t* sigs, const uint32_t* pk_off,
              const uint32_t* pk_cnt, const uint32_t* pk_idx, size_t n_idx, const uint8_t* msg_base,
              const uint64_t* msg_off, const uint32_t* msg_len, size_t msg_bytes, const uint8_t* dst, size_t dl,
              int32_t* status) {
    LaneLease lane(d);
    if (lane.rc()) return lane.rc();
    BlsLane& L = *lane;
    static const uint8_t zero[8] = {0};
    // pairing-check mode: the wave engine per item (default), or the 8-lane group kernels -- one
    // random-linear-combination batch check (NWV_FLAG_BLS_BATCH) or per item (NWV_FLAG_BLS_PER_ITEM)
    const bool group_item = (d.flags & NWV_FLAG_BLS_PER_ITEM) != 0;
    const bool batch = !group_item && (d.flags & NWV_FLAG_BLS_BATCH) != 0;
    const bool wavem = !group_item && !batch;
    // wave-per-item hashing and G1 checks while the call has fewer items than the chip has SIMDs
    // (latency); above that, one item per lane keeps every lane busy (throughput)
    static const size_t wave_max = [] {
        const char* e = std::getenv("NWV_BLS_WAVE_MAX");
        return e ? (size_t)std::strtoul(e, nullptr, 10) : (size_t)1024;
    }();
    const bool wave_small = wavem && n <= wave_max;
    int rc;
    // the call's key table: cache slots (lookups only) or scratch entries KC_CAP + j
    std::shared_lock<std::shared_mutex> kc_hold(d.kc.mu);  // records stay put while our kernels read them
    const bool cached = !(d.flags & NWV_FLAG_NO_KEYCACHE) && d.kc.rec.p != nullptr;
    std::vector<uint32_t> ktab(n_keys), fill_slot;
    std::vector<uint8_t> fill_keys;
    uint64_t hits = 0;
    {
        std::unordered_map<std::string, uint32_t> fresh;
        for (size_t j = 0; j < n_keys; j++) {
            std::string kb(reinterpret_cast<const char*>(keys + 96 * j), 96);
            if (cached) {
                auto it = d.kc.slot.find(kb);
                if (it != d.kc.slot.end()) {
                    ktab[j] = it->second;
                    hits++;
                    continue;
                }
            }
            auto f = fresh.find(kb);
            if (f != fresh.end()) {
                ktab[j] = KC_CAP + f->second;
                continue;
            }
            const uint32_t e = (uint32_t)fresh.size();
            fresh.emplace(std::move(kb), e);
            ktab[j] = KC_CAP + e;
            fill_slot.push_back(e);
            fill_keys.insert(fill_keys.end(), keys + 96 * j, keys + 96 * (j + 1));
        }
    }
    std::vector<uint32_t> remap(n_idx);
    for (size_t t = 0; t < n_idx; t++) remap[t] = ktab[pk_idx[t]];
    // key-side cofactor clearing (wave path): items whose keys are all in the cache use the keys'
    // [h_eff] pk records and line tables, and their hash skips the h_eff chain
    const bool kside = wavem && cached && d.kc.lines_slots;
    std::vector<uint32_t> kmode(kside ? n : 0);
    for (size_t i = 0; i < kmode.size(); i++) {
        bool all = pk_cnt[i] > 0;
        for (uint32_t j = 0; j < pk_cnt[i] && all; j++) all = remap[pk_off[i] + j] < KC_CAP;
        kmode[i] = all ? 1u : 0u;
    }
    const size_t n_dec = fill_slot.size();  // keys decoded by this call
    // verified signatures stay decoded in the device's ring (BlsSigCache) for aggregates
    // (n <= 1,024 whatever NWV_BLS_WAVE_MAX says: kMaxLanes calls hold at most 8,192 busy slots)
    const bool keep = wave_small && n <= 1024 && !(d.flags & NWV_FLAG_NO_SIGCACHE);
    SigSlots kept;
    if (keep) {
        if ((rc = d.sc.reserve(n, kept.slots))) return rc;
        kept.sc = &d.sc;
        kept.n = n;
    }
    uint8_t seed[32];
    nwv_internal_fill_seed(nullptr, seed);  // the batch coefficients' key: OS entropy per call
    Arena a;
    const size_t o_keys = a.add(n_dec ? (const void*)fill_keys.data() : zero, 96 * n_dec + 8),
                 o_kslot = a.add(n_dec ? (const void*)fill_slot.data() : zero, 4 * n_dec + 4),
                 o_sigs = a.add(sigs, 48 * n), o_off = a.add(pk_off, 4 * n), o_cnt = a.add(pk_cnt, 4 * n),
                 o_idx = a.add(n_idx ? (const void*)remap.data() : zero, 4 * n_idx + 4),
                 o_msg = a.add(msg_bytes ? (const void*)msg_base : zero, msg_bytes + 1),
                 o_moff = a.add(msg_off, 8 * n), o_mlen = a.add(msg_len, 4 * n), o_dst = a.add(dst, dl),
                 o_seed = a.add(seed, 32), o_kmode = a.add(kside ? (const void*)kmode.data() : zero, 4 * kmode.size() + 4),
                 o_scs = a.add(keep ? (const void*)kept.slots.data() : zero, 4 * kept.slots.size() + 4);
    if ((rc = L.stage.ensure(al256(a.total) + 64)) || (rc = L.in.ensure(a.total))) return rc;
    uint8_t* h = static_cast<uint8_t*>(L.stage.p);
    for (size_t k = 0; k < a.parts.size(); k++)
        if (a.parts[k].second) std::memcpy(h + a.offs[k], a.parts[k].first, a.parts[k].second);
    // scratch: the call's key records + statuses, item sig / H / apk records, three status arrays,
    // the batch check's shares (W-order Fp12 + Jacobian G1 per item) and its verdict word
    const size_t w_krec = 0, w_kst = w_krec + 4 * G2_REC_WORDS * n_dec, w_srec = al256(w_kst + 4 * n_dec + 4),
                 w_hrec = w_srec + 4 * G1_REC_WORDS * n, w_arec = w_hrec + 4 * G1_REC_WORDS * n,
                 w_st = w_arec + 4 * G2_REC_WORDS * (n + 1), w_ssig = al256(w_st + 4 * n), w_sapk = al256(w_ssig + 4 * n),
                 w_ok = al256(w_sapk + 4 * n), w_frec = al256(w_ok + 4),
                 w_jrec = al256(w_frec + 4 * F12_REC_WORDS * (batch ? n + 1 : 0)),
                 w_prec = al256(w_jrec + 4 * G1J_REC_WORDS * (batch ? n : 0)),
                 w_hh = al256(w_prec + 4 * G1J_REC_WORDS * (batch ? n + 1 : 0) + 4),
                 w_sdec = al256(w_hh + 4 * G1H_REC_WORDS * (wavem ? n : 0)), w_ssub = al256(w_sdec + 4 * n),
                 w_spair = al256(w_ssub + 4 * n), w_aj = al256(w_spair + 4 * n + 4),
                 w_end = w_aj + 4 * G2J_WORDS * (wavem ? n : 0) + 4;
    if ((rc = L.work.ensure(w_end))) return rc;
    uint8_t* in = static_cast<uint8_t*>(L.in.p);
    uint8_t* w = static_cast<uint8_t*>(L.work.p);
    KeyTab kt{cached ? static_cast<const uint32_t*>(d.kc.rec.p) : nullptr,
              cached ? static_cast<const int32_t*>(d.kc.st.p) : nullptr, reinterpret_cast<uint32_t*>(w + w_krec),
              reinterpret_cast<int32_t*>(w + w_kst),
              cached && d.kc.lines_slots ? static_cast<const uint32_t*>(d.kc.lines.p) : nullptr,
              cached ? static_cast<const uint32_t*>(d.kc.hrec.p) : nullptr};
    const uint32_t* km = kside ? reinterpret_cast<const uint32_t*>(in + o_kmode) : nullptr;
    auto* srec = reinterpret_cast<uint32_t*>(w + w_srec);
    auto* hrec = reinterpret_cast<uint32_t*>(w + w_hrec);
    auto* arec = reinterpret_cast<uint32_t*>(w + w_arec);
    auto* st = reinterpret_cast<int32_t*>(w + w_st);
    auto* ssig = reinterpret_cast<int32_t*>(w + w_ssig);
    auto* sapk = reinterpret_cast<int32_t*>(w + w_sapk);
    auto* okw = reinterpret_cast<int32_t*>(w + w_ok);
    auto* frec = reinterpret_cast<uint32_t*>(w + w_frec);
    auto* jrec = reinterpret_cast<uint32_t*>(w + w_jrec);
    auto* prec = reinterpret_cast<uint32_t*>(w + w_prec);
    auto* hh = reinterpret_cast<uint32_t*>(w + w_hh);
    auto* sdec = reinterpret_cast<int32_t*>(w + w_sdec);
    auto* ssub = reinterpret_cast<int32_t*>(w + w_ssub);
    auto* spair = reinterpret_cast<int32_t*>(w + w_spair);
    auto* ajrec = reinterpret_cast<uint32_t*>(w + w_aj);
    hipStream_t s0 = L.stream, s1 = L.side[0], s2 = L.side[1];
    kept.stream = s0;
    // the per-stage timing events of a small call only on a NWV_FLAG_BLS_STAGE_TIMES context: else
    // just the two that order the streams (the others cost a single verification ~0.1 ms:
    // 2.85 -> 2.72-2.81 ms, profiles/round6_bls_stage_timing_ab.json)
    const bool no_timing = !(d.flags & NWV_FLAG_BLS_STAGE_TIMES);
    bool untimed = false;  // a small call that recorded no stage events (set on that path only)
    auto trec = [&](int k, hipStream_t s) { return no_timing ? hipSuccess : hipEventRecord(L.ev[k], s); };
    // stage times of the completed call, its path and key counts -> the device's "last call"
    auto finish = [&](int path_done) -> int {
        const int pairs[5][2] = {{0, 1}, {3, 4}, {5, 6}, {1, 2}, {7, 8}};  // keys, sigs, h2c, apk, pairing
        double ms5[5] = {0, 0, 0, 0, 0};
        for (int k = 0; k < 5 && !untimed; k++) {
            float ms = 0;
            BLS_HIP(hipEventElapsedTime(&ms, L.ev[pairs[k][0]], L.ev[pairs[k][1]]));
            ms5[k] = ms;
        }
        std::lock_guard<std::mutex> g(d.stat_mu);
        std::memcpy(d.last_ms, ms5, sizeof ms5);
        d.last_path = path_done;
        d.last_keys[0] = hits;
        d.last_keys[1] = n_dec;
        return NWV_OK;
    };
    BLS_HIP(nwv_stage::stage_h2d(in, h, a.total, s0));  // small calls: through kernel arguments
    BLS_HIP(hipEventRecord(L.sev[0], s0));
    BLS_HIP(hipStreamWaitEvent(s1, L.sev[0], 0));
    if (wave_small) {
        untimed = no_timing;
        // a call of up to wave_max items on two streams (8 concurrent calls then fit 16 hardware
        // queues one to one): side 0 decodes the keys the cache does not hold, then hashes to G1
        // and sums the keys in one launch (k_blsw_pre); main decodes the signatures, then runs
        // the pairing checks and the signatures' G1 checks in one launch (k_blsw_pair_sub)
        BLS_HIP(trec(0, s1));
        if (n_dec)
            hipLaunchKernelGGL(k_bls_keys_fill, dim3(kBlocks(n_dec)), dim3(BLS_LANES), 0, s1, (uint32_t)n_dec,
                               in + o_keys, reinterpret_cast<const uint32_t*>(in + o_kslot),
                               const_cast<uint32_t*>(kt.rs), const_cast<int32_t*>(kt.ss));
        BLS_HIP(trec(1, s1));
        BLS_HIP(trec(5, s1));
        hipLaunchKernelGGL(k_blsw_pre, dim3((unsigned)(2 * n)), dim3(64), 0, s1, (uint32_t)n, in + o_msg,
                           reinterpret_cast<const uint64_t*>(in + o_moff), reinterpret_cast<const uint32_t*>(in + o_mlen),
                           in + o_dst, (uint32_t)dl, hh, kt, reinterpret_cast<const uint32_t*>(in + o_off),
                           reinterpret_cast<const uint32_t*>(in + o_cnt), reinterpret_cast<const uint32_t*>(in + o_idx),
                           km, ajrec, sapk);
        BLS_HIP(trec(2, s1));
        BLS_HIP(trec(6, s1));
        BLS_HIP(trec(3, s0));
        hipLaunchKernelGGL(k_blsw_sigdec, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n, in + o_sigs, srec,
                           sdec);
        BLS_HIP(trec(4, s0));
        BLS_HIP(hipEventRecord(L.sev[1], s0));
        kept.stream = s1;  // k_blsw_status writes the ring slots there
        // the rest runs on side 0 behind the hash, which ends after the signatures' decode (one
        // lane each, ~0.45 ms against ~0.57 ms): its wait on the decode is already met, so the
        // cross-queue hand-off (~25 us in the single-verify trace) is off the critical path
        BLS_HIP(hipStreamWaitEvent(s1, L.sev[1], 0));
        BLS_HIP(trec(7, s1));
        static const bool sub_flat = [] {
            const char* e = std::getenv("NWV_BLS_SUB_FLAT");
            return e && std::atoi(e) != 0;
        }();
        if (sub_flat && ensure_pair_script()) return NWV_ERR_HIP;
        hipLaunchKernelGGL(sub_flat ? k_blsw_pair_sub_f : k_blsw_pair_sub, dim3((unsigned)(2 * n)), dim3(64), 0, s1,
                           (uint32_t)n,
                           (const uint32_t*)srec, (const int32_t*)sdec, (const uint32_t*)hh, 1, (const uint32_t*)ajrec,
                           (const int32_t*)sapk, kt, reinterpret_cast<const uint32_t*>(in + o_off),
                           reinterpret_cast<const uint32_t*>(in + o_cnt), reinterpret_cast<const uint32_t*>(in + o_idx),
                           km, spair, ssub);
        BLS_HIP(trec(8, s1));
        // (the verified records into the ring slots this call reserved)
        hipLaunchKernelGGL(k_blsw_status, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s1, (uint32_t)n,
                           (const int32_t*)sdec, (const int32_t*)ssub, (const int32_t*)sapk, (const int32_t*)spair, st,
                           (const uint32_t*)srec, keep ? static_cast<uint32_t*>(d.sc.rec.p) : nullptr,
                           reinterpret_cast<const uint32_t*>(in + o_scs));
        BLS_HIP(hipGetLastError());
        BLS_HIP(hipMemcpyAsync(status, st, 4 * n, hipMemcpyDeviceToHost, s1));
        BLS_HIP(hipStreamSynchronize(s1));
        if (keep) {
            d.sc.publish(n, sigs, status, kept.slots);
            kept.sc = nullptr;
        }
        return finish(3);
    }
    if (!L.side[1] && hipStreamCreateWithFlags(&L.side[1], hipStreamNonBlocking) != hipSuccess)
        return nwv_internal_set_err(NWV_ERR_HIP, "bls stream");
    s2 = L.side[1];
    BLS_HIP(hipStreamWaitEvent(s2, L.sev[0], 0));
    // side 0: keys, key sums
    BLS_HIP(hipEventRecord(L.ev[0], s1));
    if (n_dec)
        hipLaunchKernelGGL(k_bls_keys_fill, dim3(kBlocks(n_dec)), dim3(BLS_LANES), 0, s1, (uint32_t)n_dec, in + o_keys,
                           reinterpret_cast<const uint32_t*>(in + o_kslot), const_cast<uint32_t*>(kt.rs),
                           const_cast<int32_t*>(kt.ss));
    BLS_HIP(hipEventRecord(L.ev[1], s1));
    if (wavem)
        hipLaunchKernelGGL(k_blsw_apk, dim3((unsigned)n), dim3(64), 0, s1, (uint32_t)n, kt,
                           reinterpret_cast<const uint32_t*>(in + o_off), reinterpret_cast<const uint32_t*>(in + o_cnt),
                           reinterpret_cast<const uint32_t*>(in + o_idx), km, ajrec, sapk);
    else
        hipLaunchKernelGGL(k_bls_apk_g, dim3(gBlocks(n)), dim3(BLS_LANES), 0, s1, (uint32_t)n, kt,
                           reinterpret_cast<const uint32_t*>(in + o_off), reinterpret_cast<const uint32_t*>(in + o_cnt),
                           reinterpret_cast<const uint32_t*>(in + o_idx), arec, sapk);
    BLS_HIP(hipEventRecord(L.ev[2], s1));
    BLS_HIP(hipEventRecord(L.ev[10], s1));
    // side 1: hash to G1 (every item: the statuses are not known yet)
    BLS_HIP(hipEventRecord(L.ev[5], s2));
    // hash to G1: lane pairs (NWV_BLS_H2C_GROUP=1: the 8-lane group form)
    static const bool h2c_group = [] {
        const char* e = std::getenv("NWV_BLS_H2C_GROUP");
        return e && std::atoi(e) != 0;
    }();
    if (!h2c_group)
        hipLaunchKernelGGL(k_bls_h2c_2, dim3((unsigned)((n + BLS_LANES / 2 - 1) / (BLS_LANES / 2))), dim3(BLS_LANES), 0,
                           s2, (uint32_t)n, in + o_msg, reinterpret_cast<const uint64_t*>(in + o_moff),
                           reinterpret_cast<const uint32_t*>(in + o_mlen), in + o_dst, (uint32_t)dl, hrec, km);
    else
    hipLaunchKernelGGL(k_bls_h2c_g, dim3(gBlocks(n)), dim3(BLS_LANES), 0, s2, (uint32_t)n, in + o_msg,
                       reinterpret_cast<const uint64_t*>(in + o_moff), reinterpret_cast<const uint32_t*>(in + o_mlen),
                       in + o_dst, (uint32_t)dl, hrec, km);
    BLS_HIP(hipEventRecord(L.ev[6], s2));
    BLS_HIP(hipEventRecord(L.ev[11], s2));
    if (wavem) {
        // large wave calls: the one-lane-per-item decode + G1 check of the group path, which keeps
        // every lane busy (an all-Ok subgroup column), then every item's pairing check on a wave
        BLS_HIP(hipEventRecord(L.ev[3], s0));
        hipLaunchKernelGGL(k_bls_sigs, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n, in + o_sigs, srec, sdec);
        BLS_HIP(hipMemsetAsync(ssub, 0, 4 * n, s0));
        BLS_HIP(hipEventRecord(L.ev[4], s0));
        BLS_HIP(hipStreamWaitEvent(s0, L.ev[10], 0));
        BLS_HIP(hipStreamWaitEvent(s0, L.ev[11], 0));
        BLS_HIP(hipEventRecord(L.ev[7], s0));
        // items per pairing wave (env NWV_BLS_PACK, 1..4): one LDS bank of ~6.5 KB each
        static const uint32_t pack = [] {
            const char* e = std::getenv("NWV_BLS_PACK");
            const long v = e ? std::strtol(e, nullptr, 10) : 3;
            return (uint32_t)(v < 1 ? 1 : v > BLS_PACK_MAX ? BLS_PACK_MAX : v);
        }();
        // diagnostic (occupancy experiments): NWV_BLS_LDS_PAD bytes of extra LDS per pairing wave
        static const size_t lds_pad = [] {
            const char* e = std::getenv("NWV_BLS_LDS_PAD");
            return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)0;
        }();
        if (pack > 1 && ensure_pair_script()) return NWV_ERR_HIP;
        if (pack > 1)
            hipLaunchKernelGGL(k_blsw_pair_k, dim3((unsigned)((n + pack - 1) / pack)), dim3(64),
                               (size_t)4 * (wave::KP_WORDS + pack * wave::SW * wave::NSLOTS_PC) + lds_pad, s0,
                               (uint32_t)n, pack, (const uint32_t*)srec, (const int32_t*)sdec, (const uint32_t*)hrec, 0,
                               (const uint32_t*)ajrec, (const int32_t*)sapk, kt,
                               reinterpret_cast<const uint32_t*>(in + o_off), reinterpret_cast<const uint32_t*>(in + o_cnt),
                               reinterpret_cast<const uint32_t*>(in + o_idx), km, spair);
        else
            hipLaunchKernelGGL(k_blsw_pair, dim3((unsigned)n), dim3(64), lds_pad, s0, (uint32_t)n, (const uint32_t*)srec,
                               (const int32_t*)sdec, (const uint32_t*)hrec, 0, (const uint32_t*)ajrec,
                               (const int32_t*)sapk, kt, reinterpret_cast<const uint32_t*>(in + o_off),
                               reinterpret_cast<const uint32_t*>(in + o_cnt), reinterpret_cast<const uint32_t*>(in + o_idx),
                               km, spair);
        BLS_HIP(hipEventRecord(L.ev[8], s0));
        hipLaunchKernelGGL(k_blsw_status, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n,
                           (const int32_t*)sdec, (const int32_t*)ssub, (const int32_t*)sapk, (const int32_t*)spair, st,
                           (const uint32_t*)srec, nullptr, nullptr);
        BLS_HIP(hipGetLastError());
        BLS_HIP(hipMemcpyAsync(status, st, 4 * n, hipMemcpyDeviceToHost, s0));
        BLS_HIP(hipStreamSynchronize(s0));
        return finish(3);
    }
    // main: signatures, then the join
    BLS_HIP(hipEventRecord(L.ev[3], s0));
    hipLaunchKernelGGL(k_bls_sigs, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n, in + o_sigs, srec, ssig);
    BLS_HIP(hipEventRecord(L.ev[4], s0));
    BLS_HIP(hipStreamWaitEvent(s0, L.ev[10], 0));
    BLS_HIP(hipStreamWaitEvent(s0, L.ev[11], 0));
    hipLaunchKernelGGL(k_bls_status, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n, (const int32_t*)ssig,
                       (const int32_t*)sapk, st);
    BLS_HIP(hipEventRecord(L.ev[7], s0));
    auto per_item = [&]() {
        hipLaunchKernelGGL(k_bls_pair, dim3(gBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n, (const uint32_t*)srec,
                           (const uint32_t*)hrec, (const uint32_t*)arec, st);
    };
    int32_t* hst = reinterpret_cast<int32_t*>(h + al256(a.total));  // pinned: the batch verdict word
    int path;
    if (batch) {
        hipLaunchKernelGGL(k_bls_rlc_pts, dim3(gBlocks(n)), dim3(BLS_LANES), 0, s0, (uint32_t)n, (const uint32_t*)srec,
                           (const uint32_t*)hrec, (const int32_t*)st, (const uint8_t*)(in + o_seed), prec, jrec);
        for (uint32_t m = (uint32_t)n; m > 1; m = (m + 1) / 2)
            hipLaunchKernelGGL(k_bls_sfold, dim3(kBlocks(m / 2)), dim3(BLS_LANES), 0, s0, m, jrec);
        hipLaunchKernelGGL(k_bls_sig_item, dim3(1), dim3(BLS_LANES), 0, s0, (uint32_t)n, (const uint32_t*)jrec, prec,
                           arec);
        hipLaunchKernelGGL(k_bls_rlc_ml, dim3(gBlocks(n + 1)), dim3(BLS_LANES), 0, s0, (uint32_t)(n + 1),
                           (const uint32_t*)prec, (const uint32_t*)arec, frec);
        for (uint32_t m = (uint32_t)n + 1; m > 1; m = (m + 1) / 2)
            hipLaunchKernelGGL(k_bls_ffold, dim3(gBlocks(m / 2)), dim3(BLS_LANES), 0, s0, m, frec);
        hipLaunchKernelGGL(k_bls_final, dim3(1), dim3(BLS_LANES), 0, s0, (const uint32_t*)frec, okw);
        BLS_HIP(hipMemcpyAsync(hst, okw, 4, hipMemcpyDeviceToHost, s0));
        BLS_HIP(hipStreamSynchronize(s0));
        BLS_HIP(hipGetLastError());
        path = *hst == 1 ? 1 : 2;
        if (*hst != 1) per_item();  // the batch check rejected: name the failing items exactly
    } else {
        per_item();
        path = 0;
    }
    BLS_HIP(hipEventRecord(L.ev[8], s0));
    BLS_HIP(hipGetLastError());
    BLS_HIP(hipMemcpyAsync(status, st, 4 * n, hipMemcpyDeviceToHost, s0));
    BLS_HIP(hipStreamSynchronize(s0));
    return finish(path);
}

const uint8_t* dst_or_default(const uint8_t* dst, size_t* dl) {
    if (dst) return dst;
    *dl = sizeof(NWV_BLS_DST) - 1;
    return reinterpret_cast<const uint8_t*>(NWV_BLS_DST);
}

}  // namespace

__attribute__((visibility("hidden"))) void nwv_bls_ctx_release(nwv_ctx* ctx) {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_devs.find(ctx);
    if (it == g_devs.end()) return;
    for (BlsDev* d : it->second->devs) {
        (void)hipSetDevice(d->ordinal);
        delete d;
    }
    delete it->second;
    g_devs.erase(it);
}

extern "C" {

int nwv_bls_verify_many(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys, size_t n, const uint8_t* sigs,
                        const uint32_t* pk_off, const uint32_t* pk_cnt, const uint32_t* pk_idx,
                        const uint8_t* msg_base, const uint64_t* msg_off, const uint32_t* msg_len,
                        const uint8_t* dst, size_t dst_len, int32_t* status) {
    if (n == 0) return NWV_OK;
    if (!sigs || !pk_off || !pk_cnt || !msg_off || !msg_len || !status || (n_keys && !keys))
        return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    if (n > (1u << 26) || n_keys > (1u << 26)) return nwv_internal_set_err(NWV_ERR_ARG, "batch too large");
    dst = dst_or_default(dst, &dst_len);
    if (dst_len > 255) return nwv_internal_set_err(NWV_ERR_ARG, "DST longer than 255 bytes");
    // host-side shape checks: every key index and message range in bounds
    size_t n_idx = 0, msg_bytes = 0;
    for (size_t i = 0; i < n; i++) {
        n_idx = std::max<size_t>(n_idx, (size_t)pk_off[i] + pk_cnt[i]);
        if (msg_len[i] && !msg_base) return nwv_internal_set_err(NWV_ERR_ARG, "null msg_base");
        msg_bytes = std::max<size_t>(msg_bytes, msg_off[i] + msg_len[i]);
    }
    if (n_idx && !pk_idx) return nwv_internal_set_err(NWV_ERR_ARG, "null pk_idx");
    for (size_t k = 0; k < n_idx; k++)
        if (pk_idx[k] >= n_keys) return nwv_internal_set_err(NWV_ERR_ARG, "key index out of range");
    BlsCtx* c;
    int rc = ctx_of(ctx, &c);
    if (rc) return rc;
    // items split by index over the context's devices (bls_shard.h); small calls stay on device 0
    static const size_t shard_min = [] {
        const char* e = std::getenv("NWV_BLS_SHARD_MIN");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)256;
    }();
    const auto ranges = bls_shard_ranges(n, c->devs.size(), shard_min);
    if (ranges.size() == 1)
        return verify_on(*c->devs[0], n_keys, keys, n, sigs, pk_off, pk_cnt, pk_idx, n_idx, msg_base, msg_off, msg_len,
                         msg_bytes, dst, dst_len, status);
    std::vector<std::string> err(ranges.size());
    rc = bls_for_ranges(ranges, [&](size_t k, size_t lo, size_t hi) -> int {
        size_t ni = 0, mb = 0;  // the range's own key-index and message extents
        for (size_t i = lo; i < hi; i++) {
            ni = std::max<size_t>(ni, (size_t)pk_off[i] + pk_cnt[i]);
            mb = std::max<size_t>(mb, msg_off[i] + msg_len[i]);
        }
        const int e = verify_on(*c->devs[k], n_keys, keys, hi - lo, sigs + 48 * lo, pk_off + lo, pk_cnt + lo, pk_idx,
                                ni, msg_base, msg_off + lo, msg_len + lo, mb, dst, dst_len, status + lo);
        if (e) err[k] = nwv_last_error();
        return e;
    });
    if (rc)  // the failing range's message, on the caller's thread
        for (size_t k = 0; k < err.size(); k++)
            if (!err[k].empty()) return nwv_internal_set_err(rc, err[k].c_str());
    return rc;
}

int nwv_bls_last_kernel_ms(nwv_ctx* ctx, double out_ms[5]) {
    if (!out_ms) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->stat_mu);
    for (int k = 0; k < 5; k++) out_ms[k] = d->last_ms[k];
    return NWV_OK;
}

int nwv_bls_last_path(nwv_ctx* ctx) {
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->stat_mu);
    return d->last_path;
}

int nwv_bls_last_keys(nwv_ctx* ctx, uint64_t out[2]) {
    if (!out) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->stat_mu);
    out[0] = d->last_keys[0];
    out[1] = d->last_keys[1];
    return NWV_OK;
}

int nwv_bls_keycache_register(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys) {
    if (n_keys && !keys) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    if (n_keys > KC_CAP) return nwv_internal_set_err(NWV_ERR_ARG, "more keys than the cache holds");
    BlsCtx* c;
    int rc = ctx_of(ctx, &c);
    if (rc) return rc;
    // every device verifies its own item range against its own cache
    return n_keys ? on_all_devices(*c, [&](BlsDev& d) { return keycache_register(d, n_keys, keys); }) : NWV_OK;
}

int nwv_bls_keycache_reset(nwv_ctx* ctx) {
    BlsCtx* c;
    int rc = ctx_of(ctx, &c);
    if (rc) return rc;
    for (BlsDev* d : c->devs) {
        std::unique_lock<std::shared_mutex> g(d->kc.mu);  // waits for calls that read the records
        d->kc.slot.clear();
        d->kc.used = 0;
    }
    return NWV_OK;
}

int nwv_bls_keycache_size(nwv_ctx* ctx) {
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::shared_lock<std::shared_mutex> g(d->kc.mu);
    return (int)d->kc.used;
}

int nwv_bls_aggregate_verify(nwv_ctx* ctx, const uint8_t* sig48, const uint8_t* pks, size_t n_pks, const uint8_t* msg,
                             size_t msg_len) {
    if (!sig48) return NWV_ERR_SIGNATURE;  // sig: None
    if ((n_pks && !pks) || (msg_len && !msg)) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    std::vector<uint32_t> idx(n_pks);
    for (size_t k = 0; k < n_pks; k++) idx[k] = (uint32_t)k;
    const uint32_t off = 0, cnt = (uint32_t)n_pks, len = (uint32_t)msg_len;
    const uint64_t moff = 0;
    int32_t st = 0;
    static const uint8_t empty[1] = {0};
    const int rc = nwv_bls_verify_many(ctx, n_pks, pks, 1, sig48, &off, &cnt, idx.data(), msg_len ? msg : empty, &moff,
                                       &len, nullptr, 0, &st);
    if (rc) return rc;
    return st == NWV_BLS_OK ? NWV_OK : NWV_ERR_SIGNATURE;
}

int nwv_bls_verify(nwv_ctx* ctx, const uint8_t pk[96], const uint8_t* msg, size_t msg_len, const uint8_t sig[48]) {
    if (!pk || !sig) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    return nwv_bls_aggregate_verify(ctx, sig, pk, 1, msg, msg_len);
}

int nwv_bls_aggregate(nwv_ctx* ctx, size_t n, const uint8_t* sigs48, uint8_t out48[48], int32_t* status_or_null) {
    if (status_or_null) *status_or_null = NWV_BLS_AGGR_MISMATCH;
    if (n == 0) return NWV_ERR_SIGNATURE;
    if (!sigs48 || !out48) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    if (n > (1u << 26)) return nwv_internal_set_err(NWV_ERR_ARG, "batch too large");
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    LaneLease lane(*d);
    if ((rc = lane.rc())) return rc;
    BlsLane& L = *lane;
    // scratch: records, statuses, the sum tree's two partial-sum levels, the output, decode statuses
    const size_t n_part = (n + wave::G1SUM_N - 1) / wave::G1SUM_N + 1;  // g1_sum_per
    const size_t w_rec = 0, w_st = al256(4 * G1_REC_WORDS * n), w_pa = al256(w_st + 4 * n),
                 w_pb = al256(w_pa + 4 * G1P_WORDS * n_part), w_out = al256(w_pb + 4 * G1P_WORDS * n_part),
                 w_ost = w_out + 64, w_st2 = al256(w_ost + 8), w_end = w_st2 + 4 * n;
    if ((rc = L.in.ensure(48 * n)) || (rc = L.work.ensure(w_end)) || (rc = L.stage.ensure(128))) return rc;
    uint8_t* w = static_cast<uint8_t*>(L.work.p);
    // the sum of the records at `in` (through the positions idx_d when given) as a tree of
    // k_blsw_g1_sum levels; the last (one block) takes the first bad status of st_d when given
    auto sum_tree = [&](const uint32_t* in, const uint32_t* idx_d, const int32_t* st_d) {
        uint32_t m = (uint32_t)n;
        const uint32_t* src = in;
        int hom = 0, flip = 0;
        while (m > (uint32_t)wave::G1SUM_N) {
            const uint32_t per = g1_sum_per(m);
            const uint32_t nb = (m + per - 1) / per;
            auto* dst = reinterpret_cast<uint32_t*>(w + (flip ? w_pb : w_pa));
            hipLaunchKernelGGL(k_blsw_g1_sum, dim3(nb), dim3(64), 0, L.stream, m, src, idx_d, hom, dst, per);
            src = dst;
            idx_d = nullptr;
            hom = 1;
            m = nb;
            flip ^= 1;
        }
        hipLaunchKernelGGL(k_blsw_g1_sum_fin, dim3(1), dim3(64), 0, L.stream, m, src, idx_d, hom,
                           st_d ? (uint32_t)n : 0u, st_d, w + w_out, reinterpret_cast<int32_t*>(w + w_ost));
    };
    auto fetch = [&]() -> int {
        BLS_HIP(hipGetLastError());
        uint8_t* hs = static_cast<uint8_t*>(L.stage.p);
        BLS_HIP(hipMemcpyAsync(hs, w + w_out, 64 + 8, hipMemcpyDeviceToHost, L.stream));
        BLS_HIP(hipStreamSynchronize(L.stream));
        int32_t st;
        std::memcpy(&st, hs + 64, 4);
        if (status_or_null) *status_or_null = st;
        if (st != NWV_BLS_OK) return NWV_ERR_SIGNATURE;
        std::memcpy(out48, hs, 48);
        return NWV_OK;
    };
    // every signature verified by an earlier call: sum the ring's records (no decode, no G1 check)
    if (!(d->flags & NWV_FLAG_NO_SIGCACHE)) {
        std::shared_lock<std::shared_mutex> hold(d->sc.mu);
        if (d->sc.rec.p && n <= SC_CAP) {
            std::vector<uint32_t> pos(n);
            bool all = true;
            Sig48 k;
            for (size_t i = 0; i < n && all; i++) {
                std::memcpy(k.b, sigs48 + 48 * i, 48);
                auto it = d->sc.slot.find(k);
                if (it == d->sc.slot.end()) all = false;
                else pos[i] = it->second;
            }
            if (all) {
                BLS_HIP(nwv_stage::stage_h2d(L.in.p, pos.data(), 4 * n, L.stream));
                sum_tree(static_cast<const uint32_t*>(d->sc.rec.p), static_cast<const uint32_t*>(L.in.p), nullptr);
                return fetch();
            }
        }
    }
    BLS_HIP(nwv_stage::stage_h2d(L.in.p, sigs48, 48 * n, L.stream));
    if (n <= 1024) {  // decode on one lane each, the G1 checks on a wave each
        auto* sdec = reinterpret_cast<int32_t*>(w + w_st2);
        hipLaunchKernelGGL(k_blsw_sigdec, dim3(kBlocks(n)), dim3(BLS_LANES), 0, L.stream, (uint32_t)n,
                           (const uint8_t*)L.in.p, reinterpret_cast<uint32_t*>(w + w_rec), sdec);
        hipLaunchKernelGGL(k_blsw_sub, dim3((unsigned)n), dim3(64), 0, L.stream, (uint32_t)n,
                           reinterpret_cast<const uint32_t*>(w + w_rec), (const int32_t*)sdec,
                           reinterpret_cast<int32_t*>(w + w_st));
        hipLaunchKernelGGL(k_bls_st_join, dim3(kBlocks(n)), dim3(BLS_LANES), 0, L.stream, (uint32_t)n,
                           (const int32_t*)sdec, reinterpret_cast<int32_t*>(w + w_st));
    } else {
        hipLaunchKernelGGL(k_bls_sigs, dim3(kBlocks(n)), dim3(BLS_LANES), 0, L.stream, (uint32_t)n,
                           (const uint8_t*)L.in.p, reinterpret_cast<uint32_t*>(w + w_rec),
                           reinterpret_cast<int32_t*>(w + w_st));
    }
    sum_tree(reinterpret_cast<const uint32_t*>(w + w_rec), nullptr, reinterpret_cast<const int32_t*>(w + w_st));
    return fetch();
}

int nwv_bls_verify_batch_empty_fail(nwv_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* pks,
                                    size_t n_pks, const uint8_t* sigs, size_t n_sigs) {
    if (n_sigs == 0)
        return nwv_internal_set_err(NWV_ERR_EMPTY,
                                    "Critical Error! This behavious can signal something dangerous, and that "
                                    "someone may be trying to bypass signature verification through providing "
                                    "empty batches.");
    if (n_pks != n_sigs)
        return nwv_internal_set_err(NWV_ERR_LENGTH, "Mismatch between number of signatures and public keys provided");
    uint8_t agg[48];
    int rc = nwv_bls_aggregate(ctx, n_sigs, sigs, agg, nullptr);
    if (rc) return rc;
    return nwv_bls_aggregate_verify(ctx, agg, pks, n_pks, msg, msg_len);
}

int nwv_bls_aggregate_batch_verify(nwv_ctx* ctx, size_t n_aggs, const uint8_t* const* sigs48,
                                   const uint8_t* const* pks, const size_t* n_pks, const uint8_t* const* msgs,
                                   const size_t* msg_lens, size_t n_msgs) {
    if (n_aggs != n_msgs) return nwv_internal_set_err(NWV_ERR_LENGTH, "signatures / messages count mismatch");
    if (n_aggs == 0) return NWV_OK;
    if (!sigs48 || !pks || !n_pks || !msgs || !msg_lens) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    std::vector<uint8_t> keys, sg(48 * n_aggs), mb;
    std::vector<uint32_t> off(n_aggs), cnt(n_aggs), idx, len(n_aggs);
    std::vector<uint64_t> moff(n_aggs);
    for (size_t i = 0; i < n_aggs; i++) {
        if (!sigs48[i]) return NWV_ERR_SIGNATURE;  // an aggregate holding no signature
        std::memcpy(sg.data() + 48 * i, sigs48[i], 48);
        off[i] = (uint32_t)idx.size();
        cnt[i] = (uint32_t)n_pks[i];
        for (size_t k = 0; k < n_pks[i]; k++) {
            idx.push_back((uint32_t)(keys.size() / 96));
            keys.insert(keys.end(), pks[i] + 96 * k, pks[i] + 96 * (k + 1));
        }
        moff[i] = mb.size();
        len[i] = (uint32_t)msg_lens[i];
        if (msg_lens[i]) mb.insert(mb.end(), msgs[i], msgs[i] + msg_lens[i]);
    }
    mb.push_back(0);
    std::vector<int32_t> st(n_aggs);
    const int rc = nwv_bls_verify_many(ctx, keys.size() / 96, keys.data(), n_aggs, sg.data(), off.data(), cnt.data(),
                                       idx.data(), mb.data(), moff.data(), len.data(), nullptr, 0, st.data());
    if (rc) return rc;
    for (int32_t s : st)
        if (s != NWV_BLS_OK) return NWV_ERR_SIGNATURE;
    return NWV_OK;
}

static int simple_launch(nwv_ctx* ctx, size_t in_bytes, const void* in_host, size_t in2_bytes, const void* in2_host,
                         size_t out_bytes, void* out_host,
                         const std::function<void(hipStream_t, uint8_t*, uint8_t*, uint8_t*)>& launch) {
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    LaneLease lane(*d);
    if ((rc = lane.rc())) return rc;
    BlsLane& L = *lane;
    const size_t o2 = (in_bytes + 255) & ~(size_t)255;
    if ((rc = L.in.ensure(o2 + in2_bytes + 16)) || (rc = L.work.ensure(out_bytes + 16))) return rc;
    uint8_t* in = static_cast<uint8_t*>(L.in.p);
    if (in_bytes) BLS_HIP(hipMemcpyAsync(in, in_host, in_bytes, hipMemcpyHostToDevice, L.stream));
    if (in2_bytes) BLS_HIP(hipMemcpyAsync(in + o2, in2_host, in2_bytes, hipMemcpyHostToDevice, L.stream));
    launch(L.stream, in, in + o2, static_cast<uint8_t*>(L.work.p));
    BLS_HIP(hipGetLastError());
    BLS_HIP(hipMemcpyAsync(out_host, L.work.p, out_bytes, hipMemcpyDeviceToHost, L.stream));
    BLS_HIP(hipStreamSynchronize(L.stream));
    return NWV_OK;
}

// messages + offsets + lengths + dst packed into one host block (the second input)
static std::vector<uint8_t> pack_msgs(size_t n, const uint8_t* msg_base, const uint64_t* msg_off,
                                      const uint32_t* msg_len, const uint8_t* dst, size_t dl, size_t* o_off,
                                      size_t* o_len, size_t* o_dst) {
    size_t bytes = 0;
    for (size_t i = 0; i < n; i++) bytes = std::max<size_t>(bytes, msg_off[i] + msg_len[i]);
    *o_off = (bytes + 1 + 7) & ~(size_t)7;
    *o_len = *o_off + 8 * n;
    *o_dst = *o_len + 4 * n;
    std::vector<uint8_t> v(*o_dst + dl + 1, 0);
    if (bytes) std::memcpy(v.data(), msg_base, bytes);
    std::memcpy(v.data() + *o_off, msg_off, 8 * n);
    std::memcpy(v.data() + *o_len, msg_len, 4 * n);
    std::memcpy(v.data() + *o_dst, dst, dl);
    return v;
}

int nwv_bls_keygen_many(nwv_ctx* ctx, size_t n, const uint8_t* sks, uint8_t* pks) {
    if (n == 0) return NWV_OK;
    if (!sks || !pks) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    return simple_launch(ctx, 32 * n, sks, 0, nullptr, 96 * n, pks, [&](hipStream_t s, uint8_t* in, uint8_t*, uint8_t* out) {
        hipLaunchKernelGGL(k_bls_keygen, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n, in, out);
    });
}

int nwv_bls_sign_many(nwv_ctx* ctx, size_t n, const uint8_t* sks, const uint8_t* msg_base, const uint64_t* msg_off,
                      const uint32_t* msg_len, const uint8_t* dst, size_t dst_len, uint8_t* sigs) {
    if (n == 0) return NWV_OK;
    if (!sks || !msg_off || !msg_len || !sigs) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    dst = dst_or_default(dst, &dst_len);
    size_t o_off, o_len, o_dst;
    const std::vector<uint8_t> m = pack_msgs(n, msg_base, msg_off, msg_len, dst, dst_len, &o_off, &o_len, &o_dst);
    return simple_launch(ctx, 32 * n, sks, m.size(), m.data(), 48 * n, sigs,
                         [&](hipStream_t s, uint8_t* in, uint8_t* mm, uint8_t* out) {
                             hipLaunchKernelGGL(k_bls_sign, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n, in, mm,
                                                reinterpret_cast<const uint64_t*>(mm + o_off),
                                                reinterpret_cast<const uint32_t*>(mm + o_len), mm + o_dst,
                                                (uint32_t)dst_len, out);
                         });
}

int nwv_bls_hash_to_g1_many(nwv_ctx* ctx, size_t n, const uint8_t* msg_base, const uint64_t* msg_off,
                            const uint32_t* msg_len, const uint8_t* dst, size_t dst_len, uint8_t* out96) {
    if (n == 0) return NWV_OK;
    if (!msg_off || !msg_len || !out96) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    dst = dst_or_default(dst, &dst_len);
    size_t o_off, o_len, o_dst;
    const std::vector<uint8_t> m = pack_msgs(n, msg_base, msg_off, msg_len, dst, dst_len, &o_off, &o_len, &o_dst);
    return simple_launch(ctx, 0, nullptr, m.size(), m.data(), 96 * n, out96,
                         [&](hipStream_t s, uint8_t*, uint8_t* mm, uint8_t* out) {
                             hipLaunchKernelGGL(k_bls_h2c_out, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n, mm,
                                                reinterpret_cast<const uint64_t*>(mm + o_off),
                                                reinterpret_cast<const uint32_t*>(mm + o_len), mm + o_dst,
                                                (uint32_t)dst_len, out);
                         });
}

int nwv_bls_pairing_many(nwv_ctx* ctx, size_t n, const uint8_t* P96, const uint8_t* Q192, uint8_t* out576) {
    if (n == 0) return NWV_OK;
    if (!P96 || !Q192 || !out576) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    return simple_launch(ctx, 96 * n, P96, 192 * n, Q192, 576 * n, out576,
                         [&](hipStream_t s, uint8_t* in, uint8_t* in2, uint8_t* out) {
                             hipLaunchKernelGGL(k_bls_pairing_raw, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n,
                                                in, in2, out);
                         });
}

}  // extern "C"
