// hostemu.cpp -- TEST-ONLY host build of the device lane code (narwhal_amd/csrc/*.h) with
// limb-bound assertions (NWV_BOUNDS_CHECK).  Compiled with hipcc --offload-host-only: the
// __host__ __device__ functions run on the CPU so tests can check the kernel arithmetic and
// its magnitude invariants against the oracle without a GPU.  Never part of the product.
#define NWV_HD __host__ __device__ inline
#define NWV_COUNT_OPS 1
unsigned long long nwv_count_mul = 0, nwv_count_sq = 0;
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../narwhal_amd/csrc/blake2b.h"
#include "../../narwhal_amd/csrc/ed25519_lane.h"
#include "../../narwhal_amd/csrc/fe_row.h"
#include "../../narwhal_amd/csrc/msm.h"

using namespace nwv;

static std::vector<uint32_t> g_btab;

static void ensure_btab() {
    if (!g_btab.empty()) return;
    g_btab.resize(BTAB_WORDS);
    for (int j = 0; j < BASE_TABLE_ENTRIES; j++) {
        store_precomp_entry(g_btab.data() + j * PRECOMP_ENTRY_WORDS, base_multiple(j));
        store_precomp_entry(g_btab.data() + BASE128_TABLE_OFFSET + j * PRECOMP_ENTRY_WORDS, base128_multiple(j));
    }
    store_cached_entry(g_btab.data() + BASE_TABLE_WORDS, ge_cached_identity());
}

static void words(const uint8_t* p, uint32_t w[8]) { std::memcpy(w, p, 32); }

// k_msm_final on the host: window sums -> cached row limbs (as the kernel's LDS), the row Horner
// of fe_row.h on the emulated wave, then [8] d == identity.  xyz (optional): canonical words of
// the X | Y | Z that row 0 hands back.
static bool row_final_host(const MsmLayout& lay, const uint32_t* ws, uint32_t* xyz) {
    std::vector<uint32_t> cq((size_t)MSM_MAX_WINDOWS * 64, 0), top(64, 0), fin(48, 0);
    for (int t = 0; t < lay.nw; t++) {
        const ge_p3 p = load_p3(ws + (size_t)P3_WORDS * t);
        const ge_cached c = ge_p3_to_cached(p);
        fe_to_limbs16(c.YpX, cq.data() + 64 * t);
        fe_to_limbs16(c.YmX, cq.data() + 64 * t + 16);
        fe_to_limbs16(c.T2d, cq.data() + 64 * t + 32);
        fe_to_limbs16(c.Z2, cq.data() + 64 * t + 48);
        if (t == lay.nw - 1) {
            fe_to_limbs16(p.X, top.data());
            fe_to_limbs16(p.Y, top.data() + 16);
            fe_to_limbs16(p.Z, top.data() + 32);
            fe_to_limbs16(p.T, top.data() + 48);
        }
    }
    rowf::row_horner(cq.data(), top.data(), lay, fin.data());
    const fe X = fe_from_limbs16(fin.data()), Y = fe_from_limbs16(fin.data() + 16), Z = fe_from_limbs16(fin.data() + 32);
    if (xyz) {
        fe_freeze(X, xyz);
        fe_freeze(Y, xyz + 8);
        fe_freeze(Z, xyz + 8 * 2);
    }
    return fe_is_zero(X) && fe_eq(Y, Z);
}

// The fused tail of narwhal_amd/csrc/msm_kernels.hip (k_msm_tail), sequentially: per window S_w
// chunks of C buckets; each chunk's butterfly (lane 0 -> chunk total R_s, lane 2^k -> plane
// T_{s,k}); per plane a butterfly over the chunks (T_k = sum_s T_{s,k}; the R_s butterfly gives
// the high planes and U); the plane chain and [2^(pos+3)] on the emulated 16-lane rows; the sum
// over windows; the identity test.
static void butterfly(std::vector<ge_p3>& p) {
    for (size_t o = 1; o < p.size(); o <<= 1)
        for (size_t g = 0; g < p.size(); g++)
            if (!(g & o)) p[g] = p3_add(p[g], p[g + o]);
}
static int lg2(int x) {
    int l = 0;
    while ((1 << l) < x) l++;
    return l;
}
static bool tail_host(const MsmLayout& lay, const uint32_t* bs, uint32_t S) {
    ge_p3 tot = ge_p3_identity();
    std::vector<uint32_t> ladder(64, 0);  // the final sum's accumulator (row limbs), the identity
    ladder[16] = ladder[32] = 1;
    std::vector<ge_p3> scaled;
    for (int w = 0; w < lay.nw; w++) {
        const int nb = 1 << (lay.width[w] - 1);
        const int Sw = (int)S < nb ? (int)S : nb, C = nb / Sw, lgC = lg2(C), lgS = lg2(Sw), m = lgC + lgS;
        std::vector<std::vector<ge_p3>> group(lgC + 1, std::vector<ge_p3>(Sw));  // [plane q or R][s]
        for (int s = 0; s < Sw; s++) {
            std::vector<ge_p3> lane(C);
            for (int g = 0; g < C; g++)
                lane[g] = load_p3(bs + (size_t)P3_WORDS * ((size_t)lay.kbase[w] + (size_t)s * C + g));
            butterfly(lane);
            group[lgC][s] = lane[0];
            for (int k = 0; k < lgC; k++) group[k][s] = lane[(size_t)1 << k];
        }
        for (auto& g : group) butterfly(g);
        std::vector<ge_p3> planes(m + 1);
        for (int k = 0; k < lgC; k++) planes[k] = group[k][0];
        for (int i = 0; i < lgS; i++) planes[lgC + i] = group[lgC][(size_t)1 << i];
        planes[m] = group[lgC][0];
        std::vector<uint32_t> rows(64 * (m + 1)), out(64);
        for (int k = 0; k <= m; k++) {
            const ge_p3& pl = planes[k];
            fe_to_limbs16(fe_carry(fe_add(pl.Y, pl.X)), rows.data() + 64 * k);
            fe_to_limbs16(fe_carry(fe_sub(pl.Y, pl.X)), rows.data() + 64 * k + 16);
            fe_to_limbs16(fe_carry(fe_mul(pl.T, fe_d2())), rows.data() + 64 * k + 32);
            fe_to_limbs16(fe_carry(fe_add(pl.Z, pl.Z)), rows.data() + 64 * k + 48);
        }
        std::vector<uint32_t> sc(192);
        // the windows cycle through the three multiply forms (rotations, as on the device; LDS; shifts)
        const int rot = w % 3 == 0 ? 1 : 0;
        const rowf::RowP3 d = rowf::row_planes_chain(rows.data(), m, lay.pos[w] + 3, out.data(),
                                                     (w % 3 == 1) ? sc.data() : nullptr, rot);
        const ge_p3 ws{fe_from_limbs16(out.data()), fe_from_limbs16(out.data() + 16), fe_from_limbs16(out.data() + 32),
                       fe_from_limbs16(out.data() + 48)};
        scaled.push_back(ws);
        tot = p3_add(tot, ws);
        // the kernel's final sum: each window's cached row form, one ladder step per window
        rowf::RowConsts k = rowf::row_consts();
        k.rot = rot;
        k.sc = (w % 3 == 1) ? sc.data() : nullptr;
        const rowf::V c = rowf::row_to_cached(d, k);
        std::vector<uint32_t> q(64), nxt(64);
        for (int i = 0; i < 64; i++) q[i] = c.l[i];
        rowf::row_ladder_step(ladder.data(), q.data(), nxt.data(), rot);
        ladder = nxt;
    }
    {
        const fe X = fe_from_limbs16(ladder.data()), Y = fe_from_limbs16(ladder.data() + 16),
                 Z = fe_from_limbs16(ladder.data() + 32);
        const bool ladder_id = fe_is_zero(X) && fe_eq(Y, Z);
        if (ladder_id != (fe_is_zero(tot.X) && fe_eq(tot.Y, tot.Z))) abort();  // ladder vs lane sum
    }
    // a binary tree of additions over the windows (identity padded to a power of two), the round-4
    // kernel's final sum, against the sequential lane sum
    size_t P2 = 1;
    while (P2 < scaled.size()) P2 <<= 1;
    scaled.resize(P2, ge_p3_identity());
    for (size_t o = 1; o < P2; o <<= 1)
        for (size_t i = 0; i + o < P2; i += 2 * o) scaled[i] = p3_add(scaled[i], scaled[i + o]);
    const bool tree_id = fe_is_zero(scaled[0].X) && fe_eq(scaled[0].Y, scaled[0].Z);
    const bool lane_id = fe_is_zero(tot.X) && fe_eq(tot.Y, tot.Z);
    if (tree_id != lane_id) abort();  // the tree sum and the sequential sum must agree
    return tree_id;
}

extern "C" {

int he_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t len) {
    ensure_btab();
    uint32_t Aw[8], Rw[8], Sw[8];
    words(pk, Aw);
    words(sig, Rw);
    words(sig + 32, Sw);
    std::vector<uint8_t> m(len + 64, 0);
    if (len) std::memcpy(m.data(), msg, len);
    // phase-split path, as on the GPU
    uint32_t k[8];
    std::vector<uint32_t> tbl(LANE_SCRATCH_WORDS);
    uint32_t f = lane_hash(Aw, Rw, Sw, m.data(), len, k);
    f |= lane_points(Aw, Rw, tbl.data());
    const bool eq = lane_straus_check(k, Sw, tbl.data(), g_btab.data());
    // the prefetching form (k_ed_straus_pf) must agree on every input
    if (lane_straus_check<true>(k, Sw, tbl.data(), g_btab.data()) != eq) std::abort();
    return (eq && f == FLAGS_ALL) ? 1 : 0;
}

// the per-signature check's half-size split of k (< l): u (4 words), m = |v| (4 words), vneg
void he_half_split(const uint8_t* k32, uint32_t* u4, uint32_t* m4, int* vneg) {
    uint32_t k[8];
    words(k32, k);
    bool neg;
    sc_half_split(k, u4, m4, neg);
    *vneg = neg ? 1 : 0;
}

// field multiplies / squarings executed by each kernel phase of one verification:
// counts[0..1] hash (0, 0), [2..3] points, [4..5] straus+check
void he_phase_counts(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t len,
                     unsigned long long counts[6]) {
    ensure_btab();
    uint32_t Aw[8], Rw[8], Sw[8], k[8];
    words(pk, Aw);
    words(sig, Rw);
    words(sig + 32, Sw);
    std::vector<uint8_t> m(len + 64, 0);
    if (len) std::memcpy(m.data(), msg, len);
    std::vector<uint32_t> tbl(LANE_SCRATCH_WORDS);
    nwv_count_mul = nwv_count_sq = 0;
    lane_hash(Aw, Rw, Sw, m.data(), len, k);
    counts[0] = nwv_count_mul; counts[1] = nwv_count_sq;
    nwv_count_mul = nwv_count_sq = 0;
    lane_points(Aw, Rw, tbl.data());
    counts[2] = nwv_count_mul; counts[3] = nwv_count_sq;
    nwv_count_mul = nwv_count_sq = 0;
    lane_straus_check(k, Sw, tbl.data(), g_btab.data());
    counts[4] = nwv_count_mul; counts[5] = nwv_count_sq;
}

int he_decompress(const uint8_t* p, uint8_t* out_xy) {
    uint32_t w[8];
    words(p, w);
    ge_p3 P;
    bool ok = ge_decompress(w, P);
    uint32_t x[8], y[8];
    fe_freeze(P.X, x);
    fe_freeze(P.Y, y);
    std::memcpy(out_xy, x, 32);
    std::memcpy(out_xy + 32, y, 32);
    return ok ? 1 : 0;
}

// k_msm_prep's row form of the decompression (msm_kernels.hip msm_points_rows_block) on the
// emulated wave, four points at a time (one per row): the prelude, the power, the root and its
// square-root test and the record's 2d x y as row products (form 0: DPP shifts, 1: LDS, 2: row
// rotations as on the device), the zero / sign tests and the record's conversion lane-local as on
// lanes 0..2 of each row.  Each point's MSM record (30 words, canonical values compared) and decode
// flag must equal the lane-local ge_decompress's; returns the number of points that differ.
int he_row_decompress(const uint8_t* encs, int count, int form) {
    int bad = 0;
    std::vector<uint32_t> sc(192);
    for (int base = 0; base < count; base += 4) {
        rowf::V y16;
        bool sign[4] = {false, false, false, false};
        for (int l = 0; l < 64; l++) {
            const int q = l >> 4, limb = l & 15;
            uint32_t v = 0;
            if (base + q < count) v = (uint32_t)encs[32 * (base + q) + 2 * limb] | ((uint32_t)encs[32 * (base + q) + 2 * limb + 1] << 8);
            if (limb == 15) {
                sign[q] = (v >> 15) != 0;
                v &= 0x7FFFu;
            }
            y16.l[l] = v;
        }
        rowf::RowConsts k = rowf::row_consts();
        k.rot = form == 2 ? 1 : 0;
        k.sc = form == 1 ? sc.data() : nullptr;
        rowf::V u, v, uv3, uv7, r, ri, c0, c1, c2;
        rowf::row_dec_pre(y16, k, u, v, uv3, uv7);
        const rowf::V pw = rowf::row_pow_p58(uv7, k);
        rowf::row_dec_mid(uv3, pw, u, v, k, r, ri, c0, c1, c2);
        auto limbs = [](const rowf::V& x, int q, uint32_t out[16]) {
            for (int i = 0; i < 16; i++) out[i] = x.l[16 * q + i];
        };
        bool ok[4];
        rowf::V rr = r;
        for (int q = 0; q < 4; q++) {
            uint32_t a[16];
            bool z[3];
            const rowf::V* cs[3] = {&c0, &c1, &c2};
            for (int c = 0; c < 3; c++) {
                limbs(*cs[c], q, a);
                z[c] = fe_is_zero(fe_from_limbs16(a));
            }
            ok[q] = z[0] || z[1];
            if (z[1] || z[2])
                for (int i = 0; i < 16; i++) rr.l[16 * q + i] = ri.l[16 * q + i];
        }
        rowf::M flip;
        const rowf::V nrr = rowf::carry32(rowf::sub(rowf::bc(0), rr, k), k);
        for (int q = 0; q < 4; q++) {
            uint32_t a[16];
            limbs(rr, q, a);
            const bool negr = fe_is_negative(fe_from_limbs16(a)) != 0;
            for (int i = 0; i < 16; i++) flip.l[16 * q + i] = negr != sign[q];
        }
        const rowf::V x = rowf::sel(flip, rr, nrr);
        rowf::V ypx, ymx, xy2d;
        rowf::row_dec_record(x, y16, k, ypx, ymx, xy2d);
        for (int q = 0; q < 4 && base + q < count; q++) {
            uint32_t w[8];
            words(encs + 32 * (base + q), w);
            ge_p3 R;
            const bool ok_ref = ge_decompress(w, R);
            uint32_t e_ref[MSM_PT_WORDS];
            msm_store_point(e_ref, R);
            bool same = ok[q] == ok_ref;
            const rowf::V* co[3] = {&ypx, &ymx, &xy2d};
            for (int c = 0; c < 3 && same; c++) {  // canonical values of the record's coordinates
                uint32_t a[16], fa[8], fb[8];
                limbs(*co[c], q, a);
                fe_freeze(fe_from_limbs16(a), fa);
                fe_freeze(load_fe(e_ref + 10 * c), fb);
                same = std::memcmp(fa, fb, 32) == 0;
            }
            bad += same ? 0 : 1;
        }
    }
    return bad;
}

void he_sc_reduce(const uint8_t* in64, uint8_t* out32) {
    uint32_t x[16], r[8];
    std::memcpy(x, in64, 64);
    sc_reduce512(x, r);
    std::memcpy(out32, r, 32);
}

// SHA-512 of (64-byte register prefix || msg), the challenge layout R || A || M
// (the message is placed `shift` bytes past an aligned address: the block loader's funnel shift)
void he_sha512_p64_at(const uint8_t* prefix64, const uint8_t* msg, uint32_t len, uint32_t shift, uint8_t* out64) {
    std::vector<uint8_t> m(len + 64 + 16, 0xA5);
    if (len) std::memcpy(m.data() + shift, msg, len);
    uint32_t pre[16];
    std::memcpy(pre, prefix64, 64);
    const uint8_t* mp = m.data() + shift;
    sha512_state st;
    sha512_prefixed_msg(st, pre, mp, len);
    uint32_t out[16];
    sha512_digest_words(st, out);
    std::memcpy(out64, out, 64);
}
void he_sha512_p64(const uint8_t* prefix64, const uint8_t* msg, uint32_t len, uint8_t* out64) {
    he_sha512_p64_at(prefix64, msg, len, 0, out64);
}

void he_blake2b256(const uint8_t* msg, uint64_t len, uint8_t* out32) {
    std::vector<uint8_t> m(len + 64, 0);
    if (len) std::memcpy(m.data(), msg, len);
    blake2b_state s;
    blake2b_init256(s);
    const uint64_t nblocks = len == 0 ? 1 : (len + 127) / 128;
    for (uint64_t b = 0; b < nblocks; b++) {
        u64p w[16];
        for (int t = 0; t < 16; t++) {
            w[t].lo = msg_word_trim(m.data(), 128 * b + 8 * t, len);
            w[t].hi = msg_word_trim(m.data(), 128 * b + 8 * t + 4, len);
        }
        const bool last = b + 1 == nblocks;
        blake2b_compress(s, w, last ? (uint32_t)(len - 128 * b) : 128u, last);
    }
    uint32_t d[8];
    blake2b_digest256(s, d);
    std::memcpy(out32, d, 32);
}

void he_sign(const uint8_t* seed, const uint8_t* msg, uint32_t len, uint8_t* pk_out, uint8_t* sig_out) {
    ensure_btab();
    const uint32_t* ident = g_btab.data() + BASE_TABLE_WORDS;
    std::vector<uint8_t> m(len + 64, 0);
    if (len) std::memcpy(m.data(), msg, len);
    uint32_t sw[8];
    words(seed, sw);
    sha512_state st;
    sha512_prefixed(st, sw, 0, [&](uint32_t) -> uint32_t { return 0u; });
    uint32_t h[16];
    sha512_digest_words(st, h);
    h[0] &= ~7u;
    h[7] &= 0x7fffffffu;
    h[7] |= 0x40000000u;
    uint32_t ax[16], a[8], prefix[8];
    for (int j = 0; j < 16; j++) ax[j] = j < 8 ? h[j] : 0u;
    for (int j = 0; j < 8; j++) prefix[j] = h[8 + j];
    sc_reduce512(ax, a);
    const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t Aw[8], Rw[8];
    ge_compress(straus_sB_minus_kA(zero, a, nullptr, g_btab.data(), ident), Aw);
    const uint8_t* mp = m.data();
    sha512_prefixed_msg(st, prefix, mp, len);
    uint32_t rh[16], r[8];
    sha512_digest_words(st, rh);
    sc_reduce512(rh, r);
    ge_compress(straus_sB_minus_kA(zero, r, nullptr, g_btab.data(), ident), Rw);
    uint32_t k[8], ka[8], S[8];
    challenge_scalar(Rw, Aw, mp, len, k);
    sc_mul(k, a, ka);
    sc_add(ka, r, S);
    std::memcpy(pk_out, Aw, 32);
    std::memcpy(sig_out, Rw, 32);
    std::memcpy(sig_out + 32, S, 32);
}

// Batch verification through the K5 MSM, sequentially on the host with the device arithmetic
// (msm.h): same point layout, window layout, recoding, bucket rule, G-lane window reduction and
// Horner as narwhal_amd/csrc/msm_kernels.hip, without the parallel sort.  Returns the verdict.
//
// split != 0: the key-cache form (k_keycache_fill / k_msm_keysum / k_msm_bscalar with a cache):
// points [0, n) A_i with lo(z_i k_i), [n, 2n) 2^128 A_i with hi(z_i k_i), 2n = 2^128 B with hi(b),
// 2n + 1 = B with lo(b), then the R_i; every scalar < 2^128, z-only layout (msm_make_layout_z).
static int msm_batch_impl(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                          const uint32_t* len, const uint8_t* seed32, int c, int G, unsigned long long* counts,
                          bool split) {
    ensure_btab();
    MsmLayout lay;
    const bool nt = c < 0;  // c < 0: the narrow-top layout of width -c (msm_split)
    if (nt) c = -c;
    if (!(split ? msm_make_layout_z(c, lay) : msm_make_layout(c, lay, nt))) return -1;
    uint32_t seed[8];
    std::memcpy(seed, seed32, 32);
    const size_t na = split ? 2 * n + 1 : n;  // points before B
    const size_t np = na + 1 + n;
    std::vector<uint32_t> scal(8 * np, 0), pts(MSM_PT_WORDS * np);
    bool ok = true;
    unsigned long long col[9] = {0};
    for (size_t i = 0; i < n; i++) {
        uint32_t Aw[8], Rw[8], Sw[8], k[8], z[8], a[8], zs[8];
        words(pk + 32 * i, Aw);
        words(sig + 64 * i, Rw);
        words(sig + 64 * i + 32, Sw);
        std::vector<uint8_t> m(len[i] + 64, 0);
        if (len[i]) std::memcpy(m.data(), msg + off[i], len[i]);
        if (lane_hash(Aw, Rw, Sw, m.data(), len[i], k) != FLAG_S_OK) ok = false;
        msm_z(seed, i, z);
        sc_mul(z, k, a);
        sc_mul(z, Sw, zs);
        uint32_t lo[8], hi[8];
        msm_split128(a, lo, hi);
        for (int t = 0; t < 8; t++) {
            scal[8 * i + t] = split ? lo[t] : a[t];
            if (split) scal[8 * (n + i) + t] = hi[t];
            scal[8 * (na + 1 + i) + t] = z[t];
            col[t] += zs[t];
        }
        ge_p3 P;
        ok &= ge_decompress(Aw, P);
        msm_store_point(pts.data() + MSM_PT_WORDS * i, P);
        if (split) {  // the cache's second record, as k_keycache_fill builds it
            const ge_precomp q = ge_p3_to_precomp(p3_dbl_n(P, 128));
            uint32_t* e = pts.data() + MSM_PT_WORDS * (n + i);
            store_fe(e, q.ypx);
            store_fe(e + 10, q.ymx);
            store_fe(e + 20, q.xy2d);
            e[30] = e[31] = 0u;
        }
        ok &= ge_decompress(Rw, P);
        msm_store_point(pts.data() + MSM_PT_WORDS * (na + 1 + i), P);
    }
    {
        uint32_t x[16];
        unsigned long long cc = 0;
        for (int t = 0; t < 16; t++) {
            if (t < 9) cc += col[t];
            x[t] = (uint32_t)cc;
            cc >>= 32;
        }
        uint32_t r[8];
        sc_reduce512(x, r);
        uint32_t nz = 0;
        for (int t = 0; t < 8; t++) nz |= r[t];
        long long br = 0;
        uint32_t b[8];
        for (int t = 0; t < 8; t++) {
            long long d = (long long)sc_l(t) - r[t] + br;
            b[t] = nz ? (uint32_t)d : 0u;
            br = d >> 32;
        }
        uint32_t lo[8], hi[8];
        msm_split128(b, lo, hi);
        for (int t = 0; t < 8; t++) {
            scal[8 * na + t] = split ? lo[t] : b[t];
            if (split) scal[8 * (na - 1) + t] = hi[t];
        }
        msm_point_from_precomp(pts.data() + MSM_PT_WORDS * na, g_btab.data() + PRECOMP_ENTRY_WORDS);
        if (split) {
            uint32_t bw[8];
            ge_basepoint_words(bw);
            ge_p3 Bp;
            ge_decompress(bw, Bp);
            const ge_precomp q = ge_p3_to_precomp(p3_dbl_n(Bp, 128));
            uint32_t* e = pts.data() + MSM_PT_WORDS * (na - 1);
            store_fe(e, q.ypx);
            store_fe(e + 10, q.ymx);
            store_fe(e + 20, q.xy2d);
            e[30] = e[31] = 0u;
        }
    }
    nwv_count_mul = nwv_count_sq = 0;
    const uint32_t nkeys = lay.kbase[lay.nw];
    std::vector<std::vector<uint32_t>> buckets(nkeys);
    for (size_t j = 0; j < np; j++) {
        msm_recode(&scal[8 * j], lay, j <= na ? lay.nw : lay.nw_z, [&](int w, int d) {
            if (d) buckets[lay.kbase[w] + (d < 0 ? -d : d) - 1].push_back((uint32_t)j | (d < 0 ? MSM_NEG : 0u));
        });
    }
    std::vector<uint32_t> bs((size_t)P3_WORDS * nkeys), ws((size_t)P3_WORDS * lay.nw);
    for (size_t key = 0; key < nkeys; key++) {
        ge_p3 acc = ge_p3_identity();
        for (uint32_t v : buckets[key])
            acc = ge_p1p1_to_p3(ge_madd(acc, msm_load_point(pts.data() + MSM_PT_WORDS * (v & ~MSM_NEG), (v & MSM_NEG) != 0)));
        store_p3(bs.data() + P3_WORDS * key, acc);
    }
    for (int w = 0; w < lay.nw; w++) {
        const int nb = 1 << (lay.width[w] - 1);
        const int Gw = nb < G ? nb : G;
        const int L = nb / Gw;
        std::vector<ge_p3> run(Gw), acc(Gw);
        for (int g = 0; g < Gw; g++) {
            const uint32_t* bw = bs.data() + (size_t)P3_WORDS * ((size_t)lay.kbase[w] + (size_t)g * L);
            msm_segment_sums(L, [&](int k) { return load_p3(bw + (size_t)P3_WORDS * k); }, run[g], acc[g]);
        }
        int lg = 0;
        while ((1 << lg) < L) lg++;
        ge_p3 suf = ge_p3_identity(), tot = acc[0];
        for (int g = Gw - 1; g >= 1; g--) {
            suf = p3_add(suf, run[g]);
            tot = p3_add(tot, p3_add(acc[g], lg ? p3_dbl_n(suf, lg) : suf));
        }
        store_p3(ws.data() + P3_WORDS * w, tot);
    }
    ge_p3 d = load_p3(ws.data() + (size_t)P3_WORDS * (lay.nw - 1));
    for (int w = lay.nw - 2; w >= 0; w--) {
        d = p3_dbl_n(d, lay.width[w]);
        d = p3_add(d, load_p3(ws.data() + (size_t)P3_WORDS * w));
    }
    const bool eq = p3_mul8_is_identity(d);
    // the kernel's row-parallel Horner must reach the same verdict
    if (row_final_host(lay, ws.data(), nullptr) != eq) return -2;
    // and so must the fused tail's decomposition; the chunk count rotates over calls
    static const uint32_t kS[4] = {1u, 2u, 8u, 64u};
    static unsigned calls = 0;
    if (tail_host(lay, bs.data(), kS[calls++ % 4]) != eq) return -3;
    if (counts) {
        counts[0] = nwv_count_mul;
        counts[1] = nwv_count_sq;
    }
    return (ok && eq) ? 1 : 0;
}

int he_msm_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                 const uint32_t* len, const uint8_t* seed32, int c, int G, unsigned long long* counts) {
    return msm_batch_impl(n, pk, sig, msg, off, len, seed32, c, G, counts, false);
}
int he_msm_batch_split(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                       const uint32_t* len, const uint8_t* seed32, int c, int G) {
    return msm_batch_impl(n, pk, sig, msg, off, len, seed32, c, G, nullptr, true);
}

// The MSM's basepoint term as k_msm_prep's last hash workgroup computes it: c = 8 b mod l, its 64
// signed radix-16 digits, the sum of the comb entries i 16^j B (msm.h comb_entry), against
// [8]([b]B) by plain double-and-add.  Returns 1 when the two points are equal.
int he_comb_check(const uint8_t* b32) {
    uint32_t b[8], c[8];
    words(b32, b);
    const uint32_t eight[8] = {8u, 0, 0, 0, 0, 0, 0, 0};
    sc_mul(b, eight, c);
    int d[COMB_TABLES];
    comb_digits(c, d);
    ge_p3 acc = ge_p3_identity();
    std::vector<uint32_t> e(MSM_PT_WORDS);
    for (int j = 0; j < COMB_TABLES; j++) {
        if (d[j] < -8 || d[j] > 8) return -1;
        if (!d[j]) continue;
        comb_entry(j, d[j] < 0 ? -d[j] : d[j], e.data());
        acc = ge_p1p1_to_p3(ge_madd(acc, msm_load_point(e.data(), d[j] < 0)));
    }
    uint32_t bw[8];
    ge_basepoint_words(bw);
    ge_p3 B;
    ge_decompress(bw, B);
    const ge_cached cb = ge_p3_to_cached(B);
    ge_p3 ref = ge_p3_identity();
    for (int bit = 255; bit >= 0; bit--) {
        ref = ge_p3_dbl(ref);
        if ((b[bit >> 5] >> (bit & 31)) & 1) ref = ge_p1p1_to_p3(ge_add(ref, cb));
    }
    ref = p3_dbl_n(ref, 3);
    uint32_t w1[8], w2[8];
    ge_compress(acc, w1);
    ge_compress(ref, w2);
    return std::memcmp(w1, w2, 32) == 0 ? 1 : 0;
}

// The one-launch path's per-signature check (tiny_kernels.hip k_ed_tiny), sequentially: the key's
// comb table i 16^j A (k_key_comb_fill: an undecodable key gets the identity's table), the
// signed radix-16 digits of s (zeroed when s >= l) and of k, [s]B - [k]A as the sum of one entry
// of each table per digit position (the kernel's lane j), minus R, times 8, the identity test,
// and the decode / canonicity flags.  Returns the verdict (1 accept).
int he_tiny_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t len) {
    uint32_t Aw[8], Rw[8], Sw[8], k[8];
    words(pk, Aw);
    words(sig, Rw);
    words(sig + 32, Sw);
    std::vector<uint8_t> m(len + 64, 0);
    if (len) std::memcpy(m.data(), msg, len);
    const bool sok = lane_hash(Aw, Rw, Sw, m.data(), len, k) == FLAG_S_OK;
    if (!sok)
        for (int q = 0; q < 8; q++) Sw[q] = 0u;
    ge_p3 A, R;
    const bool aok = ge_decompress(Aw, A);
    if (!aok) A = ge_p3_identity();
    const bool rok = ge_decompress(Rw, R);
    int ds[COMB_TABLES], dk[COMB_TABLES];
    comb_digits(Sw, ds);
    comb_digits(k, dk);
    std::vector<uint32_t> e(MSM_PT_WORDS);
    ge_p3 P = ge_p3_identity();
    for (int j = 0; j < COMB_TABLES; j++) {
        ge_p3 Pj = ge_p3_identity();
        if (ds[j] < -8 || ds[j] > 8 || dk[j] < -8 || dk[j] > 8) return -1;  // past the tables
        if (ds[j]) {
            comb_entry(j, ds[j] < 0 ? -ds[j] : ds[j], e.data());
            Pj = ge_p1p1_to_p3(ge_madd(Pj, msm_load_point(e.data(), ds[j] < 0)));
        }
        if (dk[j]) {
            comb_entry_of(A, j, dk[j] < 0 ? -dk[j] : dk[j], e.data());
            Pj = ge_p1p1_to_p3(ge_madd(Pj, msm_load_point(e.data(), dk[j] > 0)));
        }
        P = p3_add(P, Pj);
    }
    // [8] R as the kernel computes it: three row doublings (fe_row.h row_dbl, every row holding R)
    // from (2x : 2y : 2) = ((y+x) - (y-x) : (y+x) + (y-x) : 2), R's record as row limbs
    if (!rok) R = ge_p3_identity();
    uint32_t rrec[MSM_PT_WORDS], yp[16], ym[16];
    msm_store_point(rrec, R);
    fe_to_limbs16(load_fe(rrec), yp);
    fe_to_limbs16(load_fe(rrec + 10), ym);
    rowf::RowConsts rk = rowf::row_consts();
    rk.rot = 1;
    rowf::V ypx, ymx, two;
    for (int l = 0; l < 64; l++) {
        ypx.l[l] = yp[l & 15];
        ymx.l[l] = ym[l & 15];
        two.l[l] = (l & 15) == 0 ? 2u : 0u;
    }
    rowf::RowP3 d{rowf::carry32(rowf::sub(ypx, ymx, rk), rk), rowf::carry32(ypx + ymx, rk), two, rowf::bc(0)};
    for (int r = 0; r < 3; r++) d = rowf::row_dbl(d, rk);
    uint32_t xl[16], yl[16], zl[16];
    for (int i = 0; i < 16; i++) {
        xl[i] = d.X.l[i];
        yl[i] = d.Y.l[i];
        zl[i] = d.Z.l[i];
    }
    const fe RX = fe_from_limbs16(xl), RY = fe_from_limbs16(yl), RZ = fe_from_limbs16(zl);
    // the round-5 form of the same equation, [8](P - R) = O, must agree with the kernel's
    const ge_p3 Q = ge_p1p1_to_p3(ge_madd(P, msm_load_point(rrec, true)));
    // [8] P, then [8] R = [8] P projectively (the cofactored equation [8](R - P) = 0)
    for (int r = 0; r < 3; r++) P = p3_add(P, P);
    const bool eq = fe_eq(fe_mul(P.X, RZ), fe_mul(RX, P.Z)) && fe_eq(fe_mul(P.Y, RZ), fe_mul(RY, P.Z));
    if (rok && eq != p3_mul8_is_identity(Q)) return -2;
    return (eq && aok && rok && sok) ? 1 : 0;
}

// signed digits of a 256-bit scalar over layout(c): z range (bits = 128) or full range (253);
// out: nw, then (pos, digit) pairs
int he_msm_recode(const uint8_t* s32, int c, int bits, int* out) {
    uint32_t s[8];
    words(s32, s);
    MsmLayout lay;
    if (!msm_make_layout(c < 0 ? -c : c, lay, c < 0)) return -1;  // c < 0: narrow-top layout
    const int nw = bits == MSM_BITS_Z ? lay.nw_z : lay.nw;
    msm_recode(s, lay, nw, [&](int w, int d) {
        out[2 * w] = lay.pos[w];
        out[2 * w + 1] = d;
    });
    return nw;
}

// layout(c): nw, nw_z, then widths (c < 0: the narrow-top layout of width -c)
int he_msm_layout(int c, int* out) {
    MsmLayout lay;
    if (!msm_make_layout(c < 0 ? -c : c, lay, c < 0)) return -1;
    out[0] = lay.nw;
    out[1] = lay.nw_z;
    for (int w = 0; w < lay.nw; w++) out[2 + w] = lay.width[w];
    return lay.nw;
}

void he_chacha20_block(const uint8_t* key32, uint32_t counter, const uint8_t* nonce12, uint8_t* out64) {
    uint32_t key[8], nonce[3], out[16];
    words(key32, key);
    std::memcpy(nonce, nonce12, 12);
    chacha20_block(key, counter, nonce, out);
    std::memcpy(out64, out, 64);
}

void he_msm_z(const uint8_t* seed32, uint64_t i, uint8_t* z32) {
    uint32_t seed[8], z[8];
    words(seed32, seed);
    msm_z(seed, i, z);
    std::memcpy(z32, z, 32);
}

// field multiplies / squarings of k_msm_points per signature (decompress R and A, affine entry)
void he_msm_point_counts(const uint8_t* pk, const uint8_t* sig, unsigned long long counts[2]) {
    uint32_t Aw[8], Rw[8], e[MSM_PT_WORDS];
    words(pk, Aw);
    words(sig, Rw);
    nwv_count_mul = nwv_count_sq = 0;
    ge_p3 P;
    ge_decompress(Rw, P);
    msm_store_point(e, P);
    ge_decompress(Aw, P);
    msm_store_point(e, P);
    counts[0] = nwv_count_mul;
    counts[1] = nwv_count_sq;
}

// one field multiply on the emulated wave (use_lds 0: the DPP shift form, 1: the LDS-operand form,
// 2: the row-rotation form): a, b
// given as 16 loose limbs (same in every row); out = row 0's product limbs.  Returns 0 when the four
// rows disagree.
int he_row_mul(const uint32_t* a16, const uint32_t* b16, uint32_t* out16, int use_lds) {
    rowf::V a, b;
    for (int i = 0; i < 64; i++) {
        a.l[i] = a16[i & 15];
        b.l[i] = b16[i & 15];
    }
    std::vector<uint32_t> sc(192, 0xDEADBEEFu);
    rowf::RowConsts k = rowf::row_consts();
    if (use_lds == 1) k.sc = sc.data();
    k.rot = use_lds == 2;
    const rowf::V r = rowf::mul(a, b, k);
    for (int i = 0; i < 64; i++)
        if (r.l[i] != r.l[i & 15]) return 0;
    for (int k = 0; k < 16; k++) out16[k] = r.l[k];
    return 1;
}

// Horner over nw window sums W_w = decompress(pts[w]) (widths[w] bits each): the row path of
// k_msm_final (xyz_row) against the lane-local chain (xyz_ref), both after [8]; canonical words
// of X | Y | Z.  Returns -1 if a point does not decode, else the row path's identity verdict.
int he_row_horner(int nw, const uint8_t* widths, const uint8_t* pts, uint32_t* xyz_row, uint32_t* xyz_ref) {
    MsmLayout lay{};
    lay.nw = nw;
    for (int w = 0; w < nw; w++) lay.width[w] = widths[w];
    std::vector<uint32_t> ws((size_t)P3_WORDS * nw);
    for (int w = 0; w < nw; w++) {
        uint32_t pw[8];
        words(pts + 32 * w, pw);
        ge_p3 P;
        if (!ge_decompress(pw, P)) return -1;
        store_p3(ws.data() + (size_t)P3_WORDS * w, P);
    }
    const bool id = row_final_host(lay, ws.data(), xyz_row);
    ge_p3 d = load_p3(ws.data() + (size_t)P3_WORDS * (nw - 1));
    for (int w = nw - 2; w >= 0; w--) {
        d = p3_dbl_n(d, lay.width[w]);
        d = p3_add(d, load_p3(ws.data() + (size_t)P3_WORDS * w));
    }
    d = p3_dbl_n(d, 3);
    fe_freeze(d.X, xyz_ref);
    fe_freeze(d.Y, xyz_ref + 8);
    fe_freeze(d.Z, xyz_ref + 16);
    return id ? 1 : 0;
}

}  // extern "C"
