// hostemu.cpp -- TEST-ONLY host build of the device lane code (narwhal_amd/csrc/*.h) with
// limb-bound assertions (NWV_BOUNDS_CHECK).  Compiled with hipcc --offload-host-only: the
// __host__ __device__ functions run on the CPU so tests can check the kernel arithmetic and
// its magnitude invariants against the oracle without a GPU.  Never part of the product.
#define NWV_HD __host__ __device__ inline
#define NWV_COUNT_OPS 1
unsigned long long nwv_count_mul = 0, nwv_count_sq = 0;
#include <cstring>
#include <vector>

#include "../../narwhal_amd/csrc/blake2b.h"
#include "../../narwhal_amd/csrc/ed25519_lane.h"

using namespace nwv;

static std::vector<uint32_t> g_btab;

static void ensure_btab() {
    if (!g_btab.empty()) return;
    g_btab.resize(BASE_TABLE_WORDS + CACHED_ENTRY_WORDS);
    for (int j = 0; j < BASE_TABLE_ENTRIES; j++)
        store_precomp_entry(g_btab.data() + j * PRECOMP_ENTRY_WORDS, base_multiple(j));
    store_cached_entry(g_btab.data() + BASE_TABLE_WORDS, ge_cached_identity());
}

static void words(const uint8_t* p, uint32_t w[8]) { std::memcpy(w, p, 32); }

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
    return (eq && f == FLAGS_ALL) ? 1 : 0;
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

void he_sc_reduce(const uint8_t* in64, uint8_t* out32) {
    uint32_t x[16], r[8];
    std::memcpy(x, in64, 64);
    sc_reduce512(x, r);
    std::memcpy(out32, r, 32);
}

// SHA-512 of (64-byte register prefix || msg), the challenge layout R || A || M
void he_sha512_p64(const uint8_t* prefix64, const uint8_t* msg, uint32_t len, uint8_t* out64) {
    std::vector<uint8_t> m(len + 64, 0);
    if (len) std::memcpy(m.data(), msg, len);
    uint32_t pre[16];
    std::memcpy(pre, prefix64, 64);
    const uint8_t* mp = m.data();
    sha512_state st;
    sha512_prefixed(st, pre, len, [&](uint32_t j) -> uint32_t { return ld_u32_unaligned(mp + 4 * j); });
    uint32_t out[16];
    sha512_digest_words(st, out);
    std::memcpy(out64, out, 64);
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
    sha512_prefixed(st, prefix, len, [&](uint32_t j) -> uint32_t { return ld_u32_unaligned(mp + 4 * j); });
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

}  // extern "C"
