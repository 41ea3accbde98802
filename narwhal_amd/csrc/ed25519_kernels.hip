// ed25519_kernels.hip -- gfx950 kernels of the Ed25519 verification engine.
//
// Per-signature verification (K1-K4) runs as three kernels so that each phase gets the
// occupancy its own register footprint allows (one fused kernel needed ~250 VGPRs = 1 wave
// per SIMD; the phases need 70-145):
//   k_ed_hash     K1+K3  k = SHA-512(R || A || M) mod l, s < l         (one message per lane)
//   k_ed_points   K2     decompress R and A, build the lane's 0..8 A and 0..8 R tables in HBM
//   k_ed_straus   K4     [8]([s]B - [k]A - R) == identity on half-size scalars (ed25519_lane.h),
//                        wave ballot -> verdict words
// plus
//   k_base_table  one-time: j B for j = 0..128 (affine Niels, +-2dxy) + an identity entry
//   k_sign        RFC 8032 keygen + signing per lane (synthetic data / tests only)
//
// Inputs are SoA: pk[n][32], sig[n][64] (coalesced 16-byte loads), a padded message arena
// addressed by msg_off[n] / msg_len[n].  Intermediate state per signature: k[n][8] words,
// flags[n], and a 3.5 KiB point table (LANE_SCRATCH_WORDS words).  The verdict of signature i
// is bit i % 64 of word i / 64, written by lane 0 of the wave that owns those 64 signatures.
#include "ed25519_lane.h"

using namespace nwv;

namespace {

__device__ __forceinline__ void load_words8(const uint8_t* p, uint32_t w[8]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ __forceinline__ void store_words8(uint8_t* p, const uint32_t w[8]) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

}  // namespace

// btab (BTAB_WORDS): j B precomp entries (j = 0..128), one identity cached entry, then the
// j 2^128 B precomp entries (the per-signature check's half-size scalars, ed25519_lane.h)
extern "C" __global__ void __launch_bounds__(64) k_base_table(uint32_t* btab) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < BASE_TABLE_ENTRIES) {
        store_precomp_entry(btab + j * PRECOMP_ENTRY_WORDS, base_multiple(j));
        store_precomp_entry(btab + BASE128_TABLE_OFFSET + j * PRECOMP_ENTRY_WORDS, base128_multiple(j));
    }
    if (j == 0) store_cached_entry(btab + BASE_TABLE_WORDS, ge_cached_identity());
}

extern "C" __global__ void __launch_bounds__(256) k_ed_hash(
    uint64_t n, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, uint8_t* __restrict__ kbuf, uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t Aw[8], Rw[8], Sw[8], k[8];
    load_words8(pk + 32 * i, Aw);
    load_words8(sig + 64 * i, Rw);
    load_words8(sig + 64 * i + 32, Sw);
    flags[i] = lane_hash(Aw, Rw, Sw, msg + msg_off[i], msg_len[i], k);
    store_words8(kbuf + 32 * i, k);
}

// Two lanes per signature, in different waves: even waves decompress R (table entry
// R_ENTRY) for 64 signatures, odd waves decompress A and build entries 0..8 for the same 64.
// The role is wave-uniform (no divergence); the wave count doubles and each lane's chain
// halves.  Flags are combined with an atomic OR.
extern "C" __global__ void __launch_bounds__(256) k_ed_points(
    uint64_t n, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    uint32_t* __restrict__ tables, uint32_t* __restrict__ flags) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t wv = t >> 6;
    const uint64_t i = (wv >> 1) * 64 + (t & 63);
    if (i >= n) return;
    uint32_t w[8];
    uint32_t* tbl = tables + i * LANE_SCRATCH_WORDS;
    uint32_t f;
    if ((wv & 1) == 0) {
        load_words8(sig + 64 * i, w);
        f = lane_point_R(w, tbl);
    } else {
        load_words8(pk + 32 * i, w);
        f = lane_point_A(w, tbl);
    }
    atomicOr(flags + i, f);
}

template <bool PF>
__device__ __forceinline__ void ed_straus_body(uint64_t n, const uint8_t* __restrict__ sig,
                                               const uint8_t* __restrict__ kbuf, const uint32_t* __restrict__ tables,
                                               const uint32_t* __restrict__ flags, const uint32_t* __restrict__ btab,
                                               uint64_t* __restrict__ verdict, const uint32_t* __restrict__ gate) {
    // gate: a batch MSM's state words queued just before this pass; it accepted (word 1 == 1) ->
    // every signature is valid and the host reads no verdict bits (nothing to do)
    if (gate && gate[1] == 1u) return;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    bool ok = false;
    if (i < n) {
        uint32_t Sw[8], k[8];
        load_words8(sig + 64 * i + 32, Sw);
        load_words8(kbuf + 32 * i, k);
        const bool eq = lane_straus_check<PF>(k, Sw, tables + i * LANE_SCRATCH_WORDS, btab);
        ok = eq && flags[i] == FLAGS_ALL;
    }
    const uint64_t mask = __ballot(ok);
    if (lane == 0 && i - lane < n) verdict[i >> 6] = mask;
}
extern "C" __global__ void __launch_bounds__(256) k_ed_straus(
    uint64_t n, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ kbuf,
    const uint32_t* __restrict__ tables, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ btab, uint64_t* __restrict__ verdict, const uint32_t* __restrict__ gate) {
    ed_straus_body<false>(n, sig, kbuf, tables, flags, btab, verdict, gate);
}
// the same with each window's A / R table entries loaded one window ahead (more registers, fewer
// waves per SIMD): the default (C4 2.34 -> 2.29 ms, tools/gpurun/r4_c4_pf.sh); NWV_STRAUS_PF=0
// selects k_ed_straus
extern "C" __global__ void __launch_bounds__(256) k_ed_straus_pf(
    uint64_t n, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ kbuf,
    const uint32_t* __restrict__ tables, const uint32_t* __restrict__ flags,
    const uint32_t* __restrict__ btab, uint64_t* __restrict__ verdict, const uint32_t* __restrict__ gate) {
    ed_straus_body<true>(n, sig, kbuf, tables, flags, btab, verdict, gate);
}

// RFC 8032: a = clamp(SHA-512(seed)[0..32]), prefix = [32..64], A = [a]B,
// r = SHA-512(prefix || M) mod l, R = [r]B, k = SHA-512(R || A || M) mod l, S = r + k a mod l.
extern "C" __global__ void __launch_bounds__(256) k_sign(
    uint64_t n, const uint8_t* __restrict__ seeds, const uint8_t* __restrict__ msg,
    const uint64_t* __restrict__ msg_off, const uint32_t* __restrict__ msg_len,
    const uint32_t* __restrict__ btab, uint8_t* __restrict__ pk_out, uint8_t* __restrict__ sig_out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* ident = btab + BASE_TABLE_WORDS;
    uint32_t sw[8];
    load_words8(seeds + 32 * i, sw);
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
    ge_compress(straus_sB_minus_kA(zero, a, nullptr, btab, ident), Aw);
    const uint8_t* m = msg + msg_off[i];
    const uint32_t mlen = msg_len[i];
    sha512_prefixed_msg(st, prefix, m, mlen);
    uint32_t rh[16], r[8];
    sha512_digest_words(st, rh);
    sc_reduce512(rh, r);
    ge_compress(straus_sB_minus_kA(zero, r, nullptr, btab, ident), Rw);
    uint32_t k[8], ka[8], S[8];
    challenge_scalar(Rw, Aw, m, mlen, k);
    sc_mul(k, a, ka);
    sc_add(ka, r, S);
    store_words8(pk_out + 32 * i, Aw);
    store_words8(sig_out + 64 * i, Rw);
    store_words8(sig_out + 64 * i + 32, S);
}
