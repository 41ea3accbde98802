// msm_kernels.hip -- K5: batch verification as one Pippenger MSM per batch (gfx950).
//
// Pipeline (one batch resident on one device; layout of the 2n+1 points in msm.h):
//   k_msm_scalars   lane i: k_i = SHA-512(R||A||M) mod l, s_i < l, z_i = PRF(seed, i),
//                   scalars z_i k_i and z_i recoded to signed digits -> digits[w][.] (i16);
//                   per-workgroup partial sums of z_i s_i
//                   the last hash workgroup: b = -sum z_i s_i mod l and the basepoint term
//                   [8 b]B from a fixed-base comb table (msm.h), off the MSM
//   k_msm_points    2 lanes per signature (wave-uniform R / A roles): decompress, store the
//                   128-byte affine Niels record of each point
//   k_msm_hist      workgroup (chunk, window): LDS histogram of the window's bucket ids
//   k_msm_wscan     workgroup per window: its entry base, bucket totals, their scan, the
//                   (bucket, chunk) slice offsets
//   k_msm_scatter   workgroup (chunk, window), XCD-grouped: LDS cursors place j|sign into bucket
//                   order  (one-chunk batches: k_msm_sort1 does hist + scan + scatter per window)
//   k_msm_bucket    lane per fixed-size chunk of the sorted entries: key-segment sums (mixed
//                   additions, affine Niels), balanced whatever the bucket sizes
//   k_msm_tail      bucket pieces joined, window sums by bit-plane butterflies, each window scaled on 16-lane rows
//                   (fe_row.h) as soon as its sum is known, the sum over windows, [8], identity
//                   test -> batch verdict word (one launch)
// The counting sort keeps every histogram / cursor atomic in LDS; the only global atomics are
// the (rare) failure flags.  Entry order inside a bucket depends on LDS atomic order, which
// changes the projective representation of a bucket sum but never the group element, so the
// verdict is deterministic.
#include "fe_row.h"
#include "msm.h"

using namespace nwv;

namespace {

__device__ __forceinline__ void msm_load8(const uint8_t* p, uint32_t w[8]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
__device__ __forceinline__ void msm_store8(uint32_t* p, const uint32_t w[8]) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(w[0], w[1], w[2], w[3]);
    q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__device__ __forceinline__ fe fe_quad_bcast(const fe& a, int k) {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        switch (k) {
            case 0: r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], 0x00, 0xF, 0xF, false); break;
            case 1: r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], 0x55, 0xF, 0xF, false); break;
            case 2: r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], 0xAA, 0xF, 0xF, false); break;
            default: r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], 0xFF, 0xF, 0xF, false); break;
        }
    }
    return r;
}
__device__ __forceinline__ ge_p3 shfl_down_p3(const ge_p3& p, int o) {
    ge_p3 r;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        r.X.v[k] = (uint32_t)__shfl_down((int)p.X.v[k], o, 64);
        r.Y.v[k] = (uint32_t)__shfl_down((int)p.Y.v[k], o, 64);
        r.Z.v[k] = (uint32_t)__shfl_down((int)p.Z.v[k], o, 64);
        r.T.v[k] = (uint32_t)__shfl_down((int)p.T.v[k], o, 64);
    }
    return r;
}

}  // namespace

// digits: [window][na+1+n] signed digits of every point's scalar (A points at [0, na), B's
// entry na written by k_msm_bscalar, R_i at na+1+i); partial: gridDim.x x 9 words (sum of z_i s_i over the workgroup, as a
// plain 288-bit integer); fail: bit 0 set when any s_i >= l
struct MsmScalarArgs {
    uint64_t n, na;
    int keyed;
    const uint8_t* pk;
    const uint8_t* sig;
    const uint8_t* msg;
    const uint64_t* msg_off;
    const uint32_t* msg_len;
    const uint32_t* seedp;
    uint32_t* ascal;
    int16_t* digits;
    uint32_t* partial;
    uint32_t* fail;
    // B is not an MSM point (its term comes from the fixed-base comb, k_msm_tail): workgroup 0
    // zeroes its digit column (point na, and na - 1 = 2^128 B's column of the key-cache form)
    uint32_t split;
    uint32_t* tail_ctr;  // k_msm_tail's arrival counters (128 words), zeroed by workgroup 0
    // batches over per-signature keys: k_i and the s < l flag for the per-signature fallback
    // (k_ed_hash's outputs, so a rejected batch's exact-bad-set pass skips the hashing), or null
    uint32_t* kout;
    uint32_t* fout;
    // 1: OR the flag into fout (zeroed at staging; the early form's k_ed_points_msm ORs its decode
    // flags into the same words concurrently), 0: store it
    uint32_t fout_or;
    // fuse_keysum: a keyed batch whose hashes fit ONE workgroup (n <= its threads, nkeys <= its
    // threads) sums its keys' scalars in that workgroup after the hashes (k_msm_keysum's work,
    // thread j = key j), under the decompressions running beside it in the same grid: one launch
    // and its hand-off fewer on the per-call path (C1 Certificate::verify)
    uint32_t fuse_keysum;
    uint32_t nkeys;
    const uint32_t* key_off;  // CSR of the keys' signatures (k_msm_keysum's key_off / key_sig)
    const uint32_t* key_sig;
    const uint32_t* kslot;    // split form: the keys' cache slots, the cache, the point records
    const uint32_t* kc;
    uint32_t* pts;
};

// A key's scalar (8 column sums of 32-bit words, each < 2^64) reduced mod l and recoded into its
// digit row(s): row `key`, and in the split form (kc) the 2^128 multiple's row m + key
__device__ __forceinline__ void msm_key_digits(const unsigned long long* colsum, uint32_t key, uint32_t m,
                                               uint64_t np, bool split, const MsmLayout& lay,
                                               int16_t* __restrict__ digits) {
    uint32_t x[16];
    unsigned long long c = 0;
    for (int k = 0; k < 16; k++) {
        if (k < 8) {
            const unsigned long long v = colsum[k];
            const unsigned long long lo = (c & 0xffffffffull) + (v & 0xffffffffull);
            x[k] = (uint32_t)lo;
            c = (c >> 32) + (v >> 32) + (lo >> 32);
        } else {
            x[k] = (uint32_t)c;
            c >>= 32;
        }
    }
    uint32_t r[8];
    sc_reduce512(x, r);
    if (split) {
        uint32_t lo[8], hi[8];
        msm_split128(r, lo, hi);
        msm_recode(lo, lay, lay.nw_z, [&](int w, int d) { digits[(uint64_t)w * np + key] = (int16_t)d; });
        msm_recode(hi, lay, lay.nw_z, [&](int w, int d) { digits[(uint64_t)w * np + m + key] = (int16_t)d; });
    } else {
        msm_recode(r, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + key] = (int16_t)d; });
    }
}

// word t < 2 MSM_PT_WORDS of a cached key's records (A, then 2^128 A) into points key and m + key;
// the record's last word set = the key did not decode
__device__ __forceinline__ void msm_key_record_word(const uint32_t* __restrict__ kc, const uint32_t* __restrict__ kslot,
                                                    uint32_t key, uint32_t m, uint32_t t, uint32_t* __restrict__ pts,
                                                    uint32_t* fail) {
    const uint32_t* src = kc + (size_t)KC_SLOT_WORDS * kslot[key];
    pts[(size_t)MSM_PT_WORDS * (t < MSM_PT_WORDS ? key : m + key) + (t % MSM_PT_WORDS)] = src[t];
    if (t == MSM_PT_WORDS - 1 && src[t]) atomicOr(fail, 2u);
}
struct MsmPointArgs {
    uint64_t n, na;
    uint64_t ndec;  // A points to decompress into [0, ndec): na, or 0 when they come from the key cache
    const uint8_t* apk;
    const uint8_t* sig;
    uint32_t* pts;
    uint32_t* fail;
    uint32_t rows;  // 1: the row form (msm_points_rows_block, 16 points per workgroup)
};

__device__ __forceinline__ void msm_scalars_block(uint32_t blk, const MsmScalarArgs& g, const MsmLayout& lay) {
    const uint64_t n = g.n, na = g.na;
    const uint8_t* __restrict__ pk = g.pk;
    const uint8_t* __restrict__ sig = g.sig;
    const uint8_t* __restrict__ msg = g.msg;
    const uint32_t* __restrict__ seedp = g.seedp;
    int16_t* __restrict__ digits = g.digits;
    uint32_t* __restrict__ fail = g.fail;
    const int keyed = g.keyed;
    __shared__ uint32_t zs_lds[256 * 9];
    const uint32_t nt = blockDim.x;  // 256, or 64 when the call's decompression runs on rows
    const uint64_t i = (uint64_t)blk * nt + threadIdx.x;
    uint32_t zs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (i < n) {
        uint32_t Aw[8], Rw[8], Sw[8], k[8], z[8], a[8];
        msm_load8(pk + 32 * i, Aw);
        msm_load8(sig + 64 * i, Rw);
        msm_load8(sig + 64 * i + 32, Sw);
        const uint32_t f = lane_hash(Aw, Rw, Sw, msg + g.msg_off[i], g.msg_len[i], k);
        if (f != FLAG_S_OK) atomicOr(fail, 1u);
        if (g.kout) {
            msm_store8(g.kout + 8 * i, k);
            if (g.fout_or) atomicOr(g.fout + i, f);
            else g.fout[i] = f;
        }
        uint32_t sd[8];
#pragma unroll
        for (int k = 0; k < 8; k++) sd[k] = seedp[k];
        msm_z(sd, i, z);
        sc_mul(z, k, a);
        sc_mul(z, Sw, zs);
        // signed digits straight from registers (window-major rows): R_i always; A_i's scalar
        // z_i k_i here when every signature has its own A point, else summed per key by
        // k_msm_keysum first
        const uint64_t np = na + 1 + n;
        if (keyed) msm_store8(g.ascal + 8 * i, a);
        else msm_recode(a, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + i] = (int16_t)d; });
        msm_recode(z, lay, lay.nw_z, [&](int w, int d) { digits[(uint64_t)w * np + na + 1 + i] = (int16_t)d; });
    }
#pragma unroll
    for (int k = 0; k < 8; k++) zs_lds[threadIdx.x * 9 + k] = zs[k];
    __syncthreads();
    // column sums: thread t < 8 adds word t of the nt values (< 2^40), then thread 0 carries
    __shared__ unsigned long long col[8];
    if (threadIdx.x < 8) {
        unsigned long long s = 0;
        for (uint32_t r = 0; r < nt; r++) s += zs_lds[r * 9 + threadIdx.x];
        col[threadIdx.x] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long c = 0;
        uint32_t* out = g.partial + 9 * blk;
        for (int k = 0; k < 8; k++) {
            c += col[k];
            out[k] = (uint32_t)c;
            c >>= 32;
        }
        out[8] = (uint32_t)c;
    }
    if (blk == 0 && threadIdx.x < (unsigned)lay.nw) {  // B's digit column(s) stay empty
        const uint64_t np = na + 1 + n;
        digits[(uint64_t)threadIdx.x * np + na] = 0;
        if (g.split) digits[(uint64_t)threadIdx.x * np + na - 1] = 0;
    }
    if (blk == 0)  // (no memset launch)
        for (uint32_t t = threadIdx.x; t < 128; t += nt) g.tail_ctr[t] = 0u;
    if (g.fuse_keysum) {  // (the host sets it only for a grid with one hash workgroup)
        __syncthreads();  // every z_i k_i of ascal is written (one workgroup: one CU)
        const uint32_t m = g.nkeys;
        if (g.kc)
            for (uint32_t t = threadIdx.x; t < 2u * MSM_PT_WORDS * m; t += nt)
                msm_key_record_word(g.kc, g.kslot, t / (2 * MSM_PT_WORDS), m, t % (2 * MSM_PT_WORDS), g.pts, fail);
        if (threadIdx.x < m) {
            const uint32_t key = threadIdx.x;
            unsigned long long cs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (uint32_t t = g.key_off[key]; t < g.key_off[key + 1]; t++) {
                const uint32_t* a = g.ascal + 8 * (size_t)g.key_sig[t];
#pragma unroll
                for (int k = 0; k < 8; k++) cs[k] += a[k];
            }
            msm_key_digits(cs, key, m, na + 1 + n, g.kc != nullptr, lay, digits);
        }
    }
}

// Keyed batches (ed25519_consensus groups batch entries by verification key): one workgroup per
// distinct key sums z_i k_i over its signatures (CSR: key_off[m+1], key_sig[n]), reduces mod l
// and writes the key point's digits (row entry = key index).
//
// Split form (kc != null, committee key cache): the key's record and its 2^128 multiple's come
// from cache slot kslot[key] and go to points key and m + key, with the 128-bit halves of the
// key's scalar (K = lo + 2^128 hi), so every scalar of the MSM fits the z range (layout with
// nw == nw_z: half the windows and half the final doubling chain).
extern "C" __global__ void __launch_bounds__(256) k_msm_keysum(
    uint64_t n, uint64_t na, MsmLayout lay, const uint32_t* __restrict__ key_off,
    const uint32_t* __restrict__ key_sig, const uint32_t* __restrict__ ascal, int16_t* __restrict__ digits,
    uint32_t m, const uint32_t* __restrict__ kslot, const uint32_t* __restrict__ kc, uint32_t* __restrict__ pts,
    uint32_t* __restrict__ fail) {
    __shared__ unsigned long long col[256 * 9];
    __shared__ unsigned long long part[32 * 8];
    const uint32_t key = blockIdx.x;
    if (kc && threadIdx.x < 2 * MSM_PT_WORDS) msm_key_record_word(kc, kslot, key, m, threadIdx.x, pts, fail);
    unsigned long long s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t t = key_off[key] + threadIdx.x; t < key_off[key + 1]; t += 256) {
        const uint32_t* a = ascal + 8 * (size_t)key_sig[t];
#pragma unroll
        for (int k = 0; k < 8; k++) s[k] += a[k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) col[threadIdx.x * 9 + k] = s[k];
    __syncthreads();
    // column sums over the rows that hold signatures (a committee key signs one or a few of a
    // call's messages): 32 partial sums a column, then 8 threads add the 32 (< 2^(32+32)); one
    // thread walking all 256 rows was a 256-long dependent LDS chain (~10 us)
    const uint32_t cnt = key_off[key + 1] - key_off[key], rows = cnt < 256u ? cnt : 256u;
    {
        const uint32_t c = threadIdx.x & 7, p0 = threadIdx.x >> 3;
        unsigned long long t = 0;
        for (uint32_t r = p0; r < rows; r += 32) t += col[r * 9 + c];
        part[p0 * 8 + c] = t;
    }
    __syncthreads();
    if (threadIdx.x < 8) {
        unsigned long long t = 0;
        const uint32_t np = rows < 32u ? rows : 32u;
        for (uint32_t r = 0; r < np; r++) t += part[r * 8 + threadIdx.x];
        col[threadIdx.x] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) msm_key_digits(col, key, m, na + 1 + n, kc != nullptr, lay, digits);
}

// One-time per device: the fixed-base comb table, entry 8 j + i - 1 = i 16^j B (msm.h)
extern "C" __global__ void __launch_bounds__(64) k_comb_table(uint32_t* comb) {
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= COMB_TABLES * COMB_ENTRIES) return;
    comb_entry(e / COMB_ENTRIES, e % COMB_ENTRIES + 1, comb + MSM_PT_WORDS * e);
}

// Committee key cache fill: lane i decompresses keys[i] into slot slots[i] = { A's MSM point
// record | 2^128 A's record }, word 31 = 1 when A does not decode (checked by k_msm_keysum).
// 2^128 A: 128 doublings, then one inversion to the affine record.  Runs once per new key.
extern "C" __global__ void __launch_bounds__(64) k_keycache_fill(uint32_t cnt, const uint8_t* __restrict__ keys,
                                                                 const uint32_t* __restrict__ slots,
                                                                 uint32_t* __restrict__ cache) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= cnt) return;
    uint32_t w[8];
    msm_load8(keys + 32 * (size_t)i, w);
    ge_p3 P;
    const bool ok = ge_decompress(w, P);
    uint32_t* e = cache + (size_t)KC_SLOT_WORDS * slots[i];
    msm_store_point(e, P);
    e[MSM_PT_WORDS - 1] = ok ? 0u : 1u;
    const ge_precomp q = ge_p3_to_precomp(p3_dbl_n(P, 128));
    store_fe(e + MSM_PT_WORDS, q.ypx);
    store_fe(e + MSM_PT_WORDS + 10, q.ymx);
    store_fe(e + MSM_PT_WORDS + 20, q.xy2d);
    e[MSM_PT_WORDS + 30] = 0u;
    e[MSM_PT_WORDS + 31] = 0u;
}

// Decompression, wave-uniform roles: waves [0, ceil(n/64)) decompress R_i into point na+1+i,
// the following ceil(na/64) waves decompress the A points (apk: per-signature keys, or the
// distinct keys of a keyed batch) into points [0, na).
__device__ __forceinline__ void msm_points_block(uint32_t blk, const MsmPointArgs& g) {
    const uint64_t n = g.n, na = g.na;
    const uint64_t t = (uint64_t)blk * blockDim.x + threadIdx.x;
    const uint64_t rwaves = (n + 63) / 64;
    const bool is_r = (t >> 6) < rwaves;
    const uint64_t i = is_r ? t : t - 64 * rwaves;
    if (i >= (is_r ? n : g.ndec)) return;
    uint32_t w[8];
    msm_load8(is_r ? g.sig + 64 * i : g.apk + 32 * i, w);
    ge_p3 P;
    const bool ok = ge_decompress(w, P);
    uint32_t* e = g.pts + (size_t)MSM_PT_WORDS * (is_r ? na + 1 + i : i);
    msm_store_point(e, P);
    e[MSM_PT_WORDS - 1] = ok ? 0u : 1u;  // decode flag (k_ed_points_msm); ignored by the MSM
    if (!ok) atomicOr(g.fail, 2u);
}

// Small (latency-bound) batches: the same decompression (ge25519.h ge_decompress) on 16-lane rows
// (fe_row.h, rotation-form products), one point per row, four per wave.  Point j of the call:
// R_j (into na + 1 + j) for j < n, then the A points (into j - n).  Every product -- the prelude
// u v^7, the power (250 squarings, 11 multiplies), the root and its square-root test, the record's
// 2d x y -- is a row product (~0.13 us) instead of a lane-local one (~0.3 us); only the canonical
// tests (three zero tests side by side on lanes 0..2 of the row, the root's sign on lane 0) and the
// record's conversion to ten-limb form (lanes 0..2, one coordinate each) are lane-local, handed
// through 48 words of LDS per row.  The call launches k_msm_prep with 64-thread workgroups: four
// such waves on one CU (one per SIMD) decompressed in 62 us against 52 us for single-wave
// workgroups spread over the chip (512 waves, tools/ubench_prep.hip, profiles/round5_ubench_prep.jsonl).
#if defined(__HIP_DEVICE_COMPILE__)  // (rowf's lane type is the host emulation's wave elsewhere)
// ge_decompress on the 16-lane row that holds limb `limb` of an encoding in y16 (bit 15 of limb 15
// is x's sign): leaves the affine Niels record -- y + x, y - x, 2 d x y as 16-limb rows -- in
// sh[0, 48) (this row's 48 words of LDS) and returns whether the encoding decodes (row-uniform).
// Every lane of the wave calls it (the products are DPP row operations).
__device__ __forceinline__ bool row_decompress(uint32_t y16, int lane, int row, int limb, uint32_t* sh) {
    const bool sign = (__shfl(y16, (lane & ~15) + 15) >> 15) != 0u;
    if (limb == 15) y16 &= 0x7FFFu;
    rowf::RowConsts k = rowf::row_consts();
    k.rot = 1;
    uint32_t u, v, uv3, uv7;
    rowf::row_dec_pre(y16, k, u, v, uv3, uv7);
    const uint32_t pw = rowf::row_pow_p58(uv7, k);
    uint32_t r, ri, c0, c1, c2;
    rowf::row_dec_mid(uv3, pw, u, v, k, r, ri, c0, c1, c2);
    // square-root test: zero tests of check - u, check + u, check + u sqrt(-1) on lanes 0..2
    sh[limb] = c0;
    sh[16 + limb] = c1;
    sh[32 + limb] = c2;
    rowf::lds_order();
    bool z = false;
    if (limb < 3) z = fe_is_zero(fe_from_limbs16(sh + 16 * limb));
    const uint32_t rz = (uint32_t)(__ballot(z) >> (16 * row)) & 7u;
    const bool ok = (rz & 3u) != 0u;  // correct (check = u) or flipped (check = -u)
    const uint32_t rr = (rz & 6u) ? ri : r;
    // the root made non-negative, then negated by the sign bit: x = rr or -rr
    rowf::lds_order();
    sh[limb] = rr;
    rowf::lds_order();
    bool neg = false;
    if (limb == 0) neg = fe_is_negative(fe_from_limbs16(sh));
    const bool negr = ((__ballot(neg) >> (16 * row)) & 1u) != 0u;
    const uint32_t x = negr != sign ? rowf::carry32(rowf::sub(0u, rr, k), k) : rr;
    uint32_t ypx, ymx, xy2d;
    rowf::row_dec_record(x, y16, k, ypx, ymx, xy2d);
    rowf::lds_order();
    sh[limb] = ypx;
    sh[16 + limb] = ymx;
    sh[32 + limb] = xy2d;
    rowf::lds_order();
    return ok;
}
#endif

__device__ __forceinline__ void msm_points_rows_block(uint32_t blk, const MsmPointArgs& g) {
#if defined(__HIP_DEVICE_COMPILE__)  // (rowf's lane type is the host emulation's wave elsewhere)
    __shared__ uint32_t rl[4 * 192];  // per wave: 4 rows x 48 words
    const uint64_t n = g.n, na = g.na, tot = n + g.ndec;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, row = lane >> 4, limb = lane & 15;
    const uint64_t wave = (uint64_t)blk * (blockDim.x >> 6) + wv;  // 4 points per wave
    if (wave * 4 >= tot) return;                                   // whole wave past the end (wave-uniform)
    uint32_t* sh = rl + 192 * wv + 48 * row;                       // this row's 48 words
    const uint64_t j = wave * 4 + row;
    const bool live = j < tot;
    // limb `limb` of the encoding (bit 255: the sign of x)
    uint32_t y16 = 0u;
    if (live) y16 = reinterpret_cast<const uint16_t*>(j < n ? g.sig + 64 * j : g.apk + 32 * (j - n))[limb];
    const bool ok = row_decompress(y16, lane, row, limb, sh);
    if (live && limb < 3) {
        uint32_t* e = g.pts + (size_t)MSM_PT_WORDS * (j < n ? na + 1 + j : j - n);
        store_fe(e + 10 * limb, fe_from_limbs16(sh + 16 * limb));
        if (limb == 0) {
            e[30] = 0u;
            e[MSM_PT_WORDS - 1] = ok ? 0u : 1u;
            if (!ok) atomicOr(g.fail, 2u);
        }
    }
#endif
}

// C4 fallback after a rejected batch MSM over per-signature keys: the per-signature tables
// (k_ed_points' 0..8 R and 0..8 A tables) built from the MSM's decompressed point records instead
// of a second decompression.  Record (y+x | y-x | 2dxy, Z = 1) -> x = ((y+x) - (y-x)) / 2,
// y = ((y+x) + (y-x)) / 2, T = xy; word 31 is the record's decode flag.  Same two lanes per
// signature, in different waves, as k_ed_points.
extern "C" __global__ void __launch_bounds__(256) k_ed_points_msm(uint64_t n, uint64_t na,
                                                                  const uint32_t* __restrict__ pts,
                                                                  uint32_t* __restrict__ tables,
                                                                  uint32_t* __restrict__ flags) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t wv = t >> 6;
    const uint64_t i = (wv >> 1) * 64 + (t & 63);
    if (i >= n) return;
    const bool is_r = (wv & 1) == 0;
    const uint32_t* e = pts + (size_t)MSM_PT_WORDS * (is_r ? na + 1 + i : i);
    const uint32_t half_w[8] = {0xFFFFFFF7u, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x3FFFFFFFu};  // (p + 1) / 2
    const fe half = fe_from_words(half_w);
    const fe ypx = load_fe(e), ymx = load_fe(e + 10);
    ge_p3 P;
    P.X = fe_mul(fe_sub(ypx, ymx), half);
    P.Y = fe_mul(fe_add(ypx, ymx), half);
    P.Z = fe_one();
    P.T = fe_mul(P.X, P.Y);
    uint32_t* tbl = tables + i * LANE_SCRATCH_WORDS;
    build_a_table(P, is_r ? tbl + R_ENTRY * CACHED_ENTRY_WORDS : tbl);  // j R or j A, j = 0..8
    const uint32_t f = e[MSM_PT_WORDS - 1] == 0 ? (is_r ? FLAG_R_OK : FLAG_A_OK) : 0u;
    atomicOr(flags + i, f);
}

extern "C" __global__ void __launch_bounds__(256) k_msm_scalars(MsmScalarArgs g, MsmLayout lay) {
    msm_scalars_block(blockIdx.x, g, lay);
}
extern "C" __global__ void __launch_bounds__(256) k_msm_points(MsmPointArgs g) {
    if (g.rows) msm_points_rows_block(blockIdx.x, g);
    else msm_points_block(blockIdx.x, g);
}
// Both in one grid: blocks [0, sblocks) hash / recode (one wave per SIMD at 65,536 signatures,
// latency-bound on its own), the rest decompress; sharing the SIMDs lets the decompression
// waves fill the hash waves' issue gaps.
extern "C" __global__ void __launch_bounds__(256) k_msm_prep(MsmScalarArgs gs, MsmLayout lay, MsmPointArgs gp,
                                                             uint32_t sblocks) {
    if (blockIdx.x < sblocks) msm_scalars_block(blockIdx.x, gs, lay);
    else if (gp.rows) msm_points_rows_block(blockIdx.x - sblocks, gp);
    else msm_points_block(blockIdx.x - sblocks, gp);
}

// points of window w: all na+1+n below nw_z, else the prefix [0, na] (A points and B)
__device__ __forceinline__ uint64_t msm_window_points(uint64_t n, uint64_t na, int w, int nw_z) {
    return w < nw_z ? na + 1 + n : na + 1;
}

// grid (chunks, windows); counts laid out window by window, chunk-major inside a window:
// cnt[kbase[w] * chunks + chunk * nb_w + b], so every workgroup stores one contiguous run; the
// workgroup's nonzero digits -> nzc[w * chunks + chunk] (the windows' entry bases, k_msm_wscan)
//
// Two-level sort (large batches, msm.h MsmSort2): lay is the coarse layout (widths reduced by
// shift) and every digit counts in bin (|d| - 1) >> shift; k_msm_scatter then writes packed
// entries (msm_pack2) that k_msm_lsort orders by the remaining low bits.
// A batch whose prep flagged a failed decoding or an s >= l is rejected by k_msm_tail whatever the
// sum is, so the kernels in between skip their work: the reference's batch verifier returns its
// error before the multiscalar multiplication too.  (Plain load: the flag
// was written by an earlier kernel of the same stream.)
__device__ __forceinline__ bool msm_failed(const uint32_t* fail) { return *fail != 0u; }

extern "C" __global__ void __launch_bounds__(256) k_msm_hist(
    uint64_t n, uint64_t na, MsmLayout lay, uint32_t chunk_pts, const int16_t* __restrict__ digits,
    uint32_t* __restrict__ cnt, uint32_t* __restrict__ nzc, int shift, const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    extern __shared__ uint32_t hist[];
    __shared__ uint32_t nz;
    const int w = blockIdx.y, nw_z = lay.nw_z, nb = 1 << (lay.width[w] - 1);
    const uint32_t chunks = gridDim.x, chunk = blockIdx.x;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) hist[b] = 0;
    if (threadIdx.x == 0) nz = 0;
    __syncthreads();
    const uint64_t np = na + 1 + n, cnt_w = msm_window_points(n, na, w, nw_z);
    const uint64_t lo = (uint64_t)chunk * chunk_pts;
    const uint64_t hi = lo + chunk_pts < cnt_w ? lo + chunk_pts : cnt_w;
    const int16_t* dw = digits + (uint64_t)w * np;
    uint32_t mine = 0;
    for (uint64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
        const int d = dw[j];
        if (d) {
            atomicAdd(&hist[((d < 0 ? -d : d) - 1) >> shift], 1u);
            mine++;
        }
    }
    atomicAdd(&nz, mine);
    __syncthreads();
    uint32_t* out = cnt + (uint64_t)lay.kbase[w] * chunks + (uint64_t)chunk * nb;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) out[b] = hist[b];
    if (threadIdx.x == 0) nzc[(uint64_t)w * chunks + chunk] = nz;
}

// ---- per-window scans: window w's entries start at ebase_w = the nonzero digits of the windows
// before it, so the windows sort independently and the entries stay packed ----------------------
// exclusive scan of one value per thread over the workgroup (wave prefix sums by shuffles, one
// LDS word per wave); every thread gets its prefix and the workgroup total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const int t = threadIdx.x, wid = t >> 6, lane = t & 63, nwaves = blockDim.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int k = 0; k < nwaves; k++) {
        const uint32_t s = wsum[k];
        pre += k < wid ? s : 0u;
        tot += s;
    }
    __syncthreads();  // wsum may be rewritten by the next call
    total = tot;
    return pre + inc - v;
}

// sum of one value per thread over the workgroup
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* wsum) {
    uint32_t total;
    (void)block_excl_scan(v, wsum, total);
    return total;
}

// grid (nw), 1024 threads: the window's entry base (nonzero digits of the windows before it, from
// k_msm_hist's per-chunk counts), its bucket totals over the chunks and their exclusive scan
// (1024 buckets per step); the counts become absolute slice offsets in place:
// cnt[(b, ch)] = ebase + (entries of buckets < b) + (entries of bucket b in chunks < ch);
// kstart[key] = the bucket's first entry.  The last window stores the total (tot[nw]) and
// every window its own count (tot[w]).
extern "C" __global__ void __launch_bounds__(1024) k_msm_wscan(
    MsmLayout lay, uint32_t chunks, uint32_t* __restrict__ cnt, const uint32_t* __restrict__ nzc,
    uint32_t* __restrict__ kstart, uint32_t* __restrict__ tot_out, const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    __shared__ uint32_t wsum[16];
    const int w = blockIdx.x, nb = 1 << (lay.width[w] - 1);
    uint32_t before = 0;
    for (uint32_t i = threadIdx.x; i < (uint32_t)w * chunks; i += blockDim.x) before += nzc[i];
    const uint32_t ebase = block_sum(before, wsum);
    uint32_t* c = cnt + (uint64_t)lay.kbase[w] * chunks;
    uint32_t carry = 0;
    for (int b0 = 0; b0 < nb; b0 += (int)blockDim.x) {
        const int b = b0 + (int)threadIdx.x;
        uint32_t tot = 0;
        if (b < nb) {
            // eight independent loads in flight per step (a sequential chain of loads per lane
            // was latency-bound)
            uint32_t ch = 0;
            for (; ch + 8 <= chunks; ch += 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = c[(uint64_t)(ch + u) * nb + b];
#pragma unroll
                for (int u = 0; u < 8; u++) tot += v[u];
            }
            for (; ch < chunks; ch++) tot += c[(uint64_t)ch * nb + b];
        }
        uint32_t step;
        const uint32_t ex = block_excl_scan(tot, wsum, step);
        if (b < nb) {
            uint32_t o = ebase + carry + ex;
            kstart[lay.kbase[w] + b] = o;
            uint32_t ch = 0;
            for (; ch + 8 <= chunks; ch += 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = c[(uint64_t)(ch + u) * nb + b];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    c[(uint64_t)(ch + u) * nb + b] = o;
                    o += v[u];
                }
            }
            for (; ch < chunks; ch++) {
                const uint32_t v = c[(uint64_t)ch * nb + b];
                c[(uint64_t)ch * nb + b] = o;
                o += v;
            }
        }
        carry += step;
    }
    if (threadIdx.x == 0) {
        tot_out[w] = carry;
        if (w == lay.nw - 1) tot_out[MSM_MAX_WINDOWS] = ebase + carry;
    }
}

// Small batches (one chunk per window): the whole sort of window w in ONE workgroup of 1024 --
// its entry base (the nonzero digits of the earlier windows, counted here from their digit
// rows: at most 8,192 points each), LDS histogram, scan, kstart, LDS cursors, scatter
// (replaces hist + scan + scatter)
extern "C" __global__ void __launch_bounds__(1024) k_msm_sort1(
    uint64_t n, uint64_t na, MsmLayout lay, const int16_t* __restrict__ digits, uint32_t* __restrict__ kstart,
    uint32_t* __restrict__ tot_out, uint32_t* __restrict__ entries, uint32_t seg, uint32_t* __restrict__ seg_key,
    const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    extern __shared__ uint32_t cur[];
    __shared__ uint32_t wsum[16];
    const int w = blockIdx.x, nb = 1 << (lay.width[w] - 1);
    const uint64_t np = na + 1 + n;
    // nonzero digits of the earlier windows: full rows below nw_z are one contiguous run
    // (16-byte loads, eight digits each), the rows above it hold na + 1 digits each
    uint32_t before = 0;
    {
        const uint64_t run = (uint64_t)(w < lay.nw_z ? w : lay.nw_z) * np;
        const uint4* q = reinterpret_cast<const uint4*>(digits);
        const uint64_t nq = run / 8;
        auto nz2 = [](uint32_t x) { return ((x & 0xFFFFu) != 0u) + ((x >> 16) != 0u); };
#pragma unroll 4
        for (uint64_t i = threadIdx.x; i < nq; i += blockDim.x) {
            const uint4 v = q[i];
            before += nz2(v.x) + nz2(v.y) + nz2(v.z) + nz2(v.w);
        }
        for (uint64_t j = 8 * nq + threadIdx.x; j < run; j += blockDim.x) before += digits[j] != 0;
        const uint64_t upper = w > lay.nw_z ? (uint64_t)(w - lay.nw_z) * (na + 1) : 0;
#pragma unroll 4
        for (uint64_t i = threadIdx.x; i < upper; i += blockDim.x) {
            const uint64_t v = lay.nw_z + i / (na + 1), j = i % (na + 1);
            before += digits[v * np + j] != 0;
        }
    }
    const uint32_t ebase = block_sum(before, wsum);
    const uint64_t cap = msm_window_points(n, na, w, lay.nw_z);
    const int16_t* dw = digits + (uint64_t)w * np;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) cur[b] = 0;
    __syncthreads();
    for (uint64_t j = threadIdx.x; j < cap; j += blockDim.x) {
        const int d = dw[j];
        if (d) atomicAdd(&cur[(d < 0 ? -d : d) - 1], 1u);
    }
    __syncthreads();
    uint32_t carry = 0;
    for (int b0 = 0; b0 < nb; b0 += (int)blockDim.x) {
        const int b = b0 + (int)threadIdx.x;
        const uint32_t v = b < nb ? cur[b] : 0u;
        uint32_t step;
        const uint32_t ex = block_excl_scan(v, wsum, step);
        if (b < nb) {
            const uint32_t o = ebase + carry + ex;
            cur[b] = o;
            kstart[lay.kbase[w] + b] = o;
        }
        carry += step;
    }
    __syncthreads();
    // the bucket each bucket lane of k_msm_bucket[_q] starts in (segment g = entries [g seg, ...)):
    // written here from the bucket offsets instead of a binary search of kstart per lane
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const uint32_t s0 = cur[b], e0 = b + 1 < nb ? cur[b + 1] : ebase + carry;
        for (uint32_t g = (s0 + seg - 1) / seg; g * seg < e0; g++) seg_key[g] = lay.kbase[w] + (uint32_t)b;
    }
    __syncthreads();
    for (uint64_t j = threadIdx.x; j < cap; j += blockDim.x) {
        const int d = dw[j];
        if (d) {
            const uint32_t slot = atomicAdd(&cur[(d < 0 ? -d : d) - 1], 1u);
            entries[slot] = (uint32_t)j | (d < 0 ? MSM_NEG : 0u);
        }
    }
    if (threadIdx.x == 0) {
        tot_out[w] = carry;
        if (w == lay.nw - 1) tot_out[MSM_MAX_WINDOWS] = ebase + carry;
    }
}

// grid MSM_XCD_GROUPS x xm.slots: workgroup b runs chunk s of the windows of group b % 8 (msm.h
// MsmXcdMap), s counted over those windows in order; chunks = the plan's chunks per window
// (the stride of the offsets)
extern "C" __global__ void __launch_bounds__(256) k_msm_scatter(
    uint64_t n, uint64_t na, MsmLayout lay, MsmXcdMap xm, uint32_t chunks, uint32_t chunk_pts,
    const int16_t* __restrict__ digits, const uint32_t* __restrict__ off, uint32_t* __restrict__ entries,
    int shift, const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    extern __shared__ uint32_t cur[];
    const uint32_t g = blockIdx.x % MSM_XCD_GROUPS;
    uint32_t s = blockIdx.x / MSM_XCD_GROUPS;
    int w = -1;
    for (int k = 0; k < xm.nwin[g]; k++) {
        const int wk = xm.win[g][k];
        const uint32_t c = msm_window_chunks(n, na, wk, lay.nw_z, chunk_pts);
        if (s < c) {
            w = wk;
            break;
        }
        s -= c;
    }
    if (w < 0) return;  // uniform over the workgroup: no barrier reached
    const int nw_z = lay.nw_z, nb = 1 << (lay.width[w] - 1);
    const uint32_t chunk = s;
    const uint32_t* mine = off + (uint64_t)lay.kbase[w] * chunks + (uint64_t)chunk * nb;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) cur[b] = mine[b];
    __syncthreads();
    const uint64_t np = na + 1 + n, cnt_w = msm_window_points(n, na, w, nw_z);
    const uint64_t lo = (uint64_t)chunk * chunk_pts;
    const uint64_t hi = lo + chunk_pts < cnt_w ? lo + chunk_pts : cnt_w;
    const int16_t* dw = digits + (uint64_t)w * np;
    for (uint64_t j = lo + threadIdx.x; j < hi; j += blockDim.x) {
        const int d = dw[j];
        if (d) {
            const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
            const uint32_t slot = atomicAdd(&cur[b >> shift], 1u);
            entries[slot] = shift ? msm_pack2((uint32_t)j, b, d < 0, shift) : ((uint32_t)j | (d < 0 ? MSM_NEG : 0u));
        }
    }
}

// Second level of the two-level sort: workgroup (s, w) orders coarse bin s of window w -- the
// entries of buckets [s << shift, (s + 1) << shift), contiguous in mid after the first level --
// by their low bucket bits, writing the final entries (j | sign) into the same index range of
// entries and the buckets' start offsets.  The whole range is written by one workgroup (LDS
// cursors), so its lines are written whole.
extern "C" __global__ void __launch_bounds__(256) k_msm_lsort(
    MsmLayout lay, MsmLayout lay2, int shift, const uint32_t* __restrict__ mid, const uint32_t* __restrict__ kst2,
    const uint32_t* __restrict__ tot, uint32_t* __restrict__ entries, uint32_t* __restrict__ kstart,
    const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    __shared__ uint32_t cur[1 << MSM_SORT2_MAX_SHIFT];
    __shared__ uint32_t wsum[4];
    const int w = blockIdx.y, s = blockIdx.x;
    const int nb2 = 1 << (lay2.width[w] - 1), nlo = 1 << shift;
    if (s >= nb2) return;  // whole workgroup
    const uint32_t key2 = lay2.kbase[w] + s;
    const uint32_t lo = kst2[key2];
    const uint32_t hi = key2 + 1 < lay2.kbase[lay2.nw] ? kst2[key2 + 1] : tot[MSM_MAX_WINDOWS];
    const int t = threadIdx.x;
    if (t < nlo) cur[t] = 0;
    __syncthreads();
    for (uint32_t k = lo + t; k < hi; k += 256) atomicAdd(&cur[msm_unpack2_low(mid[k], shift)], 1u);
    __syncthreads();
    uint32_t total;
    const uint32_t v = t < nlo ? cur[t] : 0u;
    const uint32_t ex = block_excl_scan(v, wsum, total);
    if (t < nlo) {
        cur[t] = lo + ex;
        kstart[lay.kbase[w] + ((uint32_t)s << shift) + t] = lo + ex;
    }
    __syncthreads();
    for (uint32_t k = lo + t; k < hi; k += 256) {
        const uint32_t e = mid[k];
        const uint32_t slot = atomicAdd(&cur[msm_unpack2_low(e, shift)], 1u);
        entries[slot] = msm_unpack2_entry(e, shift);
    }
}

// ---- bucket sums: fixed-size chunks of the sorted entries ---------------------------------
// Lane q adds the entries [qT, qT + T) (mixed additions of affine Niels points, the next point's
// words loaded while the current one is added).  Each key segment that ends inside the chunk is
// written out: to bsum[key] if the key starts in this chunk (complete, or the key's first piece),
// else to hpart[q] (a continuation from earlier chunks, joined by k_msm_tail).  Every lane
// does the same number of additions whatever the bucket sizes.
// one 128-byte record as eight 16-byte loads (affine Niels words 0..29, two padding words)
__device__ __forceinline__ void msm_load_raw(const uint32_t* __restrict__ pts, uint32_t v, uint32_t w[32]) {
    const uint4* e = reinterpret_cast<const uint4*>(pts + (size_t)MSM_PT_WORDS * (v & ~MSM_NEG));
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint4 t = e[k];
        w[4 * k] = t.x; w[4 * k + 1] = t.y; w[4 * k + 2] = t.z; w[4 * k + 3] = t.w;
    }
}
// zero: a runtime 0 the compiler cannot see through.  Folding the padding words into the sign
// test keeps their registers live until the record is used; a dead load destination is reused
// by the register allocator at once, which forces a wait on the whole prefetch.
__device__ __forceinline__ ge_precomp msm_point_of(const uint32_t w[32], uint32_t v, uint32_t zero) {
    v |= (w[30] | w[31]) & zero;
    return msm_point_select(load_fe(w), load_fe(w + 10), load_fe(w + 20), (v & MSM_NEG) != 0);
}

// Two record buffers alternate (the loop is unrolled by two, so neither is copied) and entry
// indices are read two entries ahead, so a record's load is in flight for a whole addition.
extern "C" __global__ void __launch_bounds__(256) k_msm_bucket(
    uint32_t T, uint32_t nkeys, const uint32_t* __restrict__ total, const uint32_t* __restrict__ entries,
    const uint32_t* __restrict__ kstart, const uint32_t* __restrict__ pts, uint32_t* __restrict__ bsum,
    uint32_t* __restrict__ hpart, const uint32_t* __restrict__ seg_key, const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    const uint32_t E = *total;
    const uint64_t k0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * T;
    if (k0 >= E) return;
    const uint32_t k1 = (uint32_t)(k0 + T < E ? k0 + T : E);
    // key = the largest key with kstart[key] <= k0 (non-empty, contains entry k0): from the sort's
    // segment map when it wrote one (one-chunk batches), else a binary search
    uint32_t lo = 0, hi = nkeys;
    if (seg_key) lo = seg_key[k0 / T];
    else
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (kstart[mid] <= k0) lo = mid;
            else hi = mid;
        }
    uint32_t key = lo;
    uint32_t kend = key + 1 < nkeys ? kstart[key + 1] : E;
    bool head = kstart[key] < k0;
    ge_p3 acc = ge_p3_identity();
    // kend of the next key (kstart[key + 2]) is read after every step, so closing a segment does
    // not wait for a load of its own: some lane of a wave closes one almost every step (buckets
    // average ~24 entries at 65,536 signatures)
    const uint32_t klim = nkeys - 1;
    auto next_end = [&]() { return kstart[key + 2 < klim ? key + 2 : klim]; };
    uint32_t pf_val = next_end();
    // add entry k (record w, index word v); close the key segment when it ends here
    const uint32_t zero = 0u - (T >> 31);  // T < 2^31: all-zero, opaque to the compiler
    auto step = [&](const uint32_t* w, uint32_t v, uint32_t k) {
        acc = ge_p1p1_to_p3(ge_madd(acc, msm_point_of(w, v, zero)));
        if (k + 1 == k1 || k + 1 == kend) {
            store_p3(head ? hpart + (size_t)P3_WORDS * (k0 / T) : bsum + (size_t)P3_WORDS * key, acc);
            acc = ge_p3_identity();
            head = false;
            if (k + 1 < k1) {
                kend = key + 2 < nkeys ? pf_val : E;
                key++;
                if (kend <= k + 1) {  // empty keys follow: bisect for the key holding entry k + 1
                    uint32_t lo = key, hi = nkeys;  // kstart[lo] <= k + 1
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (kstart[mid] <= k + 1) lo = mid;
                        else hi = mid;
                    }
                    key = lo;
                    kend = key + 1 < nkeys ? kstart[key + 1] : E;
                }
            }
        }
    };
    // loads are unconditional (indices clamped into the chunk): branch-free code lets the
    // compiler count outstanding loads exactly instead of waiting for all of them
    const uint32_t klast = k1 - 1;
    auto at = [&](uint32_t k) { return entries[k < klast ? k : klast]; };
    uint32_t wa[32], wb[32];
    uint32_t va = entries[k0];
    uint32_t vb = at((uint32_t)k0 + 1);
    msm_load_raw(pts, va, wa);
#pragma unroll 1
    for (uint32_t k = (uint32_t)k0;; k += 2) {
        // index loads go out before the record loads: the memory counter is in order, so a
        // wait for an index never waits for a record still in flight
        const uint32_t vc = at(k + 2);
        msm_load_raw(pts, vb, wb);
        step(wa, va, k);
        pf_val = next_end();
        if (k + 1 >= k1) break;
        const uint32_t vd = at(k + 3);
        msm_load_raw(pts, vc, wa);
        step(wb, vb, k + 1);
        pf_val = next_end();
        if (k + 2 >= k1) break;
        va = vc;
        vb = vd;
    }
}

// k_msm_bucket on quads (latency-bound small batches): quad g adds the entries [gT, gT + T), lane
// q holding coordinate q (X, Y, Z, T) of the running sum.  A mixed addition is ge_madd's field
// operations on the same operands (so the same magnitudes) in two multiply latencies instead of
// seven: step 1 MM (q0), PP (q1), T xy2d (q2), 2Z (q3); the four broadcast in the quad (DPP);
// step 2 the four products of ge_p1p1_to_p3.  Segment bookkeeping is identical on the quad's lanes.
extern "C" __global__ void __launch_bounds__(256) k_msm_bucket_q(
    uint32_t T, uint32_t nkeys, const uint32_t* __restrict__ total, const uint32_t* __restrict__ entries,
    const uint32_t* __restrict__ kstart, const uint32_t* __restrict__ pts, uint32_t* __restrict__ bsum,
    uint32_t* __restrict__ hpart, const uint32_t* __restrict__ seg_key, const uint32_t* __restrict__ fail) {
    if (msm_failed(fail)) return;
    const uint32_t E = *total;
    const int q = threadIdx.x & 3;
    const uint64_t k0 = ((uint64_t)blockIdx.x * (blockDim.x >> 2) + (threadIdx.x >> 2)) * T;
    if (k0 >= E) return;  // whole quad
    const uint32_t k1 = (uint32_t)(k0 + T < E ? k0 + T : E);
    uint32_t lo = 0, hi = nkeys;
    if (seg_key) lo = seg_key[k0 / T];  // (k_msm_sort1's segment map), else a binary search
    else
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (kstart[mid] <= k0) lo = mid;
            else hi = mid;
        }
    uint32_t key = lo;
    uint32_t kend = key + 1 < nkeys ? kstart[key + 1] : E;
    bool head = kstart[key] < k0;
    const bool q0 = q == 0, q1 = q == 1, q2 = q == 2, q3 = q == 3;
    const fe ident = (q1 || q2) ? fe_one() : fe_zero();  // (0 : 1 : 1 : 0)
    fe acc = ident;
    const uint32_t zero = 0u - (T >> 31);
    uint32_t wcur[32], wnext[32];
    uint32_t v = entries[k0];
    msm_load_raw(pts, v, wcur);
#pragma unroll 1
    for (uint32_t k = (uint32_t)k0; k < k1; k++) {
        const uint32_t vn = entries[k + 1 < k1 ? k + 1 : k];
        msm_load_raw(pts, vn, wnext);
        const ge_precomp P = msm_point_of(wcur, v, zero);
        const fe X = fe_quad_bcast(acc, 0), Y = fe_quad_bcast(acc, 1), Z = fe_quad_bcast(acc, 2),
                 Tt = fe_quad_bcast(acc, 3);
        const fe a = fe_select(fe_select(fe_select(Z, Tt, q2), fe_add(Y, X), q1), fe_sub(Y, X), q0);
        const fe b = fe_select(fe_select(fe_select(fe_one(), P.xy2d, q2), P.ypx, q1), P.ymx, q0);
        fe r = fe_mul(a, b);
        if (q3) r = fe_carry(fe_add(Z, Z));
        const fe MM = fe_quad_bcast(r, 0), PP = fe_quad_bcast(r, 1), TX = fe_quad_bcast(r, 2), Z2 = fe_quad_bcast(r, 3);
        const fe cX = fe_sub(PP, MM), cY = fe_add(PP, MM), cZ = fe_add(Z2, TX), cT = fe_sub(Z2, TX);
        const fe u = fe_select(fe_select(cZ, cY, q1), cX, q0 || q3);
        const fe w2 = fe_select(fe_select(cY, cZ, q1), cT, q0 || q2);
        acc = fe_mul(u, w2);
        if (k + 1 == k1 || k + 1 == kend) {
            uint32_t* out = head ? hpart + (size_t)P3_WORDS * (k0 / T) : bsum + (size_t)P3_WORDS * key;
            store_fe(out + 10 * q, acc);
            acc = ident;
            head = false;
            if (k + 1 < k1) {
                key++;
                kend = key + 1 < nkeys ? kstart[key + 1] : E;
                if (kend <= k + 1) {  // empty keys follow: bisect for the key holding entry k + 1
                    uint32_t l2 = key, h2 = nkeys;
                    while (h2 - l2 > 1) {
                        const uint32_t mid = (l2 + h2) >> 1;
                        if (kstart[mid] <= k + 1) l2 = mid;
                        else h2 = mid;
                    }
                    key = l2;
                    kend = key + 1 < nkeys ? kstart[key + 1] : E;
                }
            }
        }
        v = vn;
#pragma unroll
        for (int i = 0; i < 32; i++) wcur[i] = wnext[i];
    }
}

// ---- fused tail: window sums, their scaling and the batch verdict in ONE launch ------------
// The MSM total is  sum_w [2^pos_w] W_w  with  W_w = sum_{b'=0}^{nb-1} (b'+1) S_{w,b'}.  Instead
// of a window kernel followed by a one-wave Horner (every window sum on the critical path, then
// ~250 dependent doublings), each window is scaled on its own as soon as its sum is known: only
// the TOP window's sum precedes the doubling chain, and the other windows overlap it.
//
// Window sums by bit planes:  W = sum_k 2^k T_k + U,  T_k = sum over buckets b' with bit k set,
// U = sum of all buckets.  All planes of 2^m buckets come out of ONE butterfly of depth m: at step
// o = 1, 2, 4, ..., every lane whose index has bit o clear adds its partner lane + o.  After the
// last step lane 0 holds U and lane 2^k holds T_k (a lane with lowest set bit k only ever meets
// lanes of the same lowest set bit, i.e. the T_k tree, and the pair sums move up to lanes with
// more trailing zeros).  Depth m additions instead of 2m + suffix scan + tree for running sums.
//
// grid (S, nw), 256 threads.  Workgroup (s, w) owns chunk s of window w (C = nb / S_w <= 256
// consecutive buckets, one per lane): its butterfly gives R_s (= the chunk's U) and T_{s,k},
// k < lg C.  The last-arriving workgroup of window w (agent-scope release / counter / acquire,
// cdna_hip_programming.md Guideline 16, counter form) combines them with one more butterfly over
// s, per plane: T_k = sum_s T_{s,k} (k < lg C), and the butterfly of the R_s gives the planes
// k >= lg C and U.  Its wave 0 then runs, on 16-lane rows (fe_row.h), the m-step plane chain and
// pos_w + 3 doublings ([8] folded in).  The final sum runs on one wave beside the chains
// (msm_tail_body), which then tests the identity: *verdict = 1 iff accepted and no failure flag is
// set.  ctr[0, 128) must be zero at launch (k_msm_prep's first workgroup clears it).
struct MsmTailArgs {
    const uint32_t* bsum;  // [nkeys] bucket sums (P3): a bucket's first piece (k_msm_bucket[_q])
    const uint32_t* hpart;    // [nseg] continuation pieces of buckets spanning chunks
    const uint32_t* kstart;   // [nkeys] first entry of each bucket
    const uint32_t* total;    // entry count E
    uint32_t nkeys, seg;      // seg: entries per bucket lane (T of k_msm_bucket[_q])
    uint32_t* part;        // [nw][S][TAIL_PART_SLOTS] chunk planes (P3): R_s, T_{s,0}, T_{s,1}, ...
    uint32_t* wsc;         // [2 nw + 1] x 64 words: (nw + 1) x 64 unused, then the scaled windows
                           // in cached row form (the final sum's terms)
    uint32_t* ctr;         // [0, nw): chunk arrivals; [64, 64 + nw): window w's term published
    const uint32_t* fail;
    const uint32_t* partial;   // k_msm_prep's per-workgroup sums of z_i s_i (nblk x 9 words)
    const uint32_t* comb;      // fixed-base comb table
    uint32_t nblk;
    uint32_t quad_max_c;  // chunk butterflies of at most this many buckets run on quads (0: never)
    uint32_t* verdict;
    uint32_t* runs;  // [2] accepted / rejected runs since staging (never reset by a run), or null
    uint32_t S;
    unsigned long long* stamps;  // diagnostics (NWV_TAIL_STAMPS): [nw][8] s_memrealtime, or null
    // a word of coherent pinned host memory the host polls instead of copying the verdict back
    // and waiting for the stream, or null: (hseq << 2) | code, code 1 accepted, 2 rejected,
    // 3 undetermined (a window never published, below).  hseq is the call's sequence number, so a
    // store left over from an earlier call on the lane is never taken for this call's verdict.
    uint32_t* hverdict;
    // the top TAIL_QUAD_TOP windows (the longest chains) run chunk butterflies of at most this
    // many buckets on quads whatever quad_max_c says: one quad pass a level at C = 128
    uint32_t quad_top_c;
    uint32_t hseq;
};
// bound on the final-sum wave's polls of one window's ready flag (each a coherent load plus a
// short sleep; seconds in all).  Reaching it ends the kernel with *verdict = 2, "undetermined":
// the host then runs the per-signature pass instead of reporting the batch invalid.  A compile-time
// constant: read from the kernel's arguments instead, it cost the tail 10 us at 65,536 signatures
// (same-box A/B, profiles/round6_tail_spin_ab.json).  The _spin1 kernels (bound 1) are the test
// hook that forces the undetermined outcome (NWV_TAIL_SPIN_LIMIT).
static constexpr uint32_t TAIL_SPIN = 1u << 24;
static constexpr int TAIL_QUAD_TOP = 4;
// batch verdict codes in *verdict (state word 1) and the host word's low two bits
static constexpr uint32_t MSM_REJECTED = 0u, MSM_ACCEPTED = 1u, MSM_UNDETERMINED = 2u;
// the verdict into the host-polled word: a system-scope release store from a vector lane
__device__ __forceinline__ void tail_host_verdict(const MsmTailArgs& a, uint32_t code) {
    if (a.hverdict) __hip_atomic_store(a.hverdict, (a.hseq << 2) | code, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static constexpr int TAIL_PART_SLOTS = 9;  // R_s + up to 8 planes (C <= 256)

namespace {

__device__ __forceinline__ int tail_lg(int x) {
    int lg = 0;
    while ((1 << lg) < x) lg++;
    return lg;
}

// The final sum's hand-offs move 64 words between workgroups on different XCDs.  They go as
// agent-scope relaxed atomic loads / stores (coherent at the device level, past the XCD's L2)
// with the wave's own vmcnt wait before the counter, so no release / acquire fence (an L2
// write-back / invalidate of ~1-2 us each, MI355X_MICROARCH.md) sits on the ladder's path.
__device__ __forceinline__ uint32_t tail_ld_coh(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tail_st_coh(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// counter hand-off of everything this workgroup stored: returns true (uniformly) in the
// workgroup that arrives last of `expect`, after an agent-scope acquire
__device__ __forceinline__ bool tail_arrive(uint32_t* ctr, uint32_t expect, uint32_t* flag) {
    const int t = threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t last = old + 1 == expect ? 1u : 0u;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}

}  // namespace

// The basepoint term (one extra workgroup of k_msm_tail, running beside the windows' bucket
// sums): b = -(sum of k_msm_prep's per-workgroup partial sums of z_i s_i) mod l, c = 8 b mod l,
// [c]B = sum of 64 comb entries (wave 0: one entry per lane, then a six-level butterfly of
// additions) -> acc0 (64 words of LDS: row limbs, the final sum's first term), in wave 0.
__device__ __forceinline__ void msm_bterm(const uint32_t* __restrict__ partial, uint32_t nblk,
                                          const uint32_t* __restrict__ comb, uint32_t* __restrict__ acc0) {
    __shared__ unsigned long long wcol[4][9];
    __shared__ int dig[COMB_TABLES];
    const int t = threadIdx.x, wid = t >> 6, lane = t & 63;
    unsigned long long s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t q = t; q < nblk; q += 256)
#pragma unroll
        for (int k = 0; k < 9; k++) s[k] += partial[9 * (size_t)q + k];  // < 2^32 each, < 2^16 of them
#pragma unroll
    for (int k = 0; k < 9; k++) {
        unsigned long long v = s[k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) wcol[wid][k] = v;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t x[16];
        unsigned long long c = 0;
        for (int k = 0; k < 16; k++) {
            if (k < 9) c += wcol[0][k] + wcol[1][k] + wcol[2][k] + wcol[3][k];
            x[k] = (uint32_t)c;
            c >>= 32;
        }
        uint32_t r[8], b[8], c8[8];
        sc_reduce512(x, r);
        uint32_t nz = 0;
        for (int k = 0; k < 8; k++) nz |= r[k];
        long long br = 0;
        for (int k = 0; k < 8; k++) {  // b = l - r (mod l)
            const long long d = (long long)sc_l(k) - r[k] + br;
            b[k] = nz ? (uint32_t)d : 0u;
            br = d >> 32;
        }
        const uint32_t eight[8] = {8u, 0, 0, 0, 0, 0, 0, 0};
        sc_mul(b, eight, c8);
        int d[COMB_TABLES];
        comb_digits(c8, d);
        for (int j = 0; j < COMB_TABLES; j++) dig[j] = d[j];
    }
    __syncthreads();
    if (wid == 0) {  // (no early return: the caller's arrival barrier follows)
        const int dj = dig[lane], a = dj < 0 ? -dj : dj;
        ge_p3 P = ge_p3_identity();
        if (a)
            P = ge_p1p1_to_p3(ge_madd(P, msm_load_point(comb + MSM_PT_WORDS * (COMB_ENTRIES * lane + a - 1), dj < 0)));
#pragma unroll 1
        for (int o = 1; o < 64; o <<= 1) {
            const ge_p3 Q = shfl_down_p3(P, o);
            if (!(lane & (2 * o - 1))) P = p3_add(P, Q);
        }
        if (lane == 0) {  // the final sum's first term, as X | Y | Z | T row limbs (LDS)
            fe_to_limbs16(P.X, acc0);
            fe_to_limbs16(P.Y, acc0 + 16);
            fe_to_limbs16(P.Z, acc0 + 32);
            fe_to_limbs16(P.T, acc0 + 48);
        }
        rowf::lds_order();
    }
}

// Extended addition of the P3 points in LDS slots i and i + o into slot i by the four lanes of a
// quad, one coordinate each: the same field operations as p3_add (ge_p3_to_cached, ge_add,
// ge_p1p1_to_p3) on the same operands, so the same magnitudes, but three multiply latencies
// instead of nine.  Lane q: step 1 MM (q0), PP (q1), 2d T2 (q2), Z1 2Z2 (q3); step 2 TT2d = T1 2dT2
// (q2); the four products are broadcast in the quad (DPP quad_perm); step 3 X3, Y3, Z3, T3.
// Branch-free operand selection: every lane of the wave runs every multiply once.
__device__ __forceinline__ void quad_p3_add(uint32_t* lds, int i, int o, int q) {
    const uint32_t* L = lds + P3_WORDS * i;
    const uint32_t* R = lds + P3_WORDS * (i + o);
    const fe X1 = load_fe(L), Y1 = load_fe(L + 10), Z1 = load_fe(L + 20), T1 = load_fe(L + 30);
    const fe X2 = load_fe(R), Y2 = load_fe(R + 10), Z2 = load_fe(R + 20), T2 = load_fe(R + 30);
    const bool q0 = q == 0, q1 = q == 1, q2 = q == 2;
    const fe a = fe_select(fe_select(fe_select(Z1, T2, q2), fe_add(Y1, X1), q1), fe_sub(Y1, X1), q0);
    const fe b = fe_select(fe_select(fe_select(fe_carry(fe_add(Z2, Z2)), fe_d2(), q2), fe_carry(fe_add(Y2, X2)), q1),
                           fe_carry(fe_sub(Y2, X2)), q0);
    fe r = fe_mul(a, b);
    if (q2) r = fe_mul(T1, r);
    const fe MM = fe_quad_bcast(r, 0), PP = fe_quad_bcast(r, 1), TT2d = fe_quad_bcast(r, 2), ZZ2 = fe_quad_bcast(r, 3);
    const fe cX = fe_sub(PP, MM), cY = fe_add(PP, MM), cZ = fe_add(ZZ2, TT2d), cT = fe_sub(ZZ2, TT2d);
    const bool q3 = q == 3;
    const fe u = fe_select(fe_select(cZ, cY, q1), cX, q0 || q3);
    const fe v = fe_select(fe_select(cY, cZ, q1), cT, q0 || q2);
    store_fe(lds + P3_WORDS * i + 10 * q, fe_mul(u, v));
}

// Bucket sum of key `key`: its first piece from bsum plus the continuation pieces of the chunks it
// spans (T entries per bucket lane), or the identity when the bucket is empty (bsum never
// written).  The join the round-1 pipeline ran as a separate launch (k_msm_fixup), done by the
// tail lane that loads the bucket.
__device__ __forceinline__ ge_p3 msm_bucket_join(const MsmTailArgs& a, uint32_t key) {
    const uint32_t s = a.kstart[key];
    const uint32_t e = key + 1 < a.nkeys ? a.kstart[key + 1] : *a.total;
    if (s == e) return ge_p3_identity();
    ge_p3 acc = load_p3(a.bsum + (size_t)P3_WORDS * key);
    const uint32_t i1 = (e - 1) / a.seg;
#pragma unroll 1
    for (uint32_t i = s / a.seg + 1; i <= i1; i++) acc = p3_add(acc, load_p3(a.hpart + (size_t)P3_WORDS * i));
    return acc;
}

#define NWV_TAIL_STAMP(slot)                                                                       \
    do {                                                                                           \
        if (a.stamps && t == 0) a.stamps[8 * w + (slot)] = __builtin_amdgcn_s_memrealtime();       \
    } while (0)

// PER: combine items per thread (1 when every window's (lg C + 1) x S_w <= 256, else 3).  The
// variant with one item needs 163 VGPRs instead of 216; fewer registers held by the tail's
// long-lived waves leave room for other batches' waves on the same SIMDs.
// Workgroup (s, row) of a window row: chunk s of window w = nw - row.  Returns true (uniformly) in
// the workgroup that arrives last at the final counter (windows and the basepoint term).
template <int PER>
__device__ __forceinline__ bool msm_tail_window(const MsmLayout& lay, const MsmTailArgs& a, uint32_t* lds,
                                                uint32_t* flag) {
    // top window first (row 1): its sum precedes the longest doubling chain, and workgroups are
    // dispatched in blockIdx order (a grid larger than the chip runs in waves)
    const int t = threadIdx.x, w = lay.nw - (int)blockIdx.y, s = blockIdx.x;
    const int nb = 1 << (lay.width[w] - 1);
    const int Sw = (int)a.S < nb ? (int)a.S : nb;
    if (s >= Sw) return false;  // whole workgroup
    const int C = nb / Sw, lgC = tail_lg(C), lgS = tail_lg(Sw);
    if (s == 0) NWV_TAIL_STAMP(0);
    // ---- chunk butterfly: lane 0 -> R_s, lane 2^k -> T_{s,k}
    uint32_t* mine = lds + P3_WORDS * t;
    ge_p3 p = ge_p3_identity();
    const uint32_t qmax = w >= lay.nw - TAIL_QUAD_TOP && a.quad_top_c > a.quad_max_c ? a.quad_top_c : a.quad_max_c;
    // (bucket joins stay lane-local: joining on quads, each continuation piece loaded into LDS and
    // added by quad_p3_add, made the tail at 65,536 slower, 152 -> 168 us, same-box A/B,
    // profiles/round6_tail_quad_join_ab.json: each piece's global load sat on the quad's chain)
    if (t < C) p = msm_bucket_join(a, lay.kbase[w] + (uint32_t)(s * C + t));
    if (s == 0) NWV_TAIL_STAMP(7);
    if ((uint32_t)C <= qmax) {
        // on quads (latency-bound small batches): every level's C / 2 additions (lanes i with bit
        // o clear add lane i + o, in place) as 64 quads per pass
        if (t < C) store_p3(mine, p);
        __syncthreads();
        const int q = t & 3;
        for (int o = 1, lg = 0; o < C; o <<= 1, lg++) {
            for (int g = t >> 2; g < C / 2; g += 64) {
                const int i = ((g >> lg) << (lg + 1)) | (g & (o - 1));
                quad_p3_add(lds, i, o, q);
            }
            __syncthreads();
        }
        if (t < C) p = load_p3(mine);
    } else {
        // lane-local additions in LDS: every level's C / 2 additions on the first C / 2 lanes
        // (lane g adds slot i + o into slot i, i = g with a zero inserted at bit lg), so only
        // ceil(C / 128) waves of the workgroup issue them (round 4: every lane with bit o clear,
        // i.e. all four waves for o < 64, half of each idle)
        if (t < C) store_p3(mine, p);
        __syncthreads();
        for (int o = 1, lg = 0; o < C; o <<= 1, lg++) {
            if (t < C / 2) {
                uint32_t* d = lds + P3_WORDS * (((t >> lg) << (lg + 1)) | (t & (o - 1)));
                store_p3(d, p3_add(load_p3(d), load_p3(d + P3_WORDS * o)));
            }
            __syncthreads();
        }
        if (t < C && !(t & (t - 1))) p = load_p3(mine);  // lane 0 and the powers of two
    }
    uint32_t* mypart = a.part + (size_t)P3_WORDS * TAIL_PART_SLOTS * ((size_t)w * a.S + s);
    if (t == 0) store_p3(mypart, p);
    if (t < C && t && !(t & (t - 1))) store_p3(mypart + P3_WORDS * (1 + tail_lg(t)), p);
    if (!tail_arrive(a.ctr + w, (uint32_t)Sw, flag)) return false;
    NWV_TAIL_STAMP(1);
    // ---- last chunk of window w: per plane, a butterfly over the Sw chunks.  Item j = q * Sw + s:
    // plane group q < lgC sums T_{s,q}; group lgC is the butterfly of the R_s.
    const int items = (lgC + 1) * Sw, per = (items + 255) / 256;  // items per thread (<= PER)
    ge_p3 v[PER];
#pragma unroll
    for (int r = 0; r < PER; r++) {
        const int j = t + 256 * r;
        v[r] = ge_p3_identity();
        if (r < per && j < items) {
            const int q = j / Sw, sj = j % Sw;
            const uint32_t* pp = a.part + (size_t)P3_WORDS * TAIL_PART_SLOTS * ((size_t)w * a.S + sj);
            v[r] = load_p3(pp + P3_WORDS * (q < lgC ? 1 + q : 0));
        }
    }
    for (int o = 1; o < Sw; o <<= 1) {
#pragma unroll
        for (int r = 0; r < PER; r++) {
            if (r >= per) break;
            const int j = t + 256 * r;
            __syncthreads();
            if (j < items) store_p3(mine, v[r]);
            __syncthreads();
            if (j < items && !((j % Sw) & o)) v[r] = p3_add(v[r], load_p3(lds + P3_WORDS * (t + o)));
        }
    }
    // planes in cached row form: plane k < lgC at item k * Sw; plane lgC + i at item
    // lgC * Sw + 2^i; U at item lgC * Sw.  Slot order: T_0 .. T_{m-1}, U  (m = lgC + lgS).
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PER; r++) {
        const int j = t + 256 * r;
        if (r >= per || j >= items) continue;
        const int q = j / Sw, sj = j % Sw;
        int slot = -1;
        if (q < lgC && sj == 0) slot = q;
        else if (q == lgC && sj == 0) slot = lgC + lgS;
        else if (q == lgC && !(sj & (sj - 1))) slot = lgC + tail_lg(sj);
        if (slot >= 0) store_p3(lds + P3_WORDS * slot, v[r]);  // planes fit slots 0..16
    }
    __syncthreads();
    NWV_TAIL_STAMP(2);
    const int m = lgC + lgS;
    uint32_t* rows = lds + 32 * P3_WORDS;  // (m + 1) x 64 row limbs, behind the plane slots
    if (t < 4 * (m + 1)) {
        const ge_p3 pl = load_p3(lds + P3_WORDS * (t >> 2));
        const int c = t & 3;
        fe v2 = c == 0 ? fe_add(pl.Y, pl.X) : c == 1 ? fe_sub(pl.Y, pl.X) : c == 2 ? fe_mul(pl.T, fe_d2())
                                                                                   : fe_add(pl.Z, pl.Z);
        fe_to_limbs16(fe_carry(v2), rows + 64 * (t >> 2) + 16 * c);
    }
    __syncthreads();
    NWV_TAIL_STAMP(3);
#if defined(__HIP_DEVICE_COMPILE__)  // (rowf's lane type is the host emulation's wave elsewhere)
    if (t < 64) {  // the scaled window sum, in cached row form for the final sum
        const rowf::RowP3 d = rowf::row_planes_chain(rows, m, lay.pos[w] + 3, nullptr);
        rowf::RowConsts k = rowf::row_consts();
        k.rot = 1;
        tail_st_coh(a.wsc + (size_t)64 * (lay.nw + 1 + w) + t, rowf::row_to_cached(d, k));
    }
#endif
    NWV_TAIL_STAMP(4);
    return true;
}

template <int PER, uint32_t SPIN>
__device__ __forceinline__ void msm_tail_body(const MsmLayout& lay, const MsmTailArgs& a) {
    if (msm_failed(a.fail)) {  // rejected at prep (the sort and bucket kernels skipped their work)
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
            *a.verdict = MSM_REJECTED;
            if (a.runs) a.runs[1] += 1u;
            tail_host_verdict(a, 2u);
        }
        return;
    }
    // 256 point slots of P3_WORDS; row-limb planes reuse the front once the slots are done;
    // the flag word sits behind the slots
    extern __shared__ uint32_t lds[];
    uint32_t* flag = lds + 256 * P3_WORDS;
    const int t = threadIdx.x;
    // Final sum by ONE accumulating wave (the basepoint term's workgroup, dispatched first):
    // acc = [8 b]B, then acc += (scaled window w) for w = 0 .. nw - 1 in window order, each a
    // row-form addition (fe_row.h row_add_cached, ~0.4 us) with acc kept in registers.  Window w's
    // last workgroup publishes its cached row form and sets ready[w] (ctr[64 + w]); the wave waits
    // for each flag in turn.  Window chains end in about window order (window w's chain is
    // pos_w + 3 + its plane count long), so the additions run behind the chains and one follows
    // the top window's.  Round 4 summed all nw + 1 items after the last arrival with a 5-level
    // quad-lane tree (13 us at 1,024 signatures); a hand-off ladder between workgroups cost ~1.7 us
    // a step (cross-XCD atomics and loads) and fell behind the windows.
    uint32_t* ready = a.ctr + 64;
    uint32_t* sa = lds + 16 * P3_WORDS;  // 64 words
    if (blockIdx.y != 0) {
        if (!msm_tail_window<PER>(lay, a, lds, flag)) return;
        if (t < 64) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the cached row form has landed
            if (t == 0) tail_st_coh(ready + (lay.nw - (int)blockIdx.y), 1u);
        }
        return;
    }
    if (blockIdx.x != 0) return;
    msm_bterm(a.partial, a.nblk, a.comb, sa);
    if (t >= 64) return;
#if defined(__HIP_DEVICE_COMPILE__)  // (rowf's lane type is the host emulation's wave elsewhere)
    const uint32_t* wc = a.wsc + (size_t)64 * (lay.nw + 1);  // window w's cached row form
    rowf::RowConsts k = rowf::row_consts();
    k.rot = 1;
    const uint32_t limb = t & 15;
    rowf::RowP3 d{sa[limb], sa[16 + limb], sa[32 + limb], sa[48 + limb]};
    bool timed_out = false;
#pragma unroll 1
    for (int w = 0; w < lay.nw; w++) {
        // a bounded wait: a window that never publishes ends the kernel with "undetermined"
        uint32_t spins = 0;
        while (tail_ld_coh(ready + w) == 0u && ++spins < SPIN) __builtin_amdgcn_s_sleep(1);
        if (spins >= SPIN) {
            timed_out = true;
            break;
        }
        if (w == lay.nw - 1) NWV_TAIL_STAMP(5);
        d = rowf::row_add_cached(d, tail_ld_coh(wc + (size_t)64 * w + t), k);
    }
    if (t < 16) {
        sa[t] = d.X;
        sa[16 + t] = d.Y;
        sa[32 + t] = d.Z;
    }
    rowf::lds_order();
    // the identity test X = 0 and Y = Z as two zero tests side by side: lane 0 X - 0, lane 1 Y - Z
    // (the same instructions on both lanes, one freeze each)
    const fe va = fe_from_limbs16(sa + (t == 1 ? 16 : 0));
    const fe vb = fe_select(fe_from_limbs16(sa + 32), fe_zero(), t != 1);
    const bool nz = !fe_is_zero(fe_sub(fe_carry(va), fe_carry(vb)));
    const unsigned long long bad = __ballot(t < 2 && nz);
    if (t == 0) {
        const bool ok = !timed_out && bad == 0 && *a.fail == 0;
        *a.verdict = timed_out ? MSM_UNDETERMINED : ok ? MSM_ACCEPTED : MSM_REJECTED;
        // per-run tally (runs of one batch are ordered on its stream: a plain increment); an
        // undetermined run is not an accepted one
        if (a.runs) a.runs[ok ? 0 : 1] += 1u;
        tail_host_verdict(a, timed_out ? 3u : ok ? 1u : 2u);
    }
    const int w = lay.nw - 1;  // stamp slot
    NWV_TAIL_STAMP(6);
#endif
}

extern "C" __global__ void __launch_bounds__(256) k_msm_tail(MsmLayout lay, MsmTailArgs a) {
    msm_tail_body<1, TAIL_SPIN>(lay, a);
}
extern "C" __global__ void __launch_bounds__(256) k_msm_tail_wide(MsmLayout lay, MsmTailArgs a) {
    msm_tail_body<3, TAIL_SPIN>(lay, a);
}
extern "C" __global__ void __launch_bounds__(256) k_msm_tail_spin1(MsmLayout lay, MsmTailArgs a) {
    msm_tail_body<1, 1u>(lay, a);
}
extern "C" __global__ void __launch_bounds__(256) k_msm_tail_wide_spin1(MsmLayout lay, MsmTailArgs a) {
    msm_tail_body<3, 1u>(lay, a);
}
