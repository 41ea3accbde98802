// blake2b_kernels.hip -- K6: BLAKE2b-256 digests on gfx950.
//
//   k_blake2b_many     one message per lane (header / vote / certificate digests, many
//                      independent batches): fastcrypto::blake2b_256 semantics
//   k_batch_compact    one workgroup per bincode WorkerMessage::Batch buffer: walks the
//                      [u32 variant][u64 count][(u64 len, bytes)]* layout of
//                      types/src/worker.rs:44-80 and packs the transaction bytes (the
//                      Batch::digest stream, types/src/primary.rs:65-73) contiguously; the
//                      packed streams are then hashed by k_blake2b_many.
// Message arenas are padded by >= 16 bytes (aligned over-reads are safe).
#include "blake2b.h"

using namespace nwv;

// out2 (optional): a second copy of the digests (coherent pinned host memory: no copy back)
extern "C" __global__ void __launch_bounds__(256) k_blake2b_many(
    uint64_t n, const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint64_t* __restrict__ len, uint32_t* __restrict__ out, uint32_t* __restrict__ out2) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = base + off[i];
    const uint64_t L = len[i];
    blake2b_state s;
    blake2b_init256(s);
    const uint64_t nblocks = L == 0 ? 1 : (L + 127) / 128;
#pragma unroll 1
    for (uint64_t b = 0; b < nblocks; b++) {
        u64p m[16];
        const uint64_t pos0 = 128 * b;
#pragma unroll
        for (int t = 0; t < 16; t++) {
            m[t].lo = msg_word_trim(p, pos0 + 8 * t, L);
            m[t].hi = msg_word_trim(p, pos0 + 8 * t + 4, L);
        }
        const bool last = b + 1 == nblocks;
        blake2b_compress(s, m, last ? (uint32_t)(L - pos0) : 128u, last);
    }
    uint32_t d[8];
    blake2b_digest256(s, d);
    uint4* o = reinterpret_cast<uint4*>(out + 8 * i);
    o[0] = make_uint4(d[0], d[1], d[2], d[3]);
    o[1] = make_uint4(d[4], d[5], d[6], d[7]);
    if (out2) {
        uint4* o2 = reinterpret_cast<uint4*>(out2 + 8 * i);
        o2[0] = make_uint4(d[0], d[1], d[2], d[3]);
        o2[1] = make_uint4(d[4], d[5], d[6], d[7]);
    }
}

// ---- long messages: 4 lanes per message --------------------------------------------------
// BLAKE2b is sequential over blocks, so a worker batch (types/src/primary.rs:65-73, ~500 KB =
// 3,909 compressions) is latency-bound on one lane.  Here the 4 lanes of a quad hold the 4
// columns of the 4x4 state (lane q: v[q], v[q+4], v[q+8], v[q+12]) and run the column step's
// and the diagonal step's G functions in parallel; between the two steps rows 1-3 rotate
// across the quad with DPP quad_perm moves.  The 128-byte block is staged in LDS (each lane
// loads 32 bytes) and every G reads its two sigma-selected words from there.
namespace {
// quad_perm controls: lane q reads lane (q+1)%4, (q+2)%4, (q+3)%4
constexpr int QP_NEXT1 = 0x39, QP_NEXT2 = 0x4E, QP_NEXT3 = 0x93;
// update_dpp with bound_ctrl (every lane of a quad_perm reads a live lane, so the zero fill never
// applies): in that form LLVM folds the move into a VOP2 consumer as a DPP source operand
// (v_xor_b32_dpp for d ^ a), 44 fewer instructions per compression
template <int CTRL>
__device__ __forceinline__ uint64_t quad_rot(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, true);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// rotation as two independent v_alignbit_b32 on the halves (one dependent level; the shift/or
// form the compiler picks for (x >> n) | (x << (64 - n)) is two)
__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (n == 32) return ((uint64_t)lo << 32) | hi;
    const u64p r = rotr(u64p{lo, hi}, n);
    return ((uint64_t)r.hi << 32) | r.lo;
}
// G on native 64-bit words: the adds become single v_lshl_add_u64 (gfx950).  The message word is
// added to a before b is (a + m does not wait for b, the previous G's last result), so each half
// of G has one dependent add less on the chain that bounds a long message's latency.
// opaque to reassociation: LLVM would otherwise rewrite (a + m) + b as (m + b) + a
__device__ __forceinline__ uint64_t pinned_sum(uint64_t a, uint64_t m) {
    uint64_t t = a + m;
    __asm__("" : "+v"(t));
    return t;
}
__device__ __forceinline__ void b2_g(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t x, uint64_t y) {
    a = b + pinned_sum(a, x);
    d = rotr64(d ^ a, 32);
    c = c + d;
    b = rotr64(b ^ c, 24);
    a = b + pinned_sum(a, y);
    d = rotr64(d ^ a, 16);
    c = c + d;
    b = rotr64(b ^ c, 63);
}
// nibble q of the packed sigma entries for lane q
constexpr uint32_t sigma_pack(int r, int first) {
    uint32_t v = 0;
    for (int q = 0; q < 4; q++) v |= (uint32_t)BLAKE2B_SIGMA[r][first + 2 * q] << (4 * q);
    return v;
}
__device__ __forceinline__ uint64_t iv64(int k) {
    return (uint64_t)BLAKE2B_IV32[2 * k] | ((uint64_t)BLAKE2B_IV32[2 * k + 1] << 32);
}
}  // namespace

extern "C" __global__ void __launch_bounds__(64) k_blake2b_quad(
    uint64_t n, const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint64_t* __restrict__ len, uint32_t* __restrict__ out, uint32_t* __restrict__ out2) {
    __shared__ uint64_t blk[16][16];
    const int lane = threadIdx.x, q = lane & 3, slot = lane >> 2;
    const uint64_t i = (uint64_t)blockIdx.x * 16 + slot;
    const bool active = i < n;
    const uint8_t* p = active ? base + off[i] : base;
    const uint64_t L = active ? len[i] : 0;
    const uint64_t nb = active ? (L == 0 ? 1 : (L + 127) / 128) : 0;
    uint64_t nmax = nb;  // blocks of the longest message of the wave
    for (int o = 4; o < 64; o <<= 1) {
        const uint64_t t = __shfl_xor(nmax, o);
        nmax = t > nmax ? t : nmax;
    }
    const uint64_t iv0 = iv64(q), iv1 = iv64(q + 4);
    uint64_t h0 = iv0, h1 = iv1;
    if (q == 0) h0 ^= 0x01010000u ^ 32u;
    const int sh = 4 * q;
    // the next block's 32 bytes for this lane are fetched one block ahead (9 aligned dwords
    // cover an unaligned 32-byte window), so the global-load latency overlaps a compression
    uint32_t raw[9];
    auto fetch = [&](uint64_t blk_idx) {
        const uintptr_t a = (uintptr_t)(p + 128 * blk_idx + 32 * q);
        const uint32_t* wp = (const uint32_t*)(a & ~(uintptr_t)3);
#pragma unroll
        for (int t = 0; t < 9; t++) raw[t] = wp[t];
    };
    if (nb > 0) fetch(0);
#pragma unroll 1
    for (uint64_t b = 0; b < nmax; b++) {
        const bool live = b < nb;
        const uint64_t pos = 128 * b + 32 * q;
        const uint32_t ash = (uint32_t)(((uintptr_t)(p + pos)) & 3) * 8;
        uint32_t w[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint64_t two = ((uint64_t)raw[t + 1] << 32) | raw[t];
            uint32_t v = (uint32_t)(two >> ash);
            const uint64_t bp = pos + 4 * t;  // trim to the message length (zero past the end)
            if (!live || bp >= L) v = 0u;
            else if (bp + 4 > L) v &= 0xffffffffu >> (8 * (uint32_t)(bp + 4 - L));
            w[t] = v;
        }
#pragma unroll
        for (int t = 0; t < 4; t++) blk[slot][4 * q + t] = (uint64_t)w[2 * t] | ((uint64_t)w[2 * t + 1] << 32);
        if (b + 1 < nb) fetch(b + 1);
        __syncthreads();
        // every sigma-selected word this lane needs for the 12 rounds, before the chain starts
        const uint64_t* m = blk[slot];
        uint64_t mw[12][4];
#pragma unroll
        for (int r = 0; r < 12; r++) {
            mw[r][0] = m[(sigma_pack(r, 0) >> sh) & 15];
            mw[r][1] = m[(sigma_pack(r, 1) >> sh) & 15];
            mw[r][2] = m[(sigma_pack(r, 8) >> sh) & 15];
            mw[r][3] = m[(sigma_pack(r, 9) >> sh) & 15];
        }
        const bool last = b + 1 == nb;
        const uint64_t tb = last ? L : 128 * (b + 1);  // bytes compressed so far
        uint64_t va = h0, vb = h1, vc = iv0, vd = iv1;
        if (q == 0) vd ^= tb;
        if (q == 2 && last) vd = ~vd;
#pragma unroll
        for (int r = 0; r < 12; r++) {
            b2_g(va, vb, vc, vd, mw[r][0], mw[r][1]);
            vb = quad_rot<QP_NEXT1>(vb);
            vc = quad_rot<QP_NEXT2>(vc);
            vd = quad_rot<QP_NEXT3>(vd);
            b2_g(va, vb, vc, vd, mw[r][2], mw[r][3]);
            vb = quad_rot<QP_NEXT3>(vb);
            vc = quad_rot<QP_NEXT2>(vc);
            vd = quad_rot<QP_NEXT1>(vd);
        }
        if (live) {
            h0 ^= va ^ vc;
            h1 ^= vb ^ vd;
        }
        __syncthreads();
    }
    if (active) {
        out[8 * i + 2 * q] = (uint32_t)h0;
        out[8 * i + 2 * q + 1] = (uint32_t)(h0 >> 32);
        if (out2) {
            out2[8 * i + 2 * q] = (uint32_t)h0;
            out2[8 * i + 2 * q + 1] = (uint32_t)(h0 >> 32);
        }
    }
}

namespace {
__device__ __forceinline__ uint64_t ld_u64_unaligned(const uint8_t* p) {
    return (uint64_t)ld_u32_unaligned(p) | ((uint64_t)ld_u32_unaligned(p + 4) << 32);
}
}  // namespace

// One workgroup per serialized batch i (buffer base + off[i], len[i] bytes).  Lane 0 walks
// the length prefixes (a dependent chain by construction of the format) and records the
// segments in LDS in chunks; all lanes then copy each chunk's transaction bytes into
// packed + off[i] (payload <= len[i] - 12).  payload_len[i] = packed length, or err[i] =
// offset of the u64 field that could not be read (DigestError::InvalidArgumentError).
static constexpr int SEG_CHUNK = 1024;
extern "C" __global__ void __launch_bounds__(256) k_batch_compact(
    uint64_t n, const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint64_t* __restrict__ len, uint8_t* __restrict__ packed,
    uint64_t* __restrict__ payload_len, int64_t* __restrict__ err) {
    const uint64_t i = blockIdx.x;
    if (i >= n) return;
    __shared__ uint64_t seg_src[SEG_CHUNK];
    __shared__ uint64_t seg_dst[SEG_CHUNK];
    __shared__ uint64_t seg_len[SEG_CHUNK];
    __shared__ int nseg;
    __shared__ int done;
    __shared__ int64_t err_off;
    __shared__ uint64_t walk_pos, walk_left, walk_dst;
    const uint8_t* buf = base + off[i];
    uint8_t* dst = packed + off[i];
    const uint64_t L = len[i];
    if (threadIdx.x == 0) {
        err_off = -1;
        done = 0;
        walk_dst = 0;
        if (L < 12) {
            err_off = 4;
            done = 1;
        } else {
            walk_left = ld_u64_unaligned(buf + 4);
            walk_pos = 12;
        }
    }
    __syncthreads();
    if (done) {
        if (threadIdx.x == 0) { err[i] = err_off; payload_len[i] = 0; }
        return;
    }
    for (;;) {
        if (threadIdx.x == 0) {
            int k = 0;
            uint64_t pos = walk_pos, left = walk_left, d = walk_dst;
            while (left > 0 && k < SEG_CHUNK) {
                if (pos + 8 > L) { err_off = (int64_t)pos; break; }
                const uint64_t tl = ld_u64_unaligned(buf + pos);
                if (tl > L - pos - 8) { err_off = (int64_t)pos; break; }
                seg_src[k] = pos + 8;
                seg_dst[k] = d;
                seg_len[k] = tl;
                d += tl;
                pos += 8 + tl;
                left--;
                k++;
            }
            nseg = k;
            walk_pos = pos;
            walk_left = left;
            walk_dst = d;
            done = (left == 0 || err_off >= 0) ? 1 : 0;
        }
        __syncthreads();
        const bool finished = done != 0;  // read between the two barriers: stable
        // copy this chunk's segments: lanes stride over the bytes of each segment
        for (int s = 0; s < nseg; s++) {
            const uint64_t sl = seg_len[s], ss = seg_src[s], sd = seg_dst[s];
            for (uint64_t b = threadIdx.x; b < sl; b += blockDim.x) dst[sd + b] = buf[ss + b];
        }
        __syncthreads();
        if (finished) break;
    }
    if (threadIdx.x == 0) {
        err[i] = err_off;
        payload_len[i] = err_off >= 0 ? 0 : walk_dst;
    }
}
