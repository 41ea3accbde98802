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

extern "C" __global__ void __launch_bounds__(256) k_blake2b_many(
    uint64_t n, const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
    const uint64_t* __restrict__ len, uint32_t* __restrict__ out) {
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
