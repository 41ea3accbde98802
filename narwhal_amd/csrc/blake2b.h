// blake2b.h -- BLAKE2b with digest_length 32 (RFC 7693) on gfx950 VALU.
//
// Replaces fastcrypto::blake2b_256 = blake2 0.9.2 VarBlake2b::new(32)
// (/root/reference/Cargo.lock:536; used by types/src/primary.rs:65-73 Batch::digest,
// :209-227 Header::digest, :351-364 Vote::digest, :594-607 Certificate::digest and by
// types/src/worker.rs:44-62 serialized_batch_digest).  64-bit words are (lo, hi) VGPR pairs
// as in sha512.h; rotations by 32/24/16/63 are a swap and v_alignbit pairs.
#pragma once
#include "sha512.h"

namespace nwv {

static constexpr uint8_t BLAKE2B_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static constexpr uint32_t BLAKE2B_IV32[16] = {
    0xf3bcc908u, 0x6a09e667u, 0x84caa73bu, 0xbb67ae85u, 0xfe94f82bu, 0x3c6ef372u,
    0x5f1d36f1u, 0xa54ff53au, 0xade682d1u, 0x510e527fu, 0x2b3e6c1fu, 0x9b05688cu,
    0xfb41bd6bu, 0x1f83d9abu, 0x137e2179u, 0x5be0cd19u};

struct blake2b_state {
    u64p h[8];
    uint64_t t;  // bytes compressed so far
};

NWV_HD void blake2b_init256(blake2b_state& s) {
#pragma unroll
    for (int i = 0; i < 8; i++) s.h[i] = u64p{BLAKE2B_IV32[2 * i], BLAKE2B_IV32[2 * i + 1]};
    s.h[0].lo ^= 0x01010000u ^ 32u;  // depth 1, fanout 1, key length 0, digest length 32
    s.t = 0;
}

NWV_HD u64p xor2(u64p a, u64p b) { return u64p{a.lo ^ b.lo, a.hi ^ b.hi}; }
NWV_HD u64p swap_halves(u64p a) { return u64p{a.hi, a.lo}; }  // rotation by 32

// little-endian word at byte position pos of a message of `len` bytes (zero past the end);
// the arena is padded so the aligned word after the last byte may be read
NWV_HD uint32_t msg_word_trim(const uint8_t* p, uint64_t pos, uint64_t len) {
    if (pos >= len) return 0u;
    uint32_t v = ld_u32_unaligned(p + pos);
    if (pos + 4 > len) v &= 0xffffffffu >> (8 * (uint32_t)(pos + 4 - len));
    return v;
}

// F(h, m, t, last); m = 16 little-endian 64-bit words
NWV_HD void blake2b_compress(blake2b_state& s, const u64p m[16], uint32_t add_bytes, bool last) {
    s.t += add_bytes;
    u64p v[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        v[i] = s.h[i];
        v[8 + i] = u64p{BLAKE2B_IV32[2 * i], BLAKE2B_IV32[2 * i + 1]};
    }
    v[12] = xor2(v[12], u64p{(uint32_t)s.t, (uint32_t)(s.t >> 32)});
    if (last) v[14] = u64p{~v[14].lo, ~v[14].hi};
#pragma unroll
    for (int r = 0; r < 12; r++) {
#define NWV_B2G(a, b, c, d, x, y)                       \
    v[a] = add(add(v[a], v[b]), m[BLAKE2B_SIGMA[r][x]]); \
    v[d] = swap_halves(xor2(v[d], v[a]));               \
    v[c] = add(v[c], v[d]);                             \
    v[b] = rotr(xor2(v[b], v[c]), 24);                  \
    v[a] = add(add(v[a], v[b]), m[BLAKE2B_SIGMA[r][y]]); \
    v[d] = rotr(xor2(v[d], v[a]), 16);                  \
    v[c] = add(v[c], v[d]);                             \
    v[b] = rotr(xor2(v[b], v[c]), 63);
        NWV_B2G(0, 4, 8, 12, 0, 1)
        NWV_B2G(1, 5, 9, 13, 2, 3)
        NWV_B2G(2, 6, 10, 14, 4, 5)
        NWV_B2G(3, 7, 11, 15, 6, 7)
        NWV_B2G(0, 5, 10, 15, 8, 9)
        NWV_B2G(1, 6, 11, 12, 10, 11)
        NWV_B2G(2, 7, 8, 13, 12, 13)
        NWV_B2G(3, 4, 9, 14, 14, 15)
#undef NWV_B2G
        if ((r & 1) == 1) NWV_SEQ();
    }
#pragma unroll
    for (int i = 0; i < 8; i++) s.h[i] = xor2(s.h[i], xor2(v[i], v[8 + i]));
}

NWV_HD void blake2b_digest256(const blake2b_state& s, uint32_t out[8]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        out[2 * i] = s.h[i].lo;
        out[2 * i + 1] = s.h[i].hi;
    }
}

}  // namespace nwv
