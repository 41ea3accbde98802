// sha512.h -- SHA-512 (FIPS 180-4) for one message per lane on gfx950.
//
// Replaces sha2 0.9.9 (/root/reference/Cargo.lock:3845) as used by ed25519-consensus for the
// challenge k = SHA-512(R || A || M).  64-bit words are kept as two independent 32-bit
// VGPRs (no register-pair constraints): rotates are two v_alignbit_b32, additions are
// v_add_co_u32 / v_addc_co_u32.  The input stream is produced word by word by a
// caller-supplied functor so the kernel can splice R, A and an unaligned message in place.
#pragma once
#include "fe25519.h"

namespace nwv {

struct u64p {
    uint32_t lo, hi;
};

// round constants as (lo, hi) pairs; a namespace-scope constexpr table folds into immediates
static constexpr uint32_t SHA512_K32[160] = {
    0xd728ae22u, 0x428a2f98u, 0x23ef65cdu, 0x71374491u, 0xec4d3b2fu, 0xb5c0fbcfu, 0x8189dbbcu, 0xe9b5dba5u,
    0xf348b538u, 0x3956c25bu, 0xb605d019u, 0x59f111f1u, 0xaf194f9bu, 0x923f82a4u, 0xda6d8118u, 0xab1c5ed5u,
    0xa3030242u, 0xd807aa98u, 0x45706fbeu, 0x12835b01u, 0x4ee4b28cu, 0x243185beu, 0xd5ffb4e2u, 0x550c7dc3u,
    0xf27b896fu, 0x72be5d74u, 0x3b1696b1u, 0x80deb1feu, 0x25c71235u, 0x9bdc06a7u, 0xcf692694u, 0xc19bf174u,
    0x9ef14ad2u, 0xe49b69c1u, 0x384f25e3u, 0xefbe4786u, 0x8b8cd5b5u, 0x0fc19dc6u, 0x77ac9c65u, 0x240ca1ccu,
    0x592b0275u, 0x2de92c6fu, 0x6ea6e483u, 0x4a7484aau, 0xbd41fbd4u, 0x5cb0a9dcu, 0x831153b5u, 0x76f988dau,
    0xee66dfabu, 0x983e5152u, 0x2db43210u, 0xa831c66du, 0x98fb213fu, 0xb00327c8u, 0xbeef0ee4u, 0xbf597fc7u,
    0x3da88fc2u, 0xc6e00bf3u, 0x930aa725u, 0xd5a79147u, 0xe003826fu, 0x06ca6351u, 0x0a0e6e70u, 0x14292967u,
    0x46d22ffcu, 0x27b70a85u, 0x5c26c926u, 0x2e1b2138u, 0x5ac42aedu, 0x4d2c6dfcu, 0x9d95b3dfu, 0x53380d13u,
    0x8baf63deu, 0x650a7354u, 0x3c77b2a8u, 0x766a0abbu, 0x47edaee6u, 0x81c2c92eu, 0x1482353bu, 0x92722c85u,
    0x4cf10364u, 0xa2bfe8a1u, 0xbc423001u, 0xa81a664bu, 0xd0f89791u, 0xc24b8b70u, 0x0654be30u, 0xc76c51a3u,
    0xd6ef5218u, 0xd192e819u, 0x5565a910u, 0xd6990624u, 0x5771202au, 0xf40e3585u, 0x32bbd1b8u, 0x106aa070u,
    0xb8d2d0c8u, 0x19a4c116u, 0x5141ab53u, 0x1e376c08u, 0xdf8eeb99u, 0x2748774cu, 0xe19b48a8u, 0x34b0bcb5u,
    0xc5c95a63u, 0x391c0cb3u, 0xe3418acbu, 0x4ed8aa4au, 0x7763e373u, 0x5b9cca4fu, 0xd6b2b8a3u, 0x682e6ff3u,
    0x5defb2fcu, 0x748f82eeu, 0x43172f60u, 0x78a5636fu, 0xa1f0ab72u, 0x84c87814u, 0x1a6439ecu, 0x8cc70208u,
    0x23631e28u, 0x90befffau, 0xde82bde9u, 0xa4506cebu, 0xb2c67915u, 0xbef9a3f7u, 0xe372532bu, 0xc67178f2u,
    0xea26619cu, 0xca273eceu, 0x21c0c207u, 0xd186b8c7u, 0xcde0eb1eu, 0xeada7dd6u, 0xee6ed178u, 0xf57d4f7fu,
    0x72176fbau, 0x06f067aau, 0xa2c898a6u, 0x0a637dc5u, 0xbef90daeu, 0x113f9804u, 0x131c471bu, 0x1b710b35u,
    0x23047d84u, 0x28db77f5u, 0x40c72493u, 0x32caab7bu, 0x15c9bebcu, 0x3c9ebe0au, 0x9c100d4cu, 0x431d67c4u,
    0xcb3e42b6u, 0x4cc5d4beu, 0xfc657e2au, 0x597f299cu, 0x3ad6faecu, 0x5fcb6fabu, 0x4a475817u, 0x6c44198cu};

NWV_HD uint32_t funnel_r(uint32_t hi, uint32_t lo, int n) {  // low 32 bits of (hi:lo) >> n, 0 < n < 32
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, n);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> n);
#endif
}
NWV_HD u64p rotr(u64p x, int n) {  // 0 < n < 64, n != 32
    if (n < 32) return u64p{funnel_r(x.hi, x.lo, n), funnel_r(x.lo, x.hi, n)};
    return u64p{funnel_r(x.lo, x.hi, n - 32), funnel_r(x.hi, x.lo, n - 32)};
}
NWV_HD u64p shr(u64p x, int n) {  // 0 < n < 32
    return u64p{funnel_r(x.hi, x.lo, n), x.hi >> n};
}
NWV_HD u64p add(u64p a, u64p b) {
#if defined(__HIP_DEVICE_COMPILE__)
    // exactly v_add_co_u32 + v_addc_co_u32 (the plain C form also materialises the carry as a
    // value with v_cndmask)
    unsigned c, c2;
    const uint32_t lo = __builtin_addc(a.lo, b.lo, 0u, &c);
    const uint32_t hi = __builtin_addc(a.hi, b.hi, c, &c2);
    return u64p{lo, hi};
#else
    const uint64_t t = (uint64_t)a.lo + b.lo;
    return u64p{(uint32_t)t, a.hi + b.hi + (uint32_t)(t >> 32)};
#endif
}
NWV_HD uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // one v_bitop3_b32 (a ^ b ^ c)
#else
    return a ^ b ^ c;
#endif
}
NWV_HD u64p xor3(u64p a, u64p b, u64p c) { return u64p{xor3_32(a.lo, b.lo, c.lo), xor3_32(a.hi, b.hi, c.hi)}; }
// Ch and Maj as one v_bitop3_b32 per half (truth tables 0xCA and 0xE8 over (x, y, z))
NWV_HD uint32_t bitop3_32(uint32_t x, uint32_t y, uint32_t z, int tt) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)(tt == 0xCA ? __builtin_amdgcn_bitop3_b32(x, y, z, 0xCA) : __builtin_amdgcn_bitop3_b32(x, y, z, 0xE8));
#else
    return tt == 0xCA ? ((x & y) ^ (~x & z)) : ((x & y) ^ (x & z) ^ (y & z));
#endif
}
NWV_HD u64p ch(u64p e, u64p f, u64p g) {
    return u64p{bitop3_32(e.lo, f.lo, g.lo, 0xCA), bitop3_32(e.hi, f.hi, g.hi, 0xCA)};
}
NWV_HD u64p maj(u64p a, u64p b, u64p c) {
    return u64p{bitop3_32(a.lo, b.lo, c.lo, 0xE8), bitop3_32(a.hi, b.hi, c.hi, 0xE8)};
}
NWV_HD uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

NWV_HD uint32_t ld_u32_unaligned(const uint8_t* p) {
    // message arenas are padded so that reading the aligned word after the last byte is safe
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* wp = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint64_t two = ((uint64_t)wp[1] << 32) | wp[0];
    return (uint32_t)(two >> sh);
}

struct sha512_state {
    u64p h[8];
};

NWV_HD void sha512_init(sha512_state& s) {
    const uint32_t IV[16] = {0xf3bcc908u, 0x6a09e667u, 0x84caa73bu, 0xbb67ae85u, 0xfe94f82bu, 0x3c6ef372u,
                             0x5f1d36f1u, 0xa54ff53au, 0xade682d1u, 0x510e527fu, 0x2b3e6c1fu, 0x9b05688cu,
                             0xfb41bd6bu, 0x1f83d9abu, 0x137e2179u, 0x5be0cd19u};
#pragma unroll
    for (int i = 0; i < 8; i++) s.h[i] = u64p{IV[2 * i], IV[2 * i + 1]};
}

// One compression; w[16] are the block's big-endian 64-bit words (consumed in place).  Inside,
// words are 64-bit values: additions are single v_lshl_add_u64 (no VCC carry chain), rotates
// are two v_alignbit_b32 on the halves.
NWV_HD uint64_t rotr64(uint64_t x, int n) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const u64p r = rotr(u64p{lo, hi}, n);
    return ((uint64_t)r.hi << 32) | r.lo;
}
NWV_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    return ((uint64_t)xor3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
           xor3_32((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
NWV_HD uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c, int tt) {
    return ((uint64_t)bitop3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32), tt) << 32) |
           bitop3_32((uint32_t)a, (uint32_t)b, (uint32_t)c, tt);
}
NWV_HD uint64_t j64(u64p x) { return ((uint64_t)x.hi << 32) | x.lo; }
#define NWV_SHA_ROUND(r, wr)                                                                   \
    do {                                                                                       \
        const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));              \
        const uint64_t kr = ((uint64_t)SHA512_K32[2 * (r) + 1] << 32) | SHA512_K32[2 * (r)];    \
        const uint64_t t1 = h + S1 + bitop3_64(e, f, g, 0xCA) + kr + (wr);                     \
        const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));              \
        const uint64_t t2 = S0 + bitop3_64(a, b, c, 0xE8);                                     \
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;                     \
    } while (0)

NWV_HD void sha512_compress(sha512_state& s, u64p win[16]) {
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = j64(win[i]);
    uint64_t a = j64(s.h[0]), b = j64(s.h[1]), c = j64(s.h[2]), d = j64(s.h[3]);
    uint64_t e = j64(s.h[4]), f = j64(s.h[5]), g = j64(s.h[6]), h = j64(s.h[7]);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        NWV_SHA_ROUND(j, w[j]);
        if ((j & 3) == 3) NWV_SEQ();
    }
#pragma unroll 1
    for (int grp = 1; grp < 5; grp++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
            const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), w15 >> 7);
            const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), w2 >> 6);
            const uint64_t wr = w[j] + s0 + w[(j + 9) & 15] + s1;
            w[j] = wr;
            NWV_SHA_ROUND(16 * grp + j, wr);
            if ((j & 3) == 3) NWV_SEQ();
        }
    }
    const uint64_t o[8] = {a, b, c, d, e, f, g, h};
#pragma unroll
    for (int i = 0; i < 8; i++) s.h[i] = add(s.h[i], u64p{(uint32_t)o[i], (uint32_t)(o[i] >> 32)});
}
#undef NWV_SHA_ROUND

// stream word at byte position pos: v = raw little-endian word, trimmed to `total` bytes and
// carrying the 0x80 terminator when the stream ends inside it
NWV_HD uint32_t sha_pad_word(uint32_t v, uint32_t pos, uint32_t total) {
    if (pos >= total + 4) return 0u;
    if (pos + 4 > total) {
        const uint32_t keep = (pos < total) ? (total - pos) : 0u;  // 0..3
        const uint32_t mask = keep ? (0xffffffffu >> (8 * (4 - keep))) : 0u;
        v &= mask;
        if (pos <= total) v |= 0x80u << (8 * (total - pos));
    }
    return v;
}

// SHA-512 of  prefix (NP words held in registers, NP <= 32)  ||  msg[0 .. mlen)  where msg
// word j is ldmsg(j) (little-endian 32-bit words).  Block 0 is emitted with compile-time word
// indices so the prefix never needs dynamic register indexing; later blocks are message only.
template <int NP, class LdMsg>
NWV_HD void sha512_prefixed(sha512_state& s, const uint32_t (&prefix)[NP], uint32_t mlen, LdMsg ldmsg) {
    static_assert(NP <= 32, "prefix must fit in the first block");
    sha512_init(s);
    const uint32_t total = 4 * NP + mlen;
    const uint32_t nblocks = (total + 17 + 127) / 128;
    u64p w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
        uint32_t half[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int q = 2 * t + u;
            const uint32_t pos = 4u * q;
            uint32_t v;
            if (q < NP) v = prefix[q];
            else v = (pos < total) ? ldmsg((uint32_t)(q - NP)) : 0u;
            half[u] = bswap32(sha_pad_word(v, pos, total));
        }
        w[t] = u64p{half[1], half[0]};
    }
    if (nblocks == 1) w[15] = u64p{total * 8, total >> 29};
    sha512_compress(s, w);
#pragma unroll 1
    for (uint32_t blk = 1; blk < nblocks; blk++) {
#pragma unroll
        for (int t = 0; t < 16; t++) {
            uint32_t half[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t q = blk * 32 + 2 * t + u;
                const uint32_t pos = 4u * q;
                const uint32_t v = (pos < total) ? ldmsg(q - NP) : 0u;
                half[u] = bswap32(sha_pad_word(v, pos, total));
            }
            w[t] = u64p{half[1], half[0]};
        }
        if (blk == nblocks - 1) w[15] = u64p{total * 8, total >> 29};  // 128-bit length
        sha512_compress(s, w);
    }
}

// 32 consecutive little-endian message words from byte address p (any alignment; the arena is
// padded past its last message): eight 16-byte loads from the dword-aligned address below p,
// one more dword, and a funnel shift by p's byte offset
NWV_HD void ld_block_unaligned(const uint8_t* p, uint32_t out[32]) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* base = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    uint32_t raw[33];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint4 t;
        __builtin_memcpy(&t, base + 4 * k, 16);
        raw[4 * k] = t.x; raw[4 * k + 1] = t.y; raw[4 * k + 2] = t.z; raw[4 * k + 3] = t.w;
    }
    raw[32] = base[32];
#pragma unroll
    for (int j = 0; j < 32; j++) out[j] = funnel_r(raw[j + 1], raw[j], (int)sh);
}

// SHA-512 of prefix || msg[0 .. mlen): sha512_prefixed with the message read from memory; every
// block that lies wholly inside the message is fetched as one 128-byte unaligned block (nine
// vector loads instead of sixty-four dword loads and a per-word padding test).
template <int NP>
NWV_HD void sha512_prefixed_msg(sha512_state& s, const uint32_t (&prefix)[NP], const uint8_t* msg, uint32_t mlen) {
    static_assert(NP <= 32, "prefix must fit in the first block");
    sha512_init(s);
    const uint32_t total = 4 * NP + mlen;
    const uint32_t nblocks = (total + 17 + 127) / 128;
    u64p w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
        uint32_t half[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int q = 2 * t + u;
            const uint32_t pos = 4u * q;
            uint32_t v;
            if (q < NP) v = prefix[q];
            else v = (pos < total) ? ld_u32_unaligned(msg + 4 * (q - NP)) : 0u;
            half[u] = bswap32(sha_pad_word(v, pos, total));
        }
        w[t] = u64p{half[1], half[0]};
    }
    if (nblocks == 1) w[15] = u64p{total * 8, total >> 29};
    sha512_compress(s, w);
#pragma unroll 1
    for (uint32_t blk = 1; blk < nblocks; blk++) {
        if (blk * 128 + 128 <= total) {
            uint32_t m[32];
            ld_block_unaligned(msg + (blk * 128 - 4 * NP), m);
#pragma unroll
            for (int t = 0; t < 16; t++) w[t] = u64p{bswap32(m[2 * t + 1]), bswap32(m[2 * t])};
        } else {
#pragma unroll
            for (int t = 0; t < 16; t++) {
                uint32_t half[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const uint32_t q = blk * 32 + 2 * t + u;
                    const uint32_t pos = 4u * q;
                    const uint32_t v = (pos < total) ? ld_u32_unaligned(msg + 4 * (q - NP)) : 0u;
                    half[u] = bswap32(sha_pad_word(v, pos, total));
                }
                w[t] = u64p{half[1], half[0]};
            }
            if (blk == nblocks - 1) w[15] = u64p{total * 8, total >> 29};  // 128-bit length
        }
        sha512_compress(s, w);
    }
}

// digest as 16 little-endian 32-bit words of the 64 output bytes
NWV_HD void sha512_digest_words(const sha512_state& s, uint32_t out[16]) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        out[2 * i] = bswap32(s.h[i].hi);
        out[2 * i + 1] = bswap32(s.h[i].lo);
    }
}

}  // namespace nwv
