/*
 * nwv_oracle.c -- TEST INFRASTRUCTURE ONLY (see nwv_oracle.h for scope and provenance).
 *
 * A plain-C restatement of the published algorithms of the third-party crates that
 * implement the reference's Ed25519 / Blake2b hot path.  Citations point at the
 * reference call sites (file:line under /root/reference) and at SURVEY.md Appendix A,
 * which restates the ed25519-consensus 2.0.1 / ZIP-215 contract.
 */
#include "nwv_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ======================================================================== */
/* SHA-512 (FIPS 180-4) -- sha2 0.9.9, used by ed25519-consensus for k      */
/* ======================================================================== */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static inline uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void sha512_block(uint64_t H[8], const uint8_t* p) {
    uint64_t W[80];
    for (int i = 0; i < 16; i++) {
        uint64_t w = 0;
        for (int j = 0; j < 8; j++) w = (w << 8) | p[8 * i + j];
        W[i] = w;
    }
    for (int i = 16; i < 80; i++) {
        uint64_t s0 = ror64(W[i - 15], 1) ^ ror64(W[i - 15], 8) ^ (W[i - 15] >> 7);
        uint64_t s1 = ror64(W[i - 2], 19) ^ ror64(W[i - 2], 61) ^ (W[i - 2] >> 6);
        W[i] = W[i - 16] + s0 + W[i - 7] + s1;
    }
    uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    for (int i = 0; i < 80; i++) {
        uint64_t S1 = ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41);
        uint64_t ch = (e & f) ^ (~e & g);
        uint64_t t1 = h + S1 + ch + K512[i] + W[i];
        uint64_t S0 = ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
        uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint64_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

typedef struct {
    uint64_t H[8];
    uint8_t buf[128];
    size_t fill;
    uint64_t total;
} sha512_ctx;

static void sha512_init(sha512_ctx* c) {
    static const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                   0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                   0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    memcpy(c->H, IV, sizeof IV);
    c->fill = 0;
    c->total = 0;
}
static void sha512_update(sha512_ctx* c, const uint8_t* m, size_t n) {
    c->total += n;
    while (n) {
        size_t take = 128 - c->fill;
        if (take > n) take = n;
        memcpy(c->buf + c->fill, m, take);
        c->fill += take; m += take; n -= take;
        if (c->fill == 128) { sha512_block(c->H, c->buf); c->fill = 0; }
    }
}
static void sha512_final(sha512_ctx* c, uint8_t out[64]) {
    uint64_t bits = c->total * 8;
    uint8_t pad = 0x80;
    sha512_update(c, &pad, 1);
    uint8_t z = 0;
    while (c->fill != 112) sha512_update(c, &z, 1);
    uint8_t len[16] = {0};
    for (int i = 0; i < 8; i++) len[15 - i] = (uint8_t)(bits >> (8 * i));
    sha512_update(c, len, 16);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(c->H[i] >> (56 - 8 * j));
}
void or_sha512(const uint8_t* m, size_t n, uint8_t out[64]) {
    sha512_ctx c;
    sha512_init(&c);
    sha512_update(&c, m, n);
    sha512_final(&c, out);
}

/* ======================================================================== */
/* BLAKE2b, digest_length 32 (RFC 7693) -- fastcrypto::blake2b_256 over     */
/* blake2 0.9.2 VarBlake2b::new(32); types/src/primary.rs:65-73,209-227      */
/* ======================================================================== */
static const uint64_t B2IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint8_t B2SIGMA[12][16] = {
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

typedef struct {
    uint64_t h[8];
    uint64_t t;
    uint8_t buf[128];
    size_t fill;
} b2_ctx;

static void b2_compress(b2_ctx* c, const uint8_t* blk, int last) {
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; i++) {
        uint64_t w = 0;
        for (int j = 7; j >= 0; j--) w = (w << 8) | blk[8 * i + j];
        m[i] = w;
    }
    for (int i = 0; i < 8; i++) { v[i] = c->h[i]; v[i + 8] = B2IV[i]; }
    v[12] ^= c->t;
    if (last) v[14] = ~v[14];
#define B2G(a, b, cc, d, x, y)                      \
    do {                                            \
        v[a] = v[a] + v[b] + (x); v[d] = ror64(v[d] ^ v[a], 32); \
        v[cc] = v[cc] + v[d]; v[b] = ror64(v[b] ^ v[cc], 24);    \
        v[a] = v[a] + v[b] + (y); v[d] = ror64(v[d] ^ v[a], 16); \
        v[cc] = v[cc] + v[d]; v[b] = ror64(v[b] ^ v[cc], 63);    \
    } while (0)
    for (int r = 0; r < 12; r++) {
        const uint8_t* s = B2SIGMA[r];
        B2G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B2G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B2G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B2G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B2G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B2G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B2G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B2G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef B2G
    for (int i = 0; i < 8; i++) c->h[i] ^= v[i] ^ v[i + 8];
}
static void b2_init(b2_ctx* c) {
    memcpy(c->h, B2IV, sizeof B2IV);
    c->h[0] ^= 0x01010000ULL ^ 32; /* depth 1, fanout 1, keylen 0, digest_length 32 */
    c->t = 0;
    c->fill = 0;
}
static void b2_update(b2_ctx* c, const uint8_t* m, size_t n) {
    while (n) {
        if (c->fill == 128) { /* only compress once more input is known to follow */
            c->t += 128;
            b2_compress(c, c->buf, 0);
            c->fill = 0;
        }
        size_t take = 128 - c->fill;
        if (take > n) take = n;
        memcpy(c->buf + c->fill, m, take);
        c->fill += take; m += take; n -= take;
    }
}
static void b2_final(b2_ctx* c, uint8_t out[32]) {
    c->t += c->fill;
    memset(c->buf + c->fill, 0, 128 - c->fill);
    b2_compress(c, c->buf, 1);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(c->h[i] >> (8 * j));
}
void or_blake2b256(const uint8_t* m, size_t n, uint8_t out[32]) {
    b2_ctx c;
    b2_init(&c);
    b2_update(&c, m, n);
    b2_final(&c, out);
}
void or_batch_digest(size_t ntx, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                     uint8_t out[32]) {
    b2_ctx c;
    b2_init(&c);
    for (size_t i = 0; i < ntx; i++) b2_update(&c, base + off[i], (size_t)len[i]);
    b2_final(&c, out);
}
static uint64_t ld64le(const uint8_t* p) {
    uint64_t w = 0;
    for (int j = 7; j >= 0; j--) w = (w << 8) | p[j];
    return w;
}
/* types/src/worker.rs:44-62 serialized_batch_digest + :71-80 read_one_transaction.
 * Layout: [u32 variant][u64 count][(u64 len, bytes)]*.  A read past the end of the buffer is
 * reported as DigestError::InvalidArgumentError(offset) where offset is the start of the u64
 * field being read (the reference panics on a slice end past the buffer). */
int or_batch_digest_serialized(const uint8_t* buf, size_t n, uint8_t out[32], int64_t* err_offset) {
    size_t off = 4;
    if (off + 8 > n) { *err_offset = (int64_t)off; return -1; }
    uint64_t cnt = ld64le(buf + off);
    off += 8;
    b2_ctx c;
    b2_init(&c);
    for (uint64_t i = 0; i < cnt; i++) {
        if (off + 8 > n) { *err_offset = (int64_t)off; return -1; }
        uint64_t l = ld64le(buf + off);
        if (l > n - off - 8) { *err_offset = (int64_t)off; return -1; }
        b2_update(&c, buf + off + 8, (size_t)l);
        off += 8 + (size_t)l;
    }
    b2_final(&c, out);
    *err_offset = -1;
    return 0;
}

/* ======================================================================== */
/* ChaCha20 block function (djb variant: 64-bit counter, zero nonce) -- the  */
/* deterministic stand-in for OsRng in batch::Verifier::verify (z_i draws)    */
/* ======================================================================== */
static inline uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static void chacha_block(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
    uint32_t s[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
    uint32_t x[16];
    memcpy(x, s, sizeof s);
#define QR(a, b, c, d)                                   \
    x[a] += x[b]; x[d] = rol32(x[d] ^ x[a], 16);         \
    x[c] += x[d]; x[b] = rol32(x[b] ^ x[c], 12);         \
    x[a] += x[b]; x[d] = rol32(x[d] ^ x[a], 8);          \
    x[c] += x[d]; x[b] = rol32(x[b] ^ x[c], 7);
    for (int i = 0; i < 10; i++) {
        QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
        QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
    }
#undef QR
    for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}
void or_chacha20_stream(const uint8_t key[32], uint64_t counter0, uint8_t* out, size_t nblocks) {
    uint32_t k[8];
    for (int i = 0; i < 8; i++)
        k[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) |
               ((uint32_t)key[4 * i + 2] << 16) | ((uint32_t)key[4 * i + 3] << 24);
    for (size_t b = 0; b < nblocks; b++) {
        uint32_t w[16];
        chacha_block(k, counter0 + b, w);
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 4; j++) out[64 * b + 4 * i + j] = (uint8_t)(w[i] >> (8 * j));
    }
}

/* ======================================================================== */
/* Field arithmetic mod p = 2^255 - 19, radix 2^51 (dalek u64_backend)      */
/* ======================================================================== */
#define M51 ((1ULL << 51) - 1)
typedef struct { uint64_t v[5]; } fe;

static const fe FE_ZERO = {{0, 0, 0, 0, 0}};
static const fe FE_ONE = {{1, 0, 0, 0, 0}};
static const fe FE_D = {{0x34dca135978a3ULL, 0x1a8283b156ebdULL, 0x5e7a26001c029ULL,
                         0x739c663a03cbbULL, 0x52036cee2b6ffULL}};
static const fe FE_D2 = {{0x69b9426b2f159ULL, 0x35050762add7aULL, 0x3cf44c0038052ULL,
                          0x6738cc7407977ULL, 0x2406d9dc56dffULL}};
static const fe FE_SQRTM1 = {{0x61b274a0ea0b0ULL, 0xd5a5fc8f189dULL, 0x7ef5e9cbd0c60ULL,
                              0x78595a6804c9eULL, 0x2b8324804fc1dULL}};

static inline void fe_weak(fe* h) {
    uint64_t c;
    c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
    c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
    c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
    c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
    c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
}
/* FieldElement51::from_bytes: the high bit is ignored; values >= p are kept unreduced. */
static void fe_frombytes(fe* h, const uint8_t s[32]) {
    uint64_t w0 = ld64le(s), w1 = ld64le(s + 8), w2 = ld64le(s + 16), w3 = ld64le(s + 24);
    h->v[0] = w0 & M51;
    h->v[1] = ((w0 >> 51) | (w1 << 13)) & M51;
    h->v[2] = ((w1 >> 38) | (w2 << 26)) & M51;
    h->v[3] = ((w2 >> 25) | (w3 << 39)) & M51;
    h->v[4] = (w3 >> 12) & M51;
}
static void fe_tobytes(uint8_t s[32], const fe* f) {
    fe h = *f;
    fe_weak(&h);
    uint64_t q = (h.v[0] + 19) >> 51;
    q = (h.v[1] + q) >> 51;
    q = (h.v[2] + q) >> 51;
    q = (h.v[3] + q) >> 51;
    q = (h.v[4] + q) >> 51;
    h.v[0] += 19 * q;
    h.v[1] += h.v[0] >> 51; h.v[0] &= M51;
    h.v[2] += h.v[1] >> 51; h.v[1] &= M51;
    h.v[3] += h.v[2] >> 51; h.v[2] &= M51;
    h.v[4] += h.v[3] >> 51; h.v[3] &= M51;
    h.v[4] &= M51;
    uint64_t w[4];
    w[0] = h.v[0] | (h.v[1] << 51);
    w[1] = (h.v[1] >> 13) | (h.v[2] << 38);
    w[2] = (h.v[2] >> 26) | (h.v[3] << 25);
    w[3] = (h.v[3] >> 39) | (h.v[4] << 12);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
static inline void fe_add(fe* h, const fe* a, const fe* b) {
    for (int i = 0; i < 5; i++) h->v[i] = a->v[i] + b->v[i];
    fe_weak(h);
}
static inline void fe_sub(fe* h, const fe* a, const fe* b) {
    /* (a + 16p) - b, as FieldElement51::sub */
    h->v[0] = (a->v[0] + 36028797018963664ULL) - b->v[0];
    h->v[1] = (a->v[1] + 36028797018963952ULL) - b->v[1];
    h->v[2] = (a->v[2] + 36028797018963952ULL) - b->v[2];
    h->v[3] = (a->v[3] + 36028797018963952ULL) - b->v[3];
    h->v[4] = (a->v[4] + 36028797018963952ULL) - b->v[4];
    fe_weak(h);
}
static inline void fe_neg(fe* h, const fe* a) { fe_sub(h, &FE_ZERO, a); }
static inline void fe_mul(fe* h, const fe* a, const fe* b) {
    const uint64_t a0 = a->v[0], a1 = a->v[1], a2 = a->v[2], a3 = a->v[3], a4 = a->v[4];
    const uint64_t b0 = b->v[0], b1 = b->v[1], b2 = b->v[2], b3 = b->v[3], b4 = b->v[4];
    const uint64_t b1_19 = 19 * b1, b2_19 = 19 * b2, b3_19 = 19 * b3, b4_19 = 19 * b4;
    u128 c0 = (u128)a0 * b0 + (u128)a4 * b1_19 + (u128)a3 * b2_19 + (u128)a2 * b3_19 + (u128)a1 * b4_19;
    u128 c1 = (u128)a1 * b0 + (u128)a0 * b1 + (u128)a4 * b2_19 + (u128)a3 * b3_19 + (u128)a2 * b4_19;
    u128 c2 = (u128)a2 * b0 + (u128)a1 * b1 + (u128)a0 * b2 + (u128)a4 * b3_19 + (u128)a3 * b4_19;
    u128 c3 = (u128)a3 * b0 + (u128)a2 * b1 + (u128)a1 * b2 + (u128)a0 * b3 + (u128)a4 * b4_19;
    u128 c4 = (u128)a4 * b0 + (u128)a3 * b1 + (u128)a2 * b2 + (u128)a1 * b3 + (u128)a0 * b4;
    c1 += (uint64_t)(c0 >> 51);
    c2 += (uint64_t)(c1 >> 51);
    c3 += (uint64_t)(c2 >> 51);
    c4 += (uint64_t)(c3 >> 51);
    uint64_t carry = (uint64_t)(c4 >> 51);
    h->v[0] = (uint64_t)c0 & M51;
    h->v[1] = (uint64_t)c1 & M51;
    h->v[2] = (uint64_t)c2 & M51;
    h->v[3] = (uint64_t)c3 & M51;
    h->v[4] = (uint64_t)c4 & M51;
    h->v[0] += carry * 19;
    h->v[1] += h->v[0] >> 51;
    h->v[0] &= M51;
}
static inline void fe_sq(fe* h, const fe* a) { fe_mul(h, a, a); }
static void fe_sqn(fe* h, const fe* a, int n) {
    fe_sq(h, a);
    for (int i = 1; i < n; i++) fe_sq(h, h);
}
/* returns (x^(2^250-1), x^11) as in dalek's pow22501 */
static void fe_pow22501(fe* t19, fe* t3, const fe* x) {
    fe t0, t1, t2, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15, t16, t17, t18;
    fe_sq(&t0, x);
    fe_sqn(&t1, &t0, 2);
    fe_mul(&t2, x, &t1);
    fe_mul(t3, &t0, &t2);
    fe_sq(&t4, t3);
    fe_mul(&t5, &t2, &t4);
    fe_sqn(&t6, &t5, 5);
    fe_mul(&t7, &t6, &t5);
    fe_sqn(&t8, &t7, 10);
    fe_mul(&t9, &t8, &t7);
    fe_sqn(&t10, &t9, 20);
    fe_mul(&t11, &t10, &t9);
    fe_sqn(&t12, &t11, 10);
    fe_mul(&t13, &t12, &t7);
    fe_sqn(&t14, &t13, 50);
    fe_mul(&t15, &t14, &t13);
    fe_sqn(&t16, &t15, 100);
    fe_mul(&t17, &t16, &t15);
    fe_sqn(&t18, &t17, 50);
    fe_mul(t19, &t18, &t13);
}
static void fe_invert(fe* out, const fe* x) {
    fe t19, t3, t20;
    fe_pow22501(&t19, &t3, x);
    fe_sqn(&t20, &t19, 5);
    fe_mul(out, &t20, &t3);
}
static void fe_pow_p58(fe* out, const fe* x) { /* x^((p-5)/8) */
    fe t19, t3, t20;
    fe_pow22501(&t19, &t3, x);
    fe_sqn(&t20, &t19, 2);
    fe_mul(out, x, &t20);
}
static int fe_eq(const fe* a, const fe* b) {
    uint8_t x[32], y[32];
    fe_tobytes(x, a);
    fe_tobytes(y, b);
    return memcmp(x, y, 32) == 0;
}
static int fe_is_negative(const fe* a) {
    uint8_t x[32];
    fe_tobytes(x, a);
    return x[0] & 1;
}
static int fe_is_zero(const fe* a) {
    uint8_t x[32];
    fe_tobytes(x, a);
    uint8_t acc = 0;
    for (int i = 0; i < 32; i++) acc |= x[i];
    return acc == 0;
}
/* FieldElement::sqrt_ratio_i (dalek): returns was_nonzero_square, r = nonneg sqrt(u/v) */
static int fe_sqrt_ratio_i(fe* r, const fe* u, const fe* v) {
    fe v3, v7, t, uv3, uv7, check, neg_u, neg_u_i, r_prime;
    fe_sq(&t, v);
    fe_mul(&v3, &t, v);
    fe_sq(&t, &v3);
    fe_mul(&v7, &t, v);
    fe_mul(&uv3, u, &v3);
    fe_mul(&uv7, u, &v7);
    fe_pow_p58(&t, &uv7);
    fe_mul(r, &uv3, &t);
    fe_sq(&t, r);
    fe_mul(&check, v, &t);
    fe_neg(&neg_u, u);
    fe_mul(&neg_u_i, &neg_u, &FE_SQRTM1);
    int correct = fe_eq(&check, u);
    int flipped = fe_eq(&check, &neg_u);
    int flipped_i = fe_eq(&check, &neg_u_i);
    fe_mul(&r_prime, r, &FE_SQRTM1);
    if (flipped | flipped_i) *r = r_prime;
    if (fe_is_negative(r)) fe_neg(r, r);
    return correct | flipped;
}

/* ======================================================================== */
/* Edwards points (extended twisted Edwards, a = -1), dalek formulas          */
/* ======================================================================== */
typedef struct { fe X, Y, Z, T; } ge_ext;
typedef struct { fe X, Y, Z; } ge_proj;
typedef struct { fe X, Y, Z, T; } ge_comp;
typedef struct { fe YpX, YmX, Z, T2d; } ge_pniels;
typedef struct { fe ypx, ymx, xy2d; } ge_aniels;

static void ge_identity(ge_ext* p) { p->X = FE_ZERO; p->Y = FE_ONE; p->Z = FE_ONE; p->T = FE_ZERO; }
static void comp_to_ext(ge_ext* r, const ge_comp* c) {
    fe_mul(&r->X, &c->X, &c->T);
    fe_mul(&r->Y, &c->Y, &c->Z);
    fe_mul(&r->Z, &c->Z, &c->T);
    fe_mul(&r->T, &c->X, &c->Y);
}
static void comp_to_proj(ge_proj* r, const ge_comp* c) {
    fe_mul(&r->X, &c->X, &c->T);
    fe_mul(&r->Y, &c->Y, &c->Z);
    fe_mul(&r->Z, &c->Z, &c->T);
}
static void ext_to_proj(ge_proj* r, const ge_ext* p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }
static void proj_dbl(ge_comp* c, const ge_proj* p) {
    fe XX, YY, ZZ2, XpY, XpY2;
    fe_sq(&XX, &p->X);
    fe_sq(&YY, &p->Y);
    fe_sq(&ZZ2, &p->Z);
    fe_add(&ZZ2, &ZZ2, &ZZ2);
    fe_add(&XpY, &p->X, &p->Y);
    fe_sq(&XpY2, &XpY);
    fe_add(&c->Y, &YY, &XX);
    fe_sub(&c->X, &XpY2, &c->Y);
    fe_sub(&c->Z, &YY, &XX);
    fe_sub(&c->T, &ZZ2, &c->Z);
}
static void ext_dbl(ge_ext* r, const ge_ext* p) {
    ge_proj q;
    ge_comp c;
    ext_to_proj(&q, p);
    proj_dbl(&c, &q);
    comp_to_ext(r, &c);
}
static void ext_to_pniels(ge_pniels* n, const ge_ext* p) {
    fe_add(&n->YpX, &p->Y, &p->X);
    fe_sub(&n->YmX, &p->Y, &p->X);
    n->Z = p->Z;
    fe_mul(&n->T2d, &p->T, &FE_D2);
}
static void ext_add_pniels(ge_comp* c, const ge_ext* p, const ge_pniels* q) {
    fe YpX, YmX, PP, MM, TT2d, ZZ, ZZ2;
    fe_add(&YpX, &p->Y, &p->X);
    fe_sub(&YmX, &p->Y, &p->X);
    fe_mul(&PP, &YpX, &q->YpX);
    fe_mul(&MM, &YmX, &q->YmX);
    fe_mul(&TT2d, &p->T, &q->T2d);
    fe_mul(&ZZ, &p->Z, &q->Z);
    fe_add(&ZZ2, &ZZ, &ZZ);
    fe_sub(&c->X, &PP, &MM);
    fe_add(&c->Y, &PP, &MM);
    fe_add(&c->Z, &ZZ2, &TT2d);
    fe_sub(&c->T, &ZZ2, &TT2d);
}
static void ext_sub_pniels(ge_comp* c, const ge_ext* p, const ge_pniels* q) {
    fe YpX, YmX, PM, MP, TT2d, ZZ, ZZ2;
    fe_add(&YpX, &p->Y, &p->X);
    fe_sub(&YmX, &p->Y, &p->X);
    fe_mul(&PM, &YpX, &q->YmX);
    fe_mul(&MP, &YmX, &q->YpX);
    fe_mul(&TT2d, &p->T, &q->T2d);
    fe_mul(&ZZ, &p->Z, &q->Z);
    fe_add(&ZZ2, &ZZ, &ZZ);
    fe_sub(&c->X, &PM, &MP);
    fe_add(&c->Y, &PM, &MP);
    fe_sub(&c->Z, &ZZ2, &TT2d);
    fe_add(&c->T, &ZZ2, &TT2d);
}
static void ext_add_aniels(ge_comp* c, const ge_ext* p, const ge_aniels* q) {
    fe YpX, YmX, PP, MM, Txy2d, Z2;
    fe_add(&YpX, &p->Y, &p->X);
    fe_sub(&YmX, &p->Y, &p->X);
    fe_mul(&PP, &YpX, &q->ypx);
    fe_mul(&MM, &YmX, &q->ymx);
    fe_mul(&Txy2d, &p->T, &q->xy2d);
    fe_add(&Z2, &p->Z, &p->Z);
    fe_sub(&c->X, &PP, &MM);
    fe_add(&c->Y, &PP, &MM);
    fe_add(&c->Z, &Z2, &Txy2d);
    fe_sub(&c->T, &Z2, &Txy2d);
}
static void ext_sub_aniels(ge_comp* c, const ge_ext* p, const ge_aniels* q) {
    fe YpX, YmX, PM, MP, Txy2d, Z2;
    fe_add(&YpX, &p->Y, &p->X);
    fe_sub(&YmX, &p->Y, &p->X);
    fe_mul(&PM, &YpX, &q->ymx);
    fe_mul(&MP, &YmX, &q->ypx);
    fe_mul(&Txy2d, &p->T, &q->xy2d);
    fe_add(&Z2, &p->Z, &p->Z);
    fe_sub(&c->X, &PM, &MP);
    fe_add(&c->Y, &PM, &MP);
    fe_sub(&c->Z, &Z2, &Txy2d);
    fe_add(&c->T, &Z2, &Txy2d);
}
static void ext_add(ge_ext* r, const ge_ext* p, const ge_ext* q) {
    ge_pniels n;
    ge_comp c;
    ext_to_pniels(&n, q);
    ext_add_pniels(&c, p, &n);
    comp_to_ext(r, &c);
}
static void ext_neg(ge_ext* r, const ge_ext* p) {
    fe_neg(&r->X, &p->X);
    r->Y = p->Y;
    r->Z = p->Z;
    fe_neg(&r->T, &p->T);
}
static void ext_mul_by_cofactor(ge_ext* r, const ge_ext* p) {
    ext_dbl(r, p);
    ext_dbl(r, r);
    ext_dbl(r, r);
}
/* EdwardsPoint::is_identity: projective compare with (0:1:1) */
static int ext_is_identity(const ge_ext* p) {
    return fe_is_zero(&p->X) && fe_eq(&p->Y, &p->Z);
}
static void ext_compress(uint8_t s[32], const ge_ext* p) {
    fe zi, x, y;
    fe_invert(&zi, &p->Z);
    fe_mul(&x, &p->X, &zi);
    fe_mul(&y, &p->Y, &zi);
    fe_tobytes(s, &y);
    s[31] ^= (uint8_t)(fe_is_negative(&x) << 7);
}
/* CompressedEdwardsY::decompress (dalek): SURVEY.md Appendix A "Decode" */
static int ge_decompress(ge_ext* p, const uint8_t s[32]) {
    fe u, v, yy;
    fe_frombytes(&p->Y, s);
    p->Z = FE_ONE;
    fe_sq(&yy, &p->Y);
    fe_sub(&u, &yy, &FE_ONE);
    fe_mul(&v, &yy, &FE_D);
    fe_add(&v, &v, &FE_ONE);
    int ok = fe_sqrt_ratio_i(&p->X, &u, &v);
    if (!ok) return 0;
    if (s[31] >> 7) fe_neg(&p->X, &p->X);
    fe_mul(&p->T, &p->X, &p->Y);
    return 1;
}
int or_point_decompress_ok(const uint8_t s[32]) {
    ge_ext p;
    return ge_decompress(&p, s);
}

/* ======================================================================== */
/* Scalars mod l = 2^252 + 27742317777372353535851937790883648493            */
/* ======================================================================== */
static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};
static const uint64_t MU64[5] = {0xed9ce5a30a2c131bULL, 0x2106215d086329a7ULL, 0xffffffffffffffebULL,
                                 0xffffffffffffffffULL, 0xfULL};
typedef struct { uint64_t v[4]; } sc; /* canonical, little-endian words */

/* Barrett reduction (HAC 14.42, b = 2^64, k = 4) of a 512-bit x into [0, l) */
static void sc_reduce_words(sc* r, const uint64_t x[8]) {
    uint64_t q1[5], q2[10] = {0}, r2[5] = {0}, rr[5];
    for (int i = 0; i < 5; i++) q1[i] = x[3 + i];
    for (int i = 0; i < 5; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 5; j++) {
            u128 t = (u128)q1[i] * MU64[j] + q2[i + j] + carry;
            q2[i + j] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        }
        q2[i + 5] = carry;
    }
    uint64_t q3[5];
    for (int i = 0; i < 5; i++) q3[i] = q2[5 + i];
    for (int i = 0; i < 5; i++) { /* r2 = (q3 * l) mod 2^320 */
        uint64_t carry = 0;
        for (int j = 0; j < 4 && i + j < 5; j++) {
            u128 t = (u128)q3[i] * L64[j] + r2[i + j] + carry;
            r2[i + j] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        }
        if (i + 4 < 5) r2[i + 4] += carry;
    }
    uint64_t borrow = 0;
    for (int i = 0; i < 5; i++) { /* rr = (x mod 2^320) - r2 mod 2^320 */
        u128 t = (u128)x[i] - r2[i] - borrow;
        rr[i] = (uint64_t)t;
        borrow = (uint64_t)(t >> 127) & 1;
    }
    for (;;) { /* while rr >= l: rr -= l (at most twice) */
        int ge = 0;
        if (rr[4]) ge = 1;
        else {
            ge = 1;
            for (int i = 3; i >= 0; i--) {
                if (rr[i] != L64[i]) { ge = rr[i] > L64[i]; break; }
            }
        }
        if (!ge) break;
        borrow = 0;
        for (int i = 0; i < 5; i++) {
            u128 t = (u128)rr[i] - (i < 4 ? L64[i] : 0) - borrow;
            rr[i] = (uint64_t)t;
            borrow = (uint64_t)(t >> 127) & 1;
        }
    }
    for (int i = 0; i < 4; i++) r->v[i] = rr[i];
}
static void sc_from_bytes64(sc* r, const uint8_t b[64]) {
    uint64_t x[8];
    for (int i = 0; i < 8; i++) x[i] = ld64le(b + 8 * i);
    sc_reduce_words(r, x);
}
static void sc_from_bytes32_raw(sc* r, const uint8_t b[32]) {
    for (int i = 0; i < 4; i++) r->v[i] = ld64le(b + 8 * i);
}
static void sc_tobytes(uint8_t b[32], const sc* s) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[8 * i + j] = (uint8_t)(s->v[i] >> (8 * j));
}
void or_sc_reduce512(const uint8_t in[64], uint8_t out[32]) {
    sc r;
    sc_from_bytes64(&r, in);
    sc_tobytes(out, &r);
}
/* Scalar::from_canonical_bytes: the top bit must be clear and s < l */
int or_sc_is_canonical(const uint8_t s[32]) {
    if (s[31] >> 7) return 0;
    sc x;
    sc_from_bytes32_raw(&x, s);
    for (int i = 3; i >= 0; i--) {
        if (x.v[i] != L64[i]) return x.v[i] < L64[i];
    }
    return 0;
}
static void sc_mul(sc* r, const sc* a, const sc* b) {
    uint64_t x[8] = {0};
    for (int i = 0; i < 4; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 4; j++) {
            u128 t = (u128)a->v[i] * b->v[j] + x[i + j] + carry;
            x[i + j] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        }
        x[i + 4] = carry;
    }
    sc_reduce_words(r, x);
}
static void sc_add(sc* r, const sc* a, const sc* b) {
    uint64_t x[8] = {0};
    uint64_t carry = 0;
    for (int i = 0; i < 4; i++) {
        u128 t = (u128)a->v[i] + b->v[i] + carry;
        x[i] = (uint64_t)t;
        carry = (uint64_t)(t >> 64);
    }
    x[4] = carry;
    sc_reduce_words(r, x);
}
static void sc_neg(sc* r, const sc* a) { /* l - a (a canonical) */
    int zero = !(a->v[0] | a->v[1] | a->v[2] | a->v[3]);
    if (zero) { *r = *a; return; }
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        u128 t = (u128)L64[i] - a->v[i] - borrow;
        r->v[i] = (uint64_t)t;
        borrow = (uint64_t)(t >> 127) & 1;
    }
}

/* Signed-digit recodings.  NAF (width w) as dalek's Scalar::non_adjacent_form; radix 2^w
 * signed digits as Scalar::to_radix_2w (used by Pippenger). */
static void sc_naf(int8_t naf[256], const sc* s, int w) {
    uint64_t x[5] = {s->v[0], s->v[1], s->v[2], s->v[3], 0};
    memset(naf, 0, 256);
    const uint64_t width = 1ULL << w, window_mask = width - 1;
    size_t pos = 0;
    uint64_t carry = 0;
    while (pos < 256) {
        size_t u64_idx = pos / 64, bit_idx = pos % 64;
        uint64_t bit_buf;
        if (bit_idx < 64 - (size_t)w) bit_buf = x[u64_idx] >> bit_idx;
        else bit_buf = (x[u64_idx] >> bit_idx) | (x[1 + u64_idx] << (64 - bit_idx));
        uint64_t window = carry + (bit_buf & window_mask);
        if ((window & 1) == 0) { pos += 1; continue; }
        if (window < width / 2) { carry = 0; naf[pos] = (int8_t)window; }
        else { carry = 1; naf[pos] = (int8_t)((int64_t)window - (int64_t)width); }
        pos += (size_t)w;
    }
}
/* digits d_i in [-2^(w-1), 2^(w-1)), sum d_i 2^(w i) = s; returns digit count */
static int sc_radix2w(int16_t* digits, const sc* s, int w) {
    int n = (256 + w - 1) / w;
    uint64_t x[5] = {s->v[0], s->v[1], s->v[2], s->v[3], 0};
    const uint64_t radix = 1ULL << w, mask = radix - 1;
    int64_t carry = 0;
    for (int i = 0; i < n; i++) {
        size_t bit = (size_t)i * w, idx = bit / 64, off = bit % 64;
        uint64_t buf;
        if (off + w <= 64 || idx + 1 >= 5) buf = x[idx] >> off;
        else buf = (x[idx] >> off) | (x[idx + 1] << (64 - off));
        int64_t coef = carry + (int64_t)(buf & mask);
        carry = (coef + (int64_t)(radix / 2)) >> w;
        digits[i] = (int16_t)(coef - (carry << w));
    }
    digits[n] = (int16_t)carry; /* final carry digit (scalars < 2^253 keep it tiny) */
    return n + 1;
}

/* ======================================================================== */
/* Basepoint tables                                                         */
/* ======================================================================== */
static ge_ext BASE;
static ge_aniels BASE_ODD[64]; /* (2i+1) B, affine Niels -- NAF width 8 table as in dalek */
static pthread_once_t base_once = PTHREAD_ONCE_INIT;

static void ext_to_aniels(ge_aniels* a, const ge_ext* p) {
    fe zi, x, y;
    fe_invert(&zi, &p->Z);
    fe_mul(&x, &p->X, &zi);
    fe_mul(&y, &p->Y, &zi);
    fe_add(&a->ypx, &y, &x);
    fe_sub(&a->ymx, &y, &x);
    fe_mul(&a->xy2d, &x, &y);
    fe_mul(&a->xy2d, &a->xy2d, &FE_D2);
}
static void base_init(void) {
    static const uint8_t Benc[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                     0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                     0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                     0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
    ge_decompress(&BASE, Benc);
    ge_ext B2, cur = BASE;
    ext_dbl(&B2, &BASE);
    for (int i = 0; i < 64; i++) {
        ext_to_aniels(&BASE_ODD[i], &cur);
        ext_add(&cur, &cur, &B2);
    }
}
static void ensure_base(void) { pthread_once(&base_once, base_init); }

/* EdwardsPoint::vartime_double_scalar_mul_basepoint: a*A + b*B (dalek's NAF-5 / NAF-8 Straus) */
static void double_scalar_mul_basepoint(ge_ext* out, const sc* a, const ge_ext* A, const sc* b) {
    ensure_base();
    int8_t an[256], bn[256];
    sc_naf(an, a, 5);
    sc_naf(bn, b, 8);
    int i = 255;
    while (i >= 0 && an[i] == 0 && bn[i] == 0) i--;
    ge_pniels tA[8];
    ge_ext A2, cur = *A;
    ext_dbl(&A2, A);
    for (int j = 0; j < 8; j++) {
        ext_to_pniels(&tA[j], &cur);
        ext_add(&cur, &cur, &A2);
    }
    ge_proj r;
    r.X = FE_ZERO; r.Y = FE_ONE; r.Z = FE_ONE;
    for (; i >= 0; i--) {
        ge_comp t;
        ge_ext e;
        proj_dbl(&t, &r);
        if (an[i] > 0) { comp_to_ext(&e, &t); ext_add_pniels(&t, &e, &tA[an[i] / 2]); }
        else if (an[i] < 0) { comp_to_ext(&e, &t); ext_sub_pniels(&t, &e, &tA[(-an[i]) / 2]); }
        if (bn[i] > 0) { comp_to_ext(&e, &t); ext_add_aniels(&t, &e, &BASE_ODD[bn[i] / 2]); }
        else if (bn[i] < 0) { comp_to_ext(&e, &t); ext_sub_aniels(&t, &e, &BASE_ODD[(-bn[i]) / 2]); }
        comp_to_proj(&r, &t);
    }
    out->X = r.X; out->Y = r.Y; out->Z = r.Z;
    fe_mul(&out->X, &r.X, &r.Z);
    fe_mul(&out->Y, &r.Y, &r.Z);
    fe_sq(&out->Z, &r.Z);
    fe_mul(&out->T, &r.X, &r.Y);
}
static void scalar_mul(ge_ext* out, const ge_ext* P, const sc* s) {
    sc zero = {{0, 0, 0, 0}};
    double_scalar_mul_basepoint(out, s, P, &zero);
}
static void basepoint_mul(ge_ext* out, const sc* s) {
    ensure_base();
    sc zero = {{0, 0, 0, 0}};
    double_scalar_mul_basepoint(out, &zero, &BASE, s);
}

/* ======================================================================== */
/* Verification -- ed25519_consensus 2.0.1          */
/* call sites: types/src/primary.rs:179-182 (Header), :325-327 (Vote)        */
/* ======================================================================== */
static void challenge(sc* k, const uint8_t R[32], const uint8_t A[32], const uint8_t* m, size_t n) {
    sha512_ctx c;
    uint8_t h[64];
    sha512_init(&c);
    sha512_update(&c, R, 32);
    sha512_update(&c, A, 32);
    sha512_update(&c, m, n);
    sha512_final(&c, h);
    sc_from_bytes64(k, h);
}
int or_ed25519_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len) {
    ge_ext A, R, minusA, Rp, diff, d8;
    if (!ge_decompress(&A, pk)) return 0;           /* VerificationKey::try_from */
    if (!or_sc_is_canonical(sig + 32)) return 0;    /* Scalar::from_canonical_bytes */
    if (!ge_decompress(&R, sig)) return 0;          /* decompress R */
    sc k, s;
    challenge(&k, sig, pk, msg, len);               /* k = H(R_bytes || A_bytes || M) */
    sc_from_bytes32_raw(&s, sig + 32);
    ext_neg(&minusA, &A);
    double_scalar_mul_basepoint(&Rp, &k, &minusA, &s); /* R' = [s]B - [k]A */
    ext_neg(&Rp, &Rp);
    ext_add(&diff, &R, &Rp);                       /* R - R' */
    ext_mul_by_cofactor(&d8, &diff);
    return ext_is_identity(&d8);
}

/* ---- multiscalar multiplication: Straus (< 190 points) / Pippenger (>= 190) ---- */
static void msm_straus(ge_ext* out, size_t n, const sc* s, const ge_ext* P) {
    int8_t(*naf)[256] = malloc(n * sizeof *naf);
    ge_pniels(*tab)[8] = malloc(n * sizeof *tab);
    for (size_t j = 0; j < n; j++) {
        sc_naf(naf[j], &s[j], 5);
        ge_ext P2, cur = P[j];
        ext_dbl(&P2, &P[j]);
        for (int t = 0; t < 8; t++) {
            ext_to_pniels(&tab[j][t], &cur);
            ext_add(&cur, &cur, &P2);
        }
    }
    ge_ext r;
    ge_identity(&r);
    for (int i = 255; i >= 0; i--) {
        ext_dbl(&r, &r);
        for (size_t j = 0; j < n; j++) {
            int8_t d = naf[j][i];
            ge_comp t;
            if (d > 0) { ext_add_pniels(&t, &r, &tab[j][d / 2]); comp_to_ext(&r, &t); }
            else if (d < 0) { ext_sub_pniels(&t, &r, &tab[j][(-d) / 2]); comp_to_ext(&r, &t); }
        }
    }
    *out = r;
    free(naf);
    free(tab);
}
static void msm_pippenger(ge_ext* out, size_t n, const sc* s, const ge_ext* P) {
    int w = n < 500 ? 6 : (n < 800 ? 7 : 8);
    int nb = 1 << (w - 1);
    int nd = (256 + w - 1) / w + 1;
    int16_t* dig = malloc(n * (size_t)nd * sizeof(int16_t));
    ge_pniels* pn = malloc(n * sizeof *pn);
    for (size_t j = 0; j < n; j++) {
        sc_radix2w(dig + j * nd, &s[j], w);
        ext_to_pniels(&pn[j], &P[j]);
    }
    ge_ext* buckets = malloc((size_t)nb * sizeof *buckets);
    ge_ext acc;
    ge_identity(&acc);
    for (int dgt = nd - 1; dgt >= 0; dgt--) {
        for (int k = 0; k < w; k++) ext_dbl(&acc, &acc);
        for (int b = 0; b < nb; b++) ge_identity(&buckets[b]);
        for (size_t j = 0; j < n; j++) {
            int d = dig[j * nd + dgt];
            ge_comp t;
            if (d > 0) { ext_add_pniels(&t, &buckets[d - 1], &pn[j]); comp_to_ext(&buckets[d - 1], &t); }
            else if (d < 0) { ext_sub_pniels(&t, &buckets[-d - 1], &pn[j]); comp_to_ext(&buckets[-d - 1], &t); }
        }
        ge_ext run = buckets[nb - 1], sum = buckets[nb - 1];
        for (int b = nb - 2; b >= 0; b--) {
            ext_add(&run, &run, &buckets[b]);
            ext_add(&sum, &sum, &run);
        }
        ext_add(&acc, &acc, &sum);
    }
    *out = acc;
    free(dig);
    free(pn);
    free(buckets);
}
static void msm(ge_ext* out, size_t n, const sc* s, const ge_ext* P) {
    if (n < 190) msm_straus(out, n, s, P);
    else msm_pippenger(out, n, s, P);
}

/* batch::Verifier::verify.  Items are grouped by raw vk bytes (the reference's HashMap key);
 * grouping only merges the A-coefficients, the equation is the same. */
typedef struct { const uint8_t* pk; size_t idx; } vk_ref;
static int cmp_vk(const void* a, const void* b) {
    const vk_ref* x = a;
    const vk_ref* y = b;
    int c = memcmp(x->pk, y->pk, 32);
    if (c) return c;
    return (x->idx > y->idx) - (x->idx < y->idx);
}
int or_ed25519_verify_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_base,
                            const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t seed[32]) {
    if (n == 0) return 1; /* an empty ed25519_consensus batch verifies (wrappers reject earlier) */
    ensure_base();
    vk_ref* order = malloc(n * sizeof *order);
    for (size_t i = 0; i < n; i++) { order[i].pk = pk + 32 * i; order[i].idx = i; }
    qsort(order, n, sizeof *order, cmp_vk);
    size_t npts = 1 + 2 * n;
    sc* coef = malloc(npts * sizeof *coef);
    ge_ext* pts = malloc(npts * sizeof *pts);
    uint8_t* zbytes = malloc(((n * 16 + 63) / 64) * 64);
    or_chacha20_stream(seed, 0, zbytes, (n * 16 + 63) / 64);
    sc Bc = {{0, 0, 0, 0}};
    size_t m = 0, np = 1;
    int ok = 1;
    for (size_t g = 0; g < n && ok;) {
        size_t h = g;
        while (h < n && memcmp(order[h].pk, order[g].pk, 32) == 0) h++;
        ge_ext A;
        if (!ge_decompress(&A, order[g].pk)) { ok = 0; break; } /* MalformedPublicKey */
        sc Ac = {{0, 0, 0, 0}};
        for (size_t t = g; t < h; t++) {
            size_t i = order[t].idx;
            const uint8_t* sg = sig + 64 * i;
            ge_ext R;
            if (!ge_decompress(&R, sg)) { ok = 0; break; }
            if (!or_sc_is_canonical(sg + 32)) { ok = 0; break; }
            sc s, k, z, zs, zk;
            sc_from_bytes32_raw(&s, sg + 32);
            challenge(&k, sg, pk + 32 * i, msg_base + msg_off[i], msg_len[i]);
            z.v[0] = ld64le(zbytes + 16 * i);
            z.v[1] = ld64le(zbytes + 16 * i + 8);
            z.v[2] = z.v[3] = 0;
            sc_mul(&zs, &z, &s);
            sc_neg(&zs, &zs);
            sc_add(&Bc, &Bc, &zs);   /* B_coeff -= z*s */
            sc_mul(&zk, &z, &k);
            sc_add(&Ac, &Ac, &zk);   /* A_coeff += z*k */
            coef[np] = z;
            pts[np] = R;
            np++;
        }
        if (!ok) break;
        coef[np] = Ac;
        pts[np] = A;
        np++;
        m++;
        g = h;
    }
    int result = 0;
    if (ok) {
        coef[0] = Bc;
        pts[0] = BASE;
        ge_ext chk, c8;
        msm(&chk, np, coef, pts);
        ext_mul_by_cofactor(&c8, &chk);
        result = ext_is_identity(&c8);
    }
    (void)m;
    free(order);
    free(coef);
    free(pts);
    free(zbytes);
    return result;
}

/* ---- multi-threaded CPU baseline helpers ---- */
typedef struct {
    size_t lo, hi;
    const uint8_t *pk, *sig, *msg_base;
    const uint64_t* msg_off;
    const uint32_t* msg_len;
    uint64_t* bits;
    const uint8_t* seed;
    int result;
} mt_job;
static void* mt_each(void* arg) {
    mt_job* j = arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        int v = or_ed25519_verify(j->pk + 32 * i, j->sig + 64 * i, j->msg_base + j->msg_off[i],
                                  j->msg_len[i]);
        if (v) __atomic_fetch_or(&j->bits[i / 64], 1ULL << (i % 64), __ATOMIC_RELAXED);
    }
    return NULL;
}
static void* mt_batch(void* arg) {
    mt_job* j = arg;
    uint8_t sd[32];
    memcpy(sd, j->seed, 32);
    sd[0] ^= (uint8_t)j->lo; sd[1] ^= (uint8_t)(j->lo >> 8); sd[2] ^= (uint8_t)(j->lo >> 16);
    sd[3] ^= (uint8_t)(j->lo >> 24);
    size_t n = j->hi - j->lo;
    /* shard-relative offsets are kept absolute: pass shifted base pointers */
    j->result = or_ed25519_verify_batch(n, j->pk + 32 * j->lo, j->sig + 64 * j->lo, j->msg_base,
                                        j->msg_off + j->lo, j->msg_len + j->lo, sd);
    return NULL;
}
static void run_mt(size_t n, int threads, mt_job* proto, void* (*fn)(void*), int* all) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = n ? (int)n : 1;
    pthread_t* th = malloc(threads * sizeof *th);
    mt_job* jobs = malloc(threads * sizeof *jobs);
    for (int t = 0; t < threads; t++) {
        jobs[t] = *proto;
        jobs[t].lo = n * t / threads;
        jobs[t].hi = n * (t + 1) / threads;
        pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    int r = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        r &= jobs[t].result;
    }
    if (all) *all = r;
    free(th);
    free(jobs);
}
void or_ed25519_verify_each_mt(size_t n, const uint8_t* pk, const uint8_t* sig,
                               const uint8_t* msg_base, const uint64_t* msg_off,
                               const uint32_t* msg_len, uint64_t* verdict_bits, int threads) {
    ensure_base();
    memset(verdict_bits, 0, ((n + 63) / 64) * 8);
    mt_job p = {0, 0, pk, sig, msg_base, msg_off, msg_len, verdict_bits, NULL, 1};
    run_mt(n, threads, &p, mt_each, NULL);
}
int or_ed25519_verify_batch_mt(size_t n, const uint8_t* pk, const uint8_t* sig,
                               const uint8_t* msg_base, const uint64_t* msg_off,
                               const uint32_t* msg_len, const uint8_t seed[32], int threads) {
    ensure_base();
    int all = 1;
    mt_job p = {0, 0, pk, sig, msg_base, msg_off, msg_len, NULL, seed, 1};
    run_mt(n, threads, &p, mt_batch, &all);
    return all;
}

/* ======================================================================== */
/* RFC 8032 key generation and signing (fixture generation only)           */
/* ======================================================================== */
static void expand_seed(const uint8_t seed[32], sc* a, uint8_t prefix[32]) {
    uint8_t h[64];
    or_sha512(seed, 32, h);
    h[0] &= 248;
    h[31] &= 127;
    h[31] |= 64;
    sc_from_bytes32_raw(a, h); /* clamped scalar, < 2^255, used as an integer */
    memcpy(prefix, h + 32, 32);
}
static void mul_base_integer(ge_ext* out, const sc* a) {
    /* a may exceed l (clamped), reduce first: [a]B == [a mod l]B since B has order l */
    uint64_t x[8] = {a->v[0], a->v[1], a->v[2], a->v[3], 0, 0, 0, 0};
    sc r;
    sc_reduce_words(&r, x);
    basepoint_mul(out, &r);
}
void or_ed25519_pubkey(const uint8_t seed[32], uint8_t pk[32]) {
    sc a;
    uint8_t prefix[32];
    expand_seed(seed, &a, prefix);
    ge_ext A;
    mul_base_integer(&A, &a);
    ext_compress(pk, &A);
}
void or_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t len, uint8_t sig[64]) {
    sc a, r, k, S;
    uint8_t prefix[32], pk[32], h[64];
    expand_seed(seed, &a, prefix);
    ge_ext A, R;
    mul_base_integer(&A, &a);
    ext_compress(pk, &A);
    sha512_ctx c;
    sha512_init(&c);
    sha512_update(&c, prefix, 32);
    sha512_update(&c, msg, len);
    sha512_final(&c, h);
    sc_from_bytes64(&r, h);
    basepoint_mul(&R, &r);
    ext_compress(sig, &R);
    challenge(&k, sig, pk, msg, len);
    uint64_t x[8] = {a.v[0], a.v[1], a.v[2], a.v[3], 0, 0, 0, 0};
    sc ar;
    sc_reduce_words(&ar, x);
    sc_mul(&S, &k, &ar);
    sc_add(&S, &S, &r);
    sc_tobytes(sig + 32, &S);
}

int or_point_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    ge_ext A, B, C;
    if (!ge_decompress(&A, a) || !ge_decompress(&B, b)) return 0;
    ext_add(&C, &A, &B);
    ext_compress(out, &C);
    return 1;
}
int or_point_scalarmul(const uint8_t a[32], const uint8_t s[32], uint8_t out[32]) {
    ge_ext A, C;
    if (!ge_decompress(&A, a)) return 0;
    sc x;
    uint64_t w[8] = {0};
    for (int i = 0; i < 4; i++) w[i] = ld64le(s + 8 * i);
    /* integer multiple (not reduced): split as q*l + r would change torsion parts, so do
     * plain double-and-add over all 256 bits */
    ge_ext acc;
    ge_identity(&acc);
    for (int i = 255; i >= 0; i--) {
        ext_dbl(&acc, &acc);
        if ((w[i / 64] >> (i % 64)) & 1) ext_add(&acc, &acc, &A);
    }
    (void)x;
    (void)scalar_mul;
    C = acc;
    ext_compress(out, &C);
    return 1;
}
void or_basepoint_mul(const uint8_t s[32], uint8_t out[32]) {
    sc x;
    uint64_t w[8] = {0};
    for (int i = 0; i < 4; i++) w[i] = ld64le(s + 8 * i);
    sc_reduce_words(&x, w);
    ge_ext P;
    basepoint_mul(&P, &x);
    ext_compress(out, &P);
}
