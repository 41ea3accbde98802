/*
 * nwv_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot-path arithmetic, used as the parity
 * checker by tests/, by __graft_entry__.smoke() and as the `cpu_baseline` leg of
 * bench.py.  Nothing in the product (narwhal_amd/, include/nwv.h) links or calls it.
 *
 * The reference (erwanor/narwhal @ 2025-02-15) does not contain this arithmetic:
 * it lives in third-party crates that are NOT vendored in /root/reference
 * (SURVEY.md §0.2).  Pinned versions, from /root/reference/Cargo.lock:
 *   fastcrypto 0.1.2            Cargo.lock:1534-1561  (trait wrappers, blake2b_256)
 *   ed25519-consensus 2.0.1     Cargo.lock:1428-1440  (ZIP-215 verify + batch::Verifier)
 *   curve25519-dalek-ng 4.1.1   Cargo.lock:1166-1177  (u64_backend, workspace-hack/Cargo.toml:91)
 *   sha2 0.9.9                  Cargo.lock:3845
 *   blake2 0.9.2                Cargo.lock:536        (VarBlake2b, types/src/primary.rs:9,213)
 * Their published algorithms are restated here:
 *   - field arithmetic mod p = 2^255-19 in radix 2^51 (dalek u64_backend),
 *   - CompressedEdwardsY::decompress with sqrt_ratio_i (y >= p accepted, "negative zero" accepted),
 *   - Scalar::from_canonical_bytes (s < l) and Scalar::from_hash (SHA-512 mod l),
 *   - VerificationKey::verify: accept iff [8](R - ([s]B - [k]A)) == identity (cofactored),
 *   - batch::Verifier::verify: random 128-bit z_i, one MSM (Straus < 190 points,
 *     Pippenger >= 190), multiplied by the cofactor, identity check,
 *   - RFC 8032 key generation / signing (test-vector generation only),
 *   - BLAKE2b with digest_length = 32 (RFC 7693), and the bincode batch walk of
 *     types/src/worker.rs:44-80.
 * Pinning: tests/test_oracle_golden.py checks every function here against
 * the tests/golden JSON fixtures, which oracle/gen_golden.py produced and cross-checked against
 * libsodium 1.0.18, OpenSSL 1.1.1 (node) and Python hashlib.
 */
#ifndef NWV_ORACLE_H
#define NWV_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void or_sha512(const uint8_t* m, size_t n, uint8_t out[64]);
void or_blake2b256(const uint8_t* m, size_t n, uint8_t out[32]);
/* types/src/worker.rs:44-80 -- returns 0 ok, -1 error (err_offset set) */
int or_batch_digest_serialized(const uint8_t* buf, size_t n, uint8_t out[32], int64_t* err_offset);
/* types/src/primary.rs:65-73 -- blake2b-256 of the concatenated transactions */
void or_batch_digest(size_t ntx, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                     uint8_t out[32]);

void or_sc_reduce512(const uint8_t in[64], uint8_t out[32]);
int or_sc_is_canonical(const uint8_t s[32]);
/* 1 if the 32 bytes decode to a curve point under dalek's decompress rules */
int or_point_decompress_ok(const uint8_t p[32]);

/* ZIP-215 single verification (ed25519_consensus::VerificationKey::verify): 1 accept / 0 reject */
int or_ed25519_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len);
/* ed25519_consensus::batch::Verifier over n items; z drawn from ChaCha20(seed). 1 ok / 0 err */
int or_ed25519_verify_batch(size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg_base,
                            const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t seed[32]);
/* multi-threaded helpers (CPU baseline): per-signature verdict bits, and batch over
 * `threads` contiguous shards (each shard its own random linear combination). */
void or_ed25519_verify_each_mt(size_t n, const uint8_t* pk, const uint8_t* sig,
                               const uint8_t* msg_base, const uint64_t* msg_off,
                               const uint32_t* msg_len, uint64_t* verdict_bits, int threads);
int or_ed25519_verify_batch_mt(size_t n, const uint8_t* pk, const uint8_t* sig,
                               const uint8_t* msg_base, const uint64_t* msg_off,
                               const uint32_t* msg_len, const uint8_t seed[32], int threads);

/* RFC 8032 */
void or_ed25519_pubkey(const uint8_t seed[32], uint8_t pk[32]);
void or_ed25519_sign(const uint8_t seed[32], const uint8_t* msg, size_t len, uint8_t sig[64]);

/* group helpers for fixture generation: out = compress(a + b), compress([8]a), returns 0 if a/b bad */
int or_point_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]);
int or_point_scalarmul(const uint8_t a[32], const uint8_t s[32], uint8_t out[32]);
void or_basepoint_mul(const uint8_t s[32], uint8_t out[32]);

void or_chacha20_stream(const uint8_t key[32], uint64_t counter0, uint8_t* out, size_t nblocks);

#ifdef __cplusplus
}
#endif
#endif
