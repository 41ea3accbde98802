/*
 * nwv_bls.h -- BLS12-381 (min_sig) verification on MI355X: SURVEY.md §8 row f4, the reference's
 * default signature scheme.
 *
 * Reference boundary replaced: crypto/src/lib.rs:29-33 aliases PublicKey / Signature /
 * AggregateSignature / PrivateKey / KeyPair to fastcrypto 0.1.2 bls12381::* (Cargo.lock:1534-1561),
 * backed by blst 0.3.10 (Cargo.lock:609-617) in its min_sig flavour: 96-byte compressed G2 public
 * keys, 48-byte compressed G1 signatures, hash to G1 by RFC 9380 under fastcrypto's DST
 * "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_" (NWV_BLS_DST).  The trait contract mirrored is the
 * in-tree template crypto/src/bls12377/mod.rs:264-291 (VerifyingKey) and :485-577
 * (AggregateAuthenticator); the call sites are Header::verify types/src/primary.rs:179-182,
 * Vote::verify :325-327, Certificate::verify :531-534, Certificate::new_unsafe :476-477 and
 * CertificatesResponse::validate_certificates primary/src/block_synchronizer/responses.rs:95-141.
 *
 * Every verification runs on the GPU: signature decode + G1 membership, public-key decode + G2
 * membership (once per device for the keys registered in the key cache below, as fastcrypto
 * validates keys once at deserialization; any other key is decoded by the call that names it),
 * aggregate public key, hash to G1 and the pairing equation e(-sig, g2) e(H(msg), apk) = 1.  By
 * default each item's hash, G1 check and pairing check run on one 64-lane wave each
 * (bls_wave.h: the Miller loop and final exponentiation as lane-parallel stage programs);
 * NWV_FLAG_BLS_BATCH checks all items' equations as one random linear combination instead (one
 * Miller loop per item, one final exponentiation per call; per item only after a rejection).
 * Per-item status codes are exact either way.
 * Buffers are the caller's; the library never retains them.  Thread-safe: concurrent calls on one
 * device run side by side (each takes one of up to eight per-device stream sets).
 */
#ifndef NWV_BLS_H
#define NWV_BLS_H

#include <stddef.h>
#include <stdint.h>

#include "nwv.h"

#ifdef __cplusplus
extern "C" {
#endif

#define NWV_BLS_DST "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"

/* per-item status (the BLST_ERROR subset blst returns on these paths) */
#define NWV_BLS_OK 0
#define NWV_BLS_BAD_ENCODING 1   /* flags / coordinate >= p / stray bits after the infinity flag */
#define NWV_BLS_NOT_ON_CURVE 2   /* x has no y on the curve */
#define NWV_BLS_NOT_IN_GROUP 3   /* signature outside G1 / public key outside G2 */
#define NWV_BLS_AGGR_MISMATCH 4  /* empty key list (or empty aggregation) */
#define NWV_BLS_VERIFY_FAIL 5    /* the pairing equation does not hold */
#define NWV_BLS_PK_INFINITY 6    /* identity public key (or a key sum that is the identity) */

/* The batch entry point (validate_certificates, a DAG round's certificates, the bench): item i is
 * AggregateAuthenticator::verify of the aggregate signature sigs[i] (48 bytes) over the message
 * msg_base[msg_off[i] .. + msg_len[i]) by the keys keys[pk_idx[pk_off[i] + j]], j < pk_cnt[i]
 * (keys: n_keys x 96 bytes, e.g. the committee; a key the device's key cache does not hold is
 * decoded and subgroup-checked once by the call).  status[i] = NWV_BLS_* for item i.  dst = NULL selects NWV_BLS_DST.
 * Returns NWV_OK (statuses valid) or a negative error. */
int nwv_bls_verify_many(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys, size_t n, const uint8_t* sigs,
                        const uint32_t* pk_off, const uint32_t* pk_cnt, const uint32_t* pk_idx,
                        const uint8_t* msg_base, const uint64_t* msg_off, const uint32_t* msg_len,
                        const uint8_t* dst, size_t dst_len, int32_t* status);

/* device time of the last nwv_bls_verify_many call on this context, per stage (HIP events; the
 * first four run on three concurrent streams): [0] keys new to the device's key cache, [1]
 * signature decode + G1 checks, [2] hash to G1, [3] key sums, [4] the pairing check (the batch
 * check k_bls_rlc + k_bls_fold + k_bls_final, plus k_bls_pair when it ran).  Calls of at most
 * 1,024 items record these only on a context opened with NWV_FLAG_BLS_STAGE_TIMES (else zeros). */
int nwv_bls_last_kernel_ms(nwv_ctx* ctx, double out_ms[5]);
/* how the last nwv_bls_verify_many call checked its pairings: 0 per item on the 8-lane group
 * kernels (NWV_FLAG_BLS_PER_ITEM), 1 one batch check that accepted every item and 2 a batch check
 * that rejected, then per item (NWV_FLAG_BLS_BATCH), 3 every item on its own wave (the default) */
int nwv_bls_last_path(nwv_ctx* ctx);
/* keys of the last nwv_bls_verify_many call: out[0] key-list entries found in the key cache,
 * out[1] distinct keys the call decoded itself */
int nwv_bls_last_keys(nwv_ctx* ctx, uint64_t out[2]);

/* The committee key cache (per device).  fastcrypto decodes and validates a public key once, at
 * deserialization; nwv_bls_keycache_register does that once per device for the committee's keys
 * (epoch start, Core::change_epoch primary/src/core.rs:592-611) and keeps the records of the keys
 * that are valid.  Verification calls only look keys up: a key the cache does not hold is decoded
 * by the call itself and never takes a slot (an invalid or stray key cannot fill the cache).
 * nwv_bls_keycache_reset (epoch change) drops every slot once the calls in flight finish.  A
 * device keeps at most 65,536 keys; NWV_FLAG_NO_KEYCACHE contexts keep none. */
int nwv_bls_keycache_register(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys);
int nwv_bls_keycache_reset(nwv_ctx* ctx);
/* number of keys the cache holds (>= 0), or a negative error */
int nwv_bls_keycache_size(nwv_ctx* ctx);

/* ---- fastcrypto 0.1.2 trait surface (bls12381 module) ---- */
/* Verifier::verify(&self = pk, msg, sig): NWV_OK or NWV_ERR_SIGNATURE */
int nwv_bls_verify(nwv_ctx* ctx, const uint8_t pk[96], const uint8_t* msg, size_t msg_len, const uint8_t sig[48]);
/* AggregateAuthenticator::verify(&self, pks, msg); sig NULL = an aggregate holding no signature
 * (sig: None) -> NWV_ERR_SIGNATURE */
int nwv_bls_aggregate_verify(nwv_ctx* ctx, const uint8_t* sig48_or_null, const uint8_t* pks, size_t n_pks,
                             const uint8_t* msg, size_t msg_len);
/* VerifyingKey::verify_batch_empty_fail(msg, pks, sigs): NWV_ERR_EMPTY, NWV_ERR_LENGTH, then the
 * signatures are aggregated (each must decode and lie in G1) and verified against the key sum */
int nwv_bls_verify_batch_empty_fail(nwv_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* pks,
                                    size_t n_pks, const uint8_t* sigs, size_t n_sigs);
/* AggregateAuthenticator::batch_verify(sigs, pks_per_sig, msgs): NWV_ERR_LENGTH on any count
 * mismatch, else NWV_OK iff every aggregate verifies over its message and keys */
int nwv_bls_aggregate_batch_verify(nwv_ctx* ctx, size_t n_aggs, const uint8_t* const* sigs48,
                                   const uint8_t* const* pks, const size_t* n_pks, const uint8_t* const* msgs,
                                   const size_t* msg_lens, size_t n_msgs);
/* AggregateAuthenticator::aggregate(sigs): out48 = the sum; NWV_ERR_SIGNATURE if n == 0 or any
 * signature fails to decode / lies outside G1 (*status_or_null = its NWV_BLS_* code) */
int nwv_bls_aggregate(nwv_ctx* ctx, size_t n, const uint8_t* sigs48, uint8_t out48[48], int32_t* status_or_null);

/* ---- key generation, signing and the primitives (synthetic workloads, tests) ---- */
/* pk = sk * g2 compressed (sk: 32 bytes big-endian, < r): the BLS12381KeyPair derivation */
int nwv_bls_keygen_many(nwv_ctx* ctx, size_t n, const uint8_t* sks, uint8_t* pks);
/* sig = sk * H(msg), compressed */
int nwv_bls_sign_many(nwv_ctx* ctx, size_t n, const uint8_t* sks, const uint8_t* msg_base, const uint64_t* msg_off,
                      const uint32_t* msg_len, const uint8_t* dst, size_t dst_len, uint8_t* sigs);
/* H(msg) = hash_to_curve G1 (RFC 9380), uncompressed affine (x || y, 96 bytes big-endian) */
int nwv_bls_hash_to_g1_many(nwv_ctx* ctx, size_t n, const uint8_t* msg_base, const uint64_t* msg_off,
                            const uint32_t* msg_len, const uint8_t* dst, size_t dst_len, uint8_t* out96);
/* e(P_i, Q_i) (P: 96-byte uncompressed G1, Q: 192-byte uncompressed G2 x.c1||x.c0||y.c1||y.c0,
 * all-zero = identity) as 12 big-endian Fp in tower order (576 bytes), = the optimal ate pairing
 * raised to 3 (the final exponentiation's x-chain computes f^(3(p^12-1)/r)) */
int nwv_bls_pairing_many(nwv_ctx* ctx, size_t n, const uint8_t* P96, const uint8_t* Q192, uint8_t* out576);

#ifdef __cplusplus
}
#endif
#endif
