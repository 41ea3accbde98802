/*
 * bls_oracle.h -- TEST INFRASTRUCTURE ONLY: plain-C restatement of the BLS12-381 signature path the
 * reference uses by default.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the engine (narwhal_amd/) never does.
 *
 * Reference boundary: crypto/src/lib.rs:29-33 aliases PublicKey / Signature / AggregateSignature
 * to fastcrypto 0.1.2 bls12381::* (Cargo.lock:1534-1561), backed by blst 0.3.10 (Cargo.lock:609-617,
 * not vendored) in its min_sig flavour: public keys in G2 (96-byte compressed), signatures in G1
 * (48-byte compressed), hash to G1 with RFC 9380 BLS12381G1_XMD:SHA-256_SSWU_RO_ under the DST
 * "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_".  The call sites are the same as the Ed25519
 * path's: Header::verify types/src/primary.rs:179-182 (Verifier::verify), Vote::verify :325-327,
 * Certificate::verify :531-534 (AggregateAuthenticator::verify), Certificate::new_unsafe :476-477
 * (aggregate), and the trait contract crypto/src/bls12377/mod.rs:264-291, :485-577.
 *
 * Parity pins (tests/golden/bls12381_kats.json, oracle/gen_bls_golden.py): the reference's own
 * BLS12381KeyPair fixtures (Docker/validators/validator-{0..3}/primary-key.json: secret -> public
 * key) and the RFC 9380 Appendix J.9.1 hash_to_curve known answers.  The pairing is pinned by
 * algebra (bilinearity, non-degeneracy, order r, the fast twisted Miller loop + x-chain final
 * exponentiation equal to a plain affine Miller loop on the untwisted curve with the final
 * exponent computed by square-and-multiply).  Verdict semantics restated from blst 0.3.10 /
 * draft-irtf-cfrg-bls-signature (see bls_oracle.c header); edge-case verdicts beyond the pins
 * (non-subgroup / infinite inputs) are "parity unpinned": no reference fixture holds them.
 */
#ifndef BLS_ORACLE_H
#define BLS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* verdict / error codes (blst BLST_ERROR subset) */
#define ORB_OK 0
#define ORB_BAD_ENCODING 1
#define ORB_NOT_ON_CURVE 2
#define ORB_NOT_IN_GROUP 3
#define ORB_AGGR_MISMATCH 4
#define ORB_VERIFY_FAIL 5
#define ORB_PK_INFINITY 6

void orb_sha256(const uint8_t* m, size_t n, uint8_t out[32]);
void orb_expand_message_xmd(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len, uint8_t* out,
                            size_t out_len);
/* hash_to_curve G1 (RFC 9380): out = uncompressed affine (x || y, 96 bytes big-endian) */
void orb_hash_to_g1(const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len, uint8_t out[96]);

/* key generation / signing (secret: 32 bytes big-endian, < r) */
int orb_keygen(const uint8_t sk[32], uint8_t pk[96]);
int orb_sign(const uint8_t sk[32], const uint8_t* msg, size_t n, const uint8_t* dst, size_t dst_len,
             uint8_t sig[48]);

/* decoding (ZCash compressed format) */
int orb_g1_decompress(const uint8_t in[48], uint8_t out_xy[96], int* infinity);
int orb_g2_decompress(const uint8_t in[96], uint8_t out_xy[192], int* infinity);
int orb_g1_in_group(const uint8_t in[48]);
int orb_g2_in_group(const uint8_t in[96]);
int orb_pubkey_validate(const uint8_t pk[96]); /* decode, not infinity, in G2 */

/* fastcrypto trait surface (min_sig); return ORB_OK or an error code */
int orb_verify(const uint8_t pk[96], const uint8_t* msg, size_t n, const uint8_t sig[48], const uint8_t* dst,
               size_t dst_len);
int orb_aggregate(size_t n, const uint8_t* sigs48, uint8_t out[48]);
int orb_aggregate_pubkeys(size_t n, const uint8_t* pks96, uint8_t out[96]);
int orb_fast_aggregate_verify(const uint8_t sig[48], size_t n_pks, const uint8_t* pks96, const uint8_t* msg,
                              size_t n, const uint8_t* dst, size_t dst_len);
/* one item per certificate, items split over `threads` host threads; verdict[i] = 1 iff valid */
void orb_fast_aggregate_verify_mt(size_t n_items, const uint8_t* sigs48, const uint32_t* pk_off,
                                  const uint32_t* pk_cnt, const uint8_t* pks96, const uint8_t* msg_base,
                                  const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* dst,
                                  size_t dst_len, uint8_t* verdict, int threads);

/* orb_fast_aggregate_verify's status for every item, the key table decoded and validated once (as
 * fastcrypto deserializes each public key once): item i = (sigs48[i], keys96[pk_idx[pk_off[i] + j]]
 * for j < pk_cnt[i], message i); items split over `threads` host threads */
void orb_verify_items_keytab_mt(size_t n_keys, const uint8_t* keys96, size_t n_items, const uint8_t* sigs48,
                                const uint32_t* pk_off, const uint32_t* pk_cnt, const uint32_t* pk_idx,
                                const uint8_t* msg_base, const uint64_t* msg_off, const uint32_t* msg_len,
                                const uint8_t* dst, size_t dst_len, int32_t* status, int threads);

/* pairing on uncompressed affine inputs (P: 96 bytes in G1, Q: 192 bytes in G2); out = 12 Fp
 * coefficients (576 bytes big-endian) in the tower order c0.c0.c0, c0.c0.c1, c0.c1.c0, ... */
void orb_pairing(const uint8_t P[96], const uint8_t Q[192], uint8_t out[576]);      /* fast: f^(3(p^12-1)/r) */
void orb_pairing_ref(const uint8_t P[96], const uint8_t Q[192], uint8_t out[576]);  /* slow: f^((p^12-1)/r) */
void orb_gt_pow(const uint8_t in[576], const uint8_t* e, size_t e_len, uint8_t out[576]); /* e big-endian */
void orb_gt_mul(const uint8_t a[576], const uint8_t b[576], uint8_t out[576]);
/* point arithmetic on uncompressed affine encodings (all-zero = infinity) */
void orb_g1_mul(const uint8_t P[96], const uint8_t* k, size_t k_len, uint8_t out[96]);
void orb_g2_mul(const uint8_t Q[192], const uint8_t* k, size_t k_len, uint8_t out[192]);
void orb_g1_add(const uint8_t A[96], const uint8_t B[96], uint8_t out[96]);
void orb_g2_add(const uint8_t A[192], const uint8_t B[192], uint8_t out[192]);
void orb_g1_compress(const uint8_t P[96], uint8_t out[48]);
void orb_g2_compress(const uint8_t Q[192], uint8_t out[96]);
void orb_g1_generator(uint8_t out[96]);
void orb_g2_generator(uint8_t out[192]);
/* the hard-part exponent (p^4 - p^2 + 1) / r the reference final exponentiation uses (160 bytes BE) */
void orb_hard_exponent(uint8_t out[160]);

#ifdef __cplusplus
}
#endif
#endif
