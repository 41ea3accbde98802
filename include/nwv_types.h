/*
 * nwv_types.h -- C ABI of the Narwhal certificate / header / vote verification layer on top of
 * the MI355X engine (include/nwv.h).
 *
 * Mirrors the verification half of erwanor/narwhal's types crate (types/src/primary.rs): the
 * digests (Header::digest :209-227, Vote::digest :351-364, Certificate::digest :594-607),
 * Header::verify (:150-183), Vote::verify (:307-328), Certificate::new_unsafe (:427-485),
 * Certificate::verify (:487-537) and the batch validation of a block-synchronizer response
 * (CertificatesResponse::validate_certificates, primary/src/block_synchronizer/responses.rs:95-141).
 * Every digest is BLAKE2b-256 computed on the GPU (nwv_blake2b256_many) and every signature check
 * runs on the GPU; the *_many entry points batch all the digests of a call into one launch and all
 * the signatures into one batch MSM (per-signature fallback only when it rejects), which is the
 * batching service SURVEY.md §8 f1/f3 asks for in front of Core::sanitize_* and
 * validate_certificates.
 *
 * Data is passed as plain structs of pointers (the Rust side would fill them from its own types
 * without copying): keys 32 bytes, digests 32 bytes, signatures 64 bytes (R || s).  Results are
 * DagError codes (types/src/error.rs), 0 = Ok.
 */
#ifndef NWV_TYPES_H
#define NWV_TYPES_H

#include <stddef.h>
#include <stdint.h>

#include "nwv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* DagError variants returned by the verify calls (types/src/error.rs) */
#define NWV_DAG_OK 0
#define NWV_DAG_INVALID_EPOCH 10              /* DagError::InvalidEpoch                    */
#define NWV_DAG_INVALID_HEADER_ID 11          /* DagError::InvalidHeaderId                 */
#define NWV_DAG_UNKNOWN_AUTHORITY 12          /* DagError::UnknownAuthority                */
#define NWV_DAG_MALFORMED_HEADER 13           /* DagError::MalformedHeader (bad worker id) */
#define NWV_DAG_INVALID_SIGNATURE 14          /* DagError::InvalidSignature                */
#define NWV_DAG_CERTIFICATE_REQUIRES_QUORUM 15 /* DagError::CertificateRequiresQuorum      */
#define NWV_DAG_INVALID_BITMAP 16             /* DagError::InvalidBitmap                   */

/* Committee (config/src/lib.rs:488-550) + the worker cache's worker ids per authority
 * (config/src/lib.rs:410-423).  keys: n x 32 bytes in ascending byte order (BTreeMap order,
 * which is also the bitmap index order); stakes[n]; worker_ids[i] lists n_workers[i] ids of
 * authority i (may be NULL when n_workers[i] == 0). */
typedef struct {
    size_t n;
    const uint8_t* keys;
    const uint64_t* stakes;
    uint64_t epoch;
    const uint32_t* n_workers;
    const uint32_t* const* worker_ids;
} nwv_committee;

/* Header (types/src/primary.rs:75-86).  payload keeps IndexMap insertion order; parents is the
 * BTreeSet, i.e. ascending byte order. */
typedef struct {
    const uint8_t* author;        /* 32 */
    uint64_t round;
    uint64_t epoch;
    size_t n_payload;
    const uint8_t* payload_digests; /* n_payload x 32 (BatchDigest) */
    const uint32_t* payload_workers; /* n_payload (WorkerId) */
    size_t n_parents;
    const uint8_t* parents;       /* n_parents x 32 (CertificateDigest) */
    const uint8_t* id;            /* 32 (HeaderDigest) */
    const uint8_t* signature;     /* 64 */
} nwv_header;

/* Vote (types/src/primary.rs:251-259) */
typedef struct {
    const uint8_t* id;        /* 32: header digest */
    uint64_t round;
    uint64_t epoch;
    const uint8_t* origin;    /* 32 */
    const uint8_t* author;    /* 32 */
    const uint8_t* signature; /* 64 */
} nwv_vote;

/* Certificate (types/src/primary.rs:388-395).  The Ed25519 aggregated signature is the list of
 * the signers' signatures in committee order; signed_authorities are the roaring bitmap's
 * indices in ascending order. */
typedef struct {
    nwv_header header;
    size_t n_signed;
    const uint32_t* signed_authorities;
    size_t n_sigs;
    const uint8_t* aggregated_signature; /* n_sigs x 64 */
} nwv_certificate;

/* ---- digests (BLAKE2b-256 on the GPU) ---- */
int nwv_header_digest(nwv_ctx* ctx, const nwv_header* h, uint8_t out[32]);
int nwv_vote_digest(nwv_ctx* ctx, const nwv_vote* v, uint8_t out[32]);
int nwv_certificate_digest(nwv_ctx* ctx, const nwv_certificate* c, uint8_t out[32]);
/* n headers / votes / certificates in one launch: out n x 32 */
int nwv_header_digest_many(nwv_ctx* ctx, size_t n, const nwv_header* h, uint8_t* out);
int nwv_vote_digest_many(nwv_ctx* ctx, size_t n, const nwv_vote* v, uint8_t* out);
int nwv_certificate_digest_many(nwv_ctx* ctx, size_t n, const nwv_certificate* c, uint8_t* out);

/* ---- verification: return an NWV_DAG_* code (>= 0) or a negative nwv error ---- */
int nwv_header_verify(nwv_ctx* ctx, const nwv_committee* committee, const nwv_header* h);
int nwv_vote_verify(nwv_ctx* ctx, const nwv_committee* committee, const nwv_vote* v);
int nwv_certificate_verify(nwv_ctx* ctx, const nwv_committee* committee, const nwv_certificate* c);
/* Batched forms: results[i] = the code the single call would return for item i, in the
 * reference's check order.  All digests of the call go to the GPU in one launch and all the
 * signatures in one batch verification.  Return NWV_OK or a negative error. */
int nwv_header_verify_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n,
                           const nwv_header* h, int32_t* results);
int nwv_vote_verify_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n, const nwv_vote* v,
                         int32_t* results);
int nwv_certificate_verify_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n,
                                const nwv_certificate* c, int32_t* results);
/* Mixed batch: the headers, votes and certificates a primary's Core has queued
 * (Core::sanitize_header / sanitize_vote / sanitize_certificate, primary/src/core.rs:497-573)
 * verified by ONE call: every digest of all three kinds in one BLAKE2b launch and every signature
 * in one batch MSM.  Each results array receives exactly what the matching *_many call would
 * (and so what Header::verify :150-183, Vote::verify :307-328, Certificate::verify :487-537
 * return item by item).  Any count may be 0 (its pointers may then be NULL). */
int nwv_verify_mixed_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n_headers,
                          const nwv_header* headers, int32_t* header_results, size_t n_votes,
                          const nwv_vote* votes, int32_t* vote_results, size_t n_certs,
                          const nwv_certificate* certs, int32_t* cert_results);

/* CertificatesResponse::validate_certificates: the certificates present in a response (absent
 * entries are simply not passed) are all verified; *n_invalid receives the number of invalid
 * ones and invalid_idx (capacity n) their indices in input order.  Returns NWV_OK when every
 * certificate is valid, NWV_ERR_SIGNATURE when at least one is invalid (ValidationError), or a
 * negative error. */
int nwv_validate_certificates(nwv_ctx* ctx, const nwv_committee* committee, size_t n,
                              const nwv_certificate* c, size_t* n_invalid, size_t* invalid_idx);

/* ---- Certificate::new / new_unsigned (types/src/primary.rs:411-485) ----
 * votes: n_votes (pk 32, sig 64) pairs in any order; they are sorted by pk, repeated pairs are
 * dropped and the signers are matched against the committee.  check_stake = 1 for new(), 0 for
 * new_unsigned().  Outputs: signed_out (capacity committee->n) the bitmap indices, *n_signed;
 * sigs_out (capacity 64 x committee->n) the aggregated signature list, *n_sigs.
 * Returns NWV_DAG_OK, NWV_DAG_UNKNOWN_AUTHORITY or NWV_DAG_CERTIFICATE_REQUIRES_QUORUM. */
int nwv_certificate_new(const nwv_committee* committee, size_t n_votes, const uint8_t* vote_pks,
                        const uint8_t* vote_sigs, int check_stake, uint32_t* signed_out,
                        size_t* n_signed, uint8_t* sigs_out, size_t* n_sigs);

/* Committee::quorum_threshold (config/src/lib.rs:537-542): 2 * total / 3 + 1 */
uint64_t nwv_committee_quorum_threshold(const nwv_committee* committee);

/* ---- the same layer under BLS12-381, the reference's default scheme (crypto/src/lib.rs:29-33:
 * PublicKey = BLS12381PublicKey, 96 bytes; Signature = BLS12381Signature, 48 bytes;
 * AggregateSignature = BLS12381AggregateSignature, one 48-byte G1 point or none).  The digests
 * hash the 96-byte keys where the Ed25519 layout has 32-byte ones (Header::digest :209-227 hashes
 * the author, Vote / Certificate::digest the origin).  Verification runs on the GPU through
 * include/nwv_bls.h; the committee's keys are registered in the device's BLS key cache. ---- */
typedef struct {
    size_t n;
    const uint8_t* keys; /* n x 96 bytes, ascending byte order (BTreeMap order = bitmap order) */
    const uint64_t* stakes;
    uint64_t epoch;
    const uint32_t* n_workers;
    const uint32_t* const* worker_ids;
} nwv_bls_committee;

typedef struct {
    const uint8_t* author;          /* 96 */
    uint64_t round;
    uint64_t epoch;
    size_t n_payload;
    const uint8_t* payload_digests; /* n_payload x 32 */
    const uint32_t* payload_workers;
    size_t n_parents;
    const uint8_t* parents;         /* n_parents x 32 */
    const uint8_t* id;              /* 32 */
    const uint8_t* signature;       /* 48 */
} nwv_bls_header;

typedef struct {
    const uint8_t* id;        /* 32 */
    uint64_t round;
    uint64_t epoch;
    const uint8_t* origin;    /* 96 */
    const uint8_t* author;    /* 96 */
    const uint8_t* signature; /* 48 */
} nwv_bls_vote;

/* aggregated_signature: the 48-byte aggregate, or NULL for an aggregate holding no signature
 * (AggregateSignature::default(), sig: None -> verification fails) */
typedef struct {
    nwv_bls_header header;
    size_t n_signed;
    const uint32_t* signed_authorities;
    const uint8_t* aggregated_signature;
} nwv_bls_certificate;

int nwv_bls_header_digest_many(nwv_ctx* ctx, size_t n, const nwv_bls_header* h, uint8_t* out);
int nwv_bls_vote_digest_many(nwv_ctx* ctx, size_t n, const nwv_bls_vote* v, uint8_t* out);
int nwv_bls_certificate_digest_many(nwv_ctx* ctx, size_t n, const nwv_bls_certificate* c, uint8_t* out);
/* Header::verify / Vote::verify / Certificate::verify of a primary's queued messages in ONE call:
 * every digest in one BLAKE2b launch, every signature check (header and vote signatures:
 * Verifier::verify; each certificate's aggregate over its signers: fast_aggregate_verify) in one
 * nwv_bls_verify_many call; results as nwv_verify_mixed_many's (NWV_DAG_* per item). */
int nwv_bls_verify_mixed_many(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t n_headers,
                              const nwv_bls_header* headers, int32_t* header_results, size_t n_votes,
                              const nwv_bls_vote* votes, int32_t* vote_results, size_t n_certs,
                              const nwv_bls_certificate* certs, int32_t* cert_results);
/* CertificatesResponse::validate_certificates under BLS (as nwv_validate_certificates) */
int nwv_bls_validate_certificates(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t n,
                                  const nwv_bls_certificate* c, size_t* n_invalid, size_t* invalid_idx);
/* Certificate::new / new_unsigned (types/src/primary.rs:411-485) under BLS: the votes (pk 96,
 * sig 48) sorted by key, repeats dropped, matched against the committee; the aggregate is the G1
 * sum of the kept signatures (AggregateSignature::aggregate on the GPU; a signature that does not
 * decode or lies outside G1 -> NWV_DAG_INVALID_SIGNATURE).  *has_agg = 0 when no vote was kept
 * (AggregateSignature::default()).  Returns an NWV_DAG_* code or a negative error. */
int nwv_bls_certificate_new(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t n_votes,
                            const uint8_t* vote_pks, const uint8_t* vote_sigs, int check_stake,
                            uint32_t* signed_out, size_t* n_signed, uint8_t* agg_out, int* has_agg);

#ifdef __cplusplus
}
#endif
#endif /* NWV_TYPES_H */
