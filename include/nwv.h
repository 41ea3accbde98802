/*
 * nwv.h -- C ABI of the MI355X (gfx950) Ed25519 / BLAKE2b-256 verification engine.
 *
 * Drop-in boundary for erwanor/narwhal's signature-verification hot path.  The reference
 * selects its scheme with the five type aliases at crypto/src/lib.rs:29-33 (swap rule
 * :19-27); a GPU-backed Ed25519 scheme module implements the fastcrypto 0.1.2 traits and calls
 * these entry points over FFI (binding stubs: INTEGRATION.md).  Plain pointers and sizes
 * only; the caller owns every buffer; nothing is retained after a call returns.
 *
 * Return codes: NWV_OK (0) on success, NWV_ERR_SIGNATURE (1) when a signature check fails,
 * negative values for usage / runtime errors.  The library never aborts the process.
 * Thread safety: a context may be shared by threads; calls on one device are serialized by
 * a per-device lock.  Every verification call runs on the GPU; if the HIP code object or a
 * device is unavailable nwv_init fails (there is no CPU fallback in this library).
 */
#ifndef NWV_H
#define NWV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NWV_OK 0
#define NWV_ERR_SIGNATURE 1      /* verification failed (signature::Error::new())          */
#define NWV_ERR_ARG (-1)         /* bad argument (null pointer, n out of range)             */
#define NWV_ERR_HIP (-2)         /* HIP runtime error                                       */
#define NWV_ERR_OOM (-3)         /* device or host allocation failed                        */
#define NWV_ERR_NODEV (-4)       /* no usable gfx950 device / code object not loadable      */
#define NWV_ERR_EMPTY (-5)       /* verify_batch_empty_fail on an empty batch               */
#define NWV_ERR_LENGTH (-6)      /* |pks| != |sigs| (or messages) in a batch API            */
#define NWV_ERR_REENTRANT (-7)   /* blocking service call made from a completion callback   */

#define NWV_ABI_VERSION 1

typedef struct nwv_ctx nwv_ctx;

/* nwv_init flags.  Batch verification (nwv_ed25519_verify_batch and the trait entry points built
 * on it) runs one Pippenger MSM per device shard (env NWV_MSM_MIN_N sets a minimum shard size,
 * below which the per-signature pipeline runs); these force one or the other. */
#define NWV_FLAG_MSM_ALWAYS 1u
#define NWV_FLAG_MSM_NEVER 2u
/* diagnostic: launch the MSM's hashing (k_msm_scalars) and decompression (k_msm_points) as two
 * kernels instead of one k_msm_prep grid (per-kernel timing of the decompression alone) */
#define NWV_FLAG_MSM_SPLIT_PREP 4u
/* keyed calls (nwv_ed25519_verify_batch_keyed[_digests], the types layer) keep each key's
 * decompressed point and its 2^128 multiple in a per-device cache, so their MSM scalars are
 * 128-bit (half the windows and doublings); this flag turns the cache off (every keyed call
 * decompresses its keys, full-width scalars).  Env NWV_KEYCACHE_MAX_KEYS (default 4096): keyed
 * calls with more distinct keys than this go uncached. */
#define NWV_FLAG_NO_KEYCACHE 8u
/* diagnostic / tests: the batch MSM's two-level counting sort (coarse bins, then each bin in one
 * workgroup) whenever the sort has more than one chunk; by default it is used for windows of
 * NWV_MSM_SORT2_MIN_PTS points or more (env, default 2^20) */
#define NWV_FLAG_MSM_SORT2 16u
/* diagnostic / tests: when a batch MSM over per-signature keys rejects and the verdict bits are
 * wanted, the per-signature pass reuses the MSM's work by default: point tables from its
 * decompressed records (k_ed_points_msm) and k_i / the s < l flag its hash role stored (no
 * k_ed_hash); this flag makes the pass hash and decompress again */
#define NWV_FLAG_NO_MSM_REUSE 32u
/* BLS12-381 (nwv_bls.h): verify every item with its own two-pair Miller loop and final
 * exponentiation on the 8-lane group kernels (round-3 form) instead of the default wave engine --
 * for tests and A/B measurements; statuses are the same either way */
#define NWV_FLAG_BLS_PER_ITEM 64u
/* BLS12-381 (nwv_bls.h): check a call's pairing equations as ONE random linear combination on the
 * 8-lane group kernels (per item only after a rejection) instead of the default, every item's
 * own pairing check on one 64-lane wave (exact per-item statuses either way) */
#define NWV_FLAG_BLS_BATCH 128u
/* BLS12-381 (nwv_bls.h): signatures that passed a verify call of up to 1024 items on the wave path
 * are kept decoded (and G1-checked) on the device, by their 48 bytes, in a ring of 65,536;
 * nwv_bls_aggregate over signatures that are all in it sums the kept points instead of decoding
 * and checking each again (the Core aggregates votes it has already verified).  This flag turns
 * the ring off (every aggregate decodes and checks its signatures). */
#define NWV_FLAG_NO_SIGCACHE 256u
/* diagnostic / tests: small batch MSMs (at most NWV_MSM_ROW_PREP_MAX points to decompress, env,
 * default 8192) run each point's decompression power on a 16-lane row (k_msm_prep's row form,
 * latency-bound batches); this flag keeps every batch on the lane-local decompression */
#define NWV_FLAG_NO_ROW_PREP 512u
/* diagnostic / tests: large host-staged batches (>= 16 MB of pk, sig and messages) start the
 * batch MSM's decompressions -- and, when verdict bits are wanted, the per-signature fallback's
 * tables -- on a second stream once pk and sig are on the device, under the messages' transfer;
 * this flag keeps the one-stream order (every kernel after the whole copy) */
#define NWV_FLAG_NO_EARLY_PREP 1024u
/* diagnostic / tests: a keyed batch MSM whose hashes fit one k_msm_prep workgroup sums its keys'
 * scalars in that workgroup (no k_msm_keysum launch); this flag keeps the separate launch */
#define NWV_FLAG_NO_FUSED_KEYSUM 2048u
/* diagnostic / tests: a keyed batch of at most 64 signatures whose keys were all registered
 * (nwv_keycache_register: each key gets a fixed-base comb table) is checked in one launch,
 * signature by signature (k_ed_tiny); this flag sends it through the batch MSM instead */
#define NWV_FLAG_NO_TINY 4096u
/* BLS12-381 calls of at most 1,024 items (the per-call paths) record the per-stage timing events
 * that nwv_bls_last_kernel_ms reports only with this flag: the events cost a single verification
 * ~0.1 ms (larger calls always record them) */
#define NWV_FLAG_BLS_STAGE_TIMES 8192u

/* ------------------------------------------------------------------ lifecycle ----- */
/* Process-wide context creation (created once, in Primary::spawn).
 * n_devices: 0 = all visible devices, k = the first k.  flags: NWV_FLAG_* or 0. */
int nwv_init(nwv_ctx** out, int n_devices, uint32_t flags);
/* Context bound to one device ordinal (one process per GPU deployments, bench.py). */
int nwv_init_device(nwv_ctx** out, int device_ordinal, uint32_t flags);
void nwv_free(nwv_ctx* ctx);
int nwv_device_count(const nwv_ctx* ctx);
/* Diagnostics: how the context's batch calls ran so far, summed over its devices: out[0] keyed
 * batches checked by the one-launch path (k_ed_tiny), out[1] batch MSMs, out[2] per-signature
 * passes (verify_each, or after a rejected MSM when verdict bits were asked for). */
int nwv_diag_counters(const nwv_ctx* ctx, uint64_t out[3]);
/* HIP ordinal of the context's i-th device (-1 if out of range) */
int nwv_device_ordinal(const nwv_ctx* ctx, int i);
int nwv_abi_version(void);
/* last error text for this thread (static storage, never NULL) */
const char* nwv_last_error(void);

/* ------------------------------------------------------------------ Ed25519 --------- */
/* Per-signature ZIP-215 verdicts (ed25519_consensus::VerificationKey::verify semantics for
 * every item; replaces the per-signature verify of types/src/primary.rs:179-182 / :325-327
 * and is the exact-bad-set fallback of primary/src/block_synchronizer/responses.rs:95-141).
 *   pk       n x 32 bytes (compressed A, raw as received: decoding happens here)
 *   sig      n x 64 bytes (R || s)
 *   msg_base message bytes; message i = msg_base[msg_off[i] .. msg_off[i] + msg_len[i])
 *            (a shared message, e.g. a certificate digest, is all msg_off[i] = 0)
 *   verdict_bits  ceil(n/64) words; bit (i % 64) of word i/64 = 1 <=> signature i accepted
 * Work is sharded by contiguous index ranges over the context's devices. */
int nwv_ed25519_verify_each(nwv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig,
                            const uint8_t* msg_base, const uint64_t* msg_off,
                            const uint32_t* msg_len, uint64_t* verdict_bits);

/* Batch verification (ed25519_consensus::batch::Verifier::verify semantics: one verdict for
 * the whole batch).  *all_valid = 1 iff every signature verifies.  seed32 keys the per-batch
 * random coefficients (the caller passes 32 bytes from a CSPRNG; OsRng in the reference).
 * When verdict_bits_or_null is non-NULL and the batch fails, it receives the exact
 * per-signature verdicts (the fallback that pinpoints the bad indices). */
int nwv_ed25519_verify_batch(nwv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig,
                             const uint8_t* msg_base, const uint64_t* msg_off,
                             const uint32_t* msg_len, const uint8_t seed32[32], int* all_valid,
                             uint64_t* verdict_bits_or_null);

/* Batch verification with each verifying key given once: keys (n_keys x 32) and key_idx[n]
 * (signature i is by keys[key_idx[i]]).  ed25519_consensus's batch verifier groups its entries
 * by key the same way (one MSM point per distinct key with coefficient sum z_i k_i), so the
 * device decompresses each distinct key once and carries one point per key instead of one per
 * signature -- the committee case of Certificate::verify / validate_certificates.  Same verdict
 * semantics and outputs as nwv_ed25519_verify_batch. */
int nwv_ed25519_verify_batch_keyed(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys, size_t n,
                                   const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                                   const uint64_t* msg_off, const uint32_t* msg_len,
                                   const uint8_t seed32[32], int* all_valid, uint64_t* verdict_bits_or_null);
/* Digest-then-verify: the n_pre preimages are hashed with BLAKE2b-256 on the
 * device (digests_out receives them, n_pre x 32) and signature i is checked over the 32-byte
 * digest digest_idx[i] straight from device memory, with no host round trip between the hash and
 * the batch verification.  This is how Narwhal signs: a vote's / certificate's signatures are over
 * Vote::digest / Certificate::digest (types/src/primary.rs:351-364, :594-607) and a header's over
 * its id = Header::digest (:209-227).  Otherwise as nwv_ed25519_verify_batch_keyed. */
int nwv_ed25519_verify_batch_keyed_digests(nwv_ctx* ctx, size_t n_pre, const uint8_t* pre_base,
                                           const uint64_t* pre_off, const uint64_t* pre_len,
                                           uint8_t* digests_out, size_t n_keys, const uint8_t* keys,
                                           size_t n, const uint32_t* key_idx, const uint8_t* sig,
                                           const uint32_t* digest_idx, const uint8_t seed32[32],
                                           int* all_valid, uint64_t* verdict_bits_or_null);

/* Fill every device's committee key cache with n_keys keys (n_keys x 32), e.g. at epoch start
 * (Core::change_epoch, primary/src/core.rs:592-611).  Batch calls fill the cache themselves;
 * nwv_ed25519_pubkey_verify only looks its key up (an unseen key runs uncached and takes no
 * slot), so registering the committee gives its members' single verifies the cached form.  Each
 * registered key also gets a fixed-base comb table (i 16^j A, 64 KiB), which sends keyed batches
 * of at most 64 signatures by registered keys -- Certificate::verify, Header::verify,
 * Vote::verify -- through the one-launch path.  Registering the same key list again is a no-op.
 * A full cache leaves further keys uncached; verdicts never depend on the cache. */
int nwv_keycache_register(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys);

/* ---- fastcrypto 0.1.2 trait surface (Ed25519 scheme module; contract of
 *      crypto/src/bls12377/mod.rs:264-291 and :485-577) ---- */
/* Verifier::verify(&self, msg, sig): NWV_OK or NWV_ERR_SIGNATURE */
int nwv_ed25519_pubkey_verify(nwv_ctx* ctx, const uint8_t pk[32], const uint8_t* msg,
                              size_t msg_len, const uint8_t sig[64]);
/* VerifyingKey::verify_batch_empty_fail(msg, pks, sigs): NWV_ERR_EMPTY if n_sigs == 0,
 * NWV_ERR_LENGTH if n_pks != n_sigs, else NWV_OK / NWV_ERR_SIGNATURE */
int nwv_ed25519_verify_batch_empty_fail(nwv_ctx* ctx, const uint8_t* msg, size_t msg_len,
                                        const uint8_t* pks, size_t n_pks, const uint8_t* sigs,
                                        size_t n_sigs, const uint8_t seed32[32]);
/* AggregateAuthenticator::verify(&self, pks, msg) for Ed25519AggregateSignature (the
 * aggregate is the list of signatures): NWV_ERR_LENGTH if n_pks != n_sigs */
int nwv_ed25519_aggregate_verify(nwv_ctx* ctx, const uint8_t* sigs, size_t n_sigs,
                                 const uint8_t* pks, size_t n_pks, const uint8_t* msg,
                                 size_t msg_len, const uint8_t seed32[32]);
/* AggregateAuthenticator::batch_verify(sigs, pks_iters, msgs): n_aggs aggregates; aggregate
 * a has n_sigs[a] signatures at sigs[a], n_pks[a] keys at pks[a] and message msgs[a].  Every
 * length mismatch -> NWV_ERR_LENGTH before any crypto. */
int nwv_ed25519_aggregate_batch_verify(nwv_ctx* ctx, size_t n_aggs, const uint8_t* const* sigs,
                                       const size_t* n_sigs, const uint8_t* const* pks,
                                       const size_t* n_pks, const uint8_t* const* msgs,
                                       const size_t* msg_lens, size_t n_msgs,
                                       const uint8_t seed32[32]);

/* ------------------------------------------------------------------ BLAKE2b-256 ------ */
/* fastcrypto::blake2b_256 (VarBlake2b::new(32)) of n independent inputs
 * (types/src/primary.rs:65-73 Batch::digest over pre-concatenated tx bytes, :209-227,
 * :351-364, :594-607 header / vote / certificate digests).  out: n x 32 bytes. */
int nwv_blake2b256_many(nwv_ctx* ctx, size_t n, const uint8_t* base, const uint64_t* off,
                        const uint64_t* len, uint8_t* out);
/* serialized_batch_digest (types/src/worker.rs:44-80) of n bincode WorkerMessage::Batch
 * buffers.  out: n x 32; err_offset[i] = -1 on success, else the byte offset reported by
 * DigestError::InvalidArgumentError.  Returns NWV_OK if all succeeded, NWV_ERR_ARG otherwise. */
int nwv_batch_digest_serialized(nwv_ctx* ctx, size_t n, const uint8_t* base, const uint64_t* off,
                                const uint64_t* len, uint8_t* out, int64_t* err_offset);

/* ------------------------------------------------------------------ resident batches --- */
/* Device-resident staging for throughput measurement and pipelined callers: the inputs are
 * copied to HBM once (SoA: pk, sig, message arena), then verified repeatedly without host
 * traffic.  One staged batch lives on one device of the context. */
typedef struct nwv_staged nwv_staged;
int nwv_stage_ed25519(nwv_ctx* ctx, int device_index, size_t n, const uint8_t* pk,
                      const uint8_t* sig, const uint8_t* msg_base, const uint64_t* msg_off,
                      const uint32_t* msg_len, nwv_staged** out);
/* keyed form (see nwv_ed25519_verify_batch_keyed): mode-1 runs carry one MSM point per key */
int nwv_stage_ed25519_keyed(nwv_ctx* ctx, int device_index, size_t n_keys, const uint8_t* keys, size_t n,
                            const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                            const uint64_t* msg_off, const uint32_t* msg_len, nwv_staged** out);
/* mode 0: per-signature verdicts (K1-K4); mode 1: batch verdict through one Pippenger MSM (K5),
 * coefficients keyed by seed32 (NULL: OS entropy).  Asynchronous on the batch's own stream;
 * nwv_staged_sync waits.  Verdicts stay on the device until nwv_staged_fetch, which after a
 * rejected mode-1 run also runs the per-signature fallback (exact bad indices). */
int nwv_staged_run(nwv_staged* st, int mode, const uint8_t seed32[32]);
/* or-ed into nwv_staged_run's mode: launch kernel by kernel with HIP events around each one
 * (feeds nwv_staged_kernel_times).  Untimed mode-1 runs replay a HIP graph of the batch MSM
 * captured on the batch's first untimed run. */
#define NWV_RUN_TIMED 0x100
int nwv_staged_sync(nwv_staged* st);
int nwv_staged_fetch(nwv_staged* st, uint64_t* verdict_bits, int* all_valid);
/* average device time (ms) per run of each pipeline kernel since the last reset, measured
 * with HIP events on the stream the kernels run on: avg_ms[0] = k_ed_hash (K1, K3),
 * avg_ms[1] = k_ed_points (K2), avg_ms[2] = k_ed_straus (K4, the dominant kernel) */
int nwv_staged_kernel_ms(nwv_staged* st, double avg_ms[3], int reset);
/* per-kernel average device time (ms) of mode `mode` runs since the last reset: fills up to
 * cap (name, ms) pairs in launch order (names point to static strings) and returns the number
 * of kernels in that pipeline (< 0 on error).  mode 1 (batch MSM, K5) kernels:
 * k_msm_prep (hash + decompression + the basepoint term), k_msm_hist, k_msm_wscan,
 * k_msm_scatter, k_msm_bucket, k_msm_tail; k_msm_keysum is timed with k_msm_prep, and
 * batches whose counting sort fits one chunk per window time k_msm_sort1 as k_msm_hist with
 * zero-length k_msm_wscan / k_msm_scatter slots.  Under NWV_FLAG_MSM_SPLIT_PREP k_msm_prep is
 * split into k_msm_scalars and k_msm_points. */
int nwv_staged_kernel_times(nwv_staged* st, int mode, int cap, const char** names, double* avg_ms,
                            int reset);
/* shape of the staged batch's MSM (diagnostics for roofline accounting): out[0] points
 * (na + 1 + n), [1] windows, [2] windows that carry the R_i points (the 128-bit z range),
 * [3] buckets over all windows, [4] bucket entries of the last mode-1 run (0 before one),
 * [5] sort chunks, [6] entries per k_msm_bucket lane, [7] A points (n, or the distinct keys) */
int nwv_staged_msm_stats(nwv_staged* st, uint64_t out[8]);
/* batch verdicts of every mode-1 run since staging, counted on the device by the run itself
 * (graph replays included): out[0] accepted runs, out[1] rejected runs.  Waits for the stream. */
int nwv_staged_run_tally(nwv_staged* st, uint64_t out[2]);
/* step-completion timestamps: record HIP event `slot` (< 65536) on the batch's stream (it fires
 * when the work queued before it on that stream is done); *ms = time from a's mark to b's */
int nwv_staged_mark(nwv_staged* st, int slot);
int nwv_staged_mark_elapsed(nwv_staged* a, int slot_a, nwv_staged* b, int slot_b, float* ms);
void nwv_staged_free(nwv_staged* st);

/* ------------------------------------------------------------------ synthetic data ----- */
/* RFC 8032 key generation and signing on the GPU, for synthetic workloads and tests
 * (the reference signs on the CPU with SignatureService; this is tooling, not the verify
 * path).  seeds n x 32, msgs as above; outputs pk n x 32, sig n x 64. */
int nwv_ed25519_sign_many(nwv_ctx* ctx, size_t n, const uint8_t* seeds, const uint8_t* msg_base,
                          const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* pk_out,
                          uint8_t* sig_out);

#ifdef __cplusplus
}
#endif
#endif /* NWV_H */
