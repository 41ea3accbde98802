/*
 * nwv_service.h -- batching verification service in front of the primary's
 * Core::sanitize_header / sanitize_vote / sanitize_certificate (primary/src/core.rs:497-573,
 * driven by Core::run :614-714) and CertificatesResponse::validate_certificates
 * (primary/src/block_synchronizer/responses.rs:95-141).
 *
 * The reference verifies one message at a time inside its single Core task, so a GPU would see
 * batches of 1 (header, vote) or 1 + Q (certificate) signatures and pay the fixed latency of a
 * batch verification for each.  The service lets any number of threads (tokio tasks through
 * spawn_blocking, or the Core loop itself) submit headers, votes and certificates; a flusher
 * thread coalesces everything pending into ONE nwv_verify_mixed_many call (one BLAKE2b launch,
 * one batch MSM) when max_batch items are queued or the oldest has waited max_wait_us, and hands
 * every submitter its own result: exactly the DagError code Header::verify (types/src/primary.rs
 * :150-183), Vote::verify (:307-328) or Certificate::verify (:487-537) returns for that item, or
 * a negative nwv error if the engine call failed.
 *
 * Items are copied at submission (the caller may free its buffers as soon as submit returns);
 * the committee is copied at creation and replaced by nwv_service_set_committee (epoch change,
 * Core::change_epoch primary/src/core.rs:592-611).  All entry points are thread-safe.
 */
#ifndef NWV_SERVICE_H
#define NWV_SERVICE_H

#include <stddef.h>
#include <stdint.h>

#include "nwv_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nwv_service nwv_service;

/* completion callback: called exactly once per submitted item, from a service thread, without
 * the service lock held.  It may submit further items asynchronously; the blocking calls
 * (nwv_service_verify_*, nwv_service_flush) on the SAME service return NWV_ERR_REENTRANT from
 * inside its callback (they would wait on the thread running it), and so do blocking calls on
 * another service whose callbacks are already waiting (directly or through others) on this one
 * (a cycle of such waits could leave every flusher waiting); it must not call nwv_service_free. */
typedef void (*nwv_done_fn)(void* user, int32_t result);

/* max_batch: flush as soon as this many items are pending (>= 1); max_wait_us: flush when the
 * oldest pending item has waited this long (0: flush whatever is pending at once). */
int nwv_service_create(nwv_ctx* ctx, const nwv_committee* committee, size_t max_batch, uint32_t max_wait_us,
                       nwv_service** out);
/* burst flush (default off): also flush once no item has been submitted for idle_us, so a burst
 * of submissions (a round of headers, votes and certificates delivered together) goes out as one
 * call as soon as it ends instead of waiting out max_wait_us, or being cut by it; max_batch and
 * max_wait_us still apply.  0 turns it off. */
int nwv_service_set_idle(nwv_service* svc, uint32_t idle_us);
/* later submissions are verified against this committee; pending items are completed first */
int nwv_service_set_committee(nwv_service* svc, const nwv_committee* committee);

/* asynchronous submission: done(user, result) fires once the item's batch is verified */
int nwv_service_submit_header(nwv_service* svc, const nwv_header* h, nwv_done_fn done, void* user);
int nwv_service_submit_vote(nwv_service* svc, const nwv_vote* v, nwv_done_fn done, void* user);
int nwv_service_submit_certificate(nwv_service* svc, const nwv_certificate* c, nwv_done_fn done, void* user);

/* blocking forms (submit, then wait for this item's result): return NWV_OK with *result set, or
 * a negative error */
int nwv_service_verify_header(nwv_service* svc, const nwv_header* h, int32_t* result);
int nwv_service_verify_vote(nwv_service* svc, const nwv_vote* v, int32_t* result);
int nwv_service_verify_certificate(nwv_service* svc, const nwv_certificate* c, int32_t* result);

/* ---- the same service under BLS12-381, the reference's default scheme (crypto/src/lib.rs:29-33):
 * the nwv_bls_* structs of nwv_types.h (96-byte keys, 48-byte signatures, one 48-byte aggregate
 * per certificate); each flush is ONE nwv_bls_verify_mixed_many call (every digest in one BLAKE2b
 * launch, every signature check -- header and vote signatures, certificates' aggregates -- in one
 * nwv_bls_verify_many call).  A service is of one scheme: the other scheme's calls on it return
 * NWV_ERR_ARG.  flush, stats and free are shared. */
int nwv_service_create_bls(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t max_batch, uint32_t max_wait_us,
                           nwv_service** out);
int nwv_service_set_committee_bls(nwv_service* svc, const nwv_bls_committee* committee);
int nwv_service_submit_bls_header(nwv_service* svc, const nwv_bls_header* h, nwv_done_fn done, void* user);
int nwv_service_submit_bls_vote(nwv_service* svc, const nwv_bls_vote* v, nwv_done_fn done, void* user);
int nwv_service_submit_bls_certificate(nwv_service* svc, const nwv_bls_certificate* c, nwv_done_fn done,
                                       void* user);
int nwv_service_verify_bls_header(nwv_service* svc, const nwv_bls_header* h, int32_t* result);
int nwv_service_verify_bls_vote(nwv_service* svc, const nwv_bls_vote* v, int32_t* result);
int nwv_service_verify_bls_certificate(nwv_service* svc, const nwv_bls_certificate* c, int32_t* result);
/* returns once every item submitted before the call has completed */
int nwv_service_flush(nwv_service* svc);

/* out[0] engine calls, [1] items verified, [2] largest batch, [3] flushes triggered by
 * max_batch, [4] by max_wait_us or the idle gap, [5] by nwv_service_flush / set_committee / free */
int nwv_service_stats(nwv_service* svc, uint64_t out[6]);

/* completes every pending item, then stops the service threads */
void nwv_service_free(nwv_service* svc);

#ifdef __cplusplus
}
#endif
#endif /* NWV_SERVICE_H */
