//! Raw bindings of the engine's C ABI: `include/nwv.h`, `include/nwv_types.h` and
//! `include/nwv_service.h` of the narwhal_amd checkout (`narwhal_amd/lib/libnwv.so`, built for
//! gfx950 by `make lib`).  Every declaration here mirrors one prototype there, parameter by
//! parameter; `tests/test_rust_ffi.py` checks that mechanically.  Safe wrappers: `lib.rs`.
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

/// `nwv_ctx`: a context over one or more gfx950 devices (opaque).
#[repr(C)]
pub struct NwvCtx {
    _private: [u8; 0],
}
/// `nwv_staged`: a device-resident batch (opaque).
#[repr(C)]
pub struct NwvStaged {
    _private: [u8; 0],
}
/// `nwv_service`: a batching verification service (opaque).
#[repr(C)]
pub struct NwvService {
    _private: [u8; 0],
}

pub const NWV_OK: c_int = 0;
pub const NWV_ERR_SIGNATURE: c_int = 1;
pub const NWV_ERR_ARG: c_int = -1;
pub const NWV_ERR_HIP: c_int = -2;
pub const NWV_ERR_OOM: c_int = -3;
pub const NWV_ERR_NODEV: c_int = -4;
pub const NWV_ERR_EMPTY: c_int = -5;
pub const NWV_ERR_LENGTH: c_int = -6;
pub const NWV_ERR_REENTRANT: c_int = -7;
pub const NWV_ABI_VERSION: c_int = 1;
// nwv_init flags
pub const NWV_FLAG_MSM_ALWAYS: u32 = 1;
pub const NWV_FLAG_MSM_NEVER: u32 = 2;
pub const NWV_FLAG_MSM_SPLIT_PREP: u32 = 4;
pub const NWV_FLAG_NO_KEYCACHE: u32 = 8;
pub const NWV_FLAG_MSM_SORT2: u32 = 16;
pub const NWV_FLAG_NO_MSM_REUSE: u32 = 32;
pub const NWV_FLAG_BLS_PER_ITEM: u32 = 64;
pub const NWV_FLAG_BLS_BATCH: u32 = 128;
/// BLS12-381: no verified-signature ring (every aggregate decodes and G1-checks its signatures)
pub const NWV_FLAG_NO_SIGCACHE: u32 = 256;
/// Keyed batches of <= 64 signatures by registered keys go through the batch MSM, not k_ed_tiny.
pub const NWV_FLAG_NO_TINY: u32 = 4096;
/// BLS12-381 calls of <= 1,024 items record the per-stage timing events (nwv_bls_last_kernel_ms).
pub const NWV_FLAG_BLS_STAGE_TIMES: u32 = 8192;

// per-item BLS12-381 statuses (include/nwv_bls.h)
pub const NWV_BLS_OK: i32 = 0;
pub const NWV_BLS_BAD_ENCODING: i32 = 1;
pub const NWV_BLS_NOT_ON_CURVE: i32 = 2;
pub const NWV_BLS_NOT_IN_GROUP: i32 = 3;
pub const NWV_BLS_AGGR_MISMATCH: i32 = 4;
pub const NWV_BLS_VERIFY_FAIL: i32 = 5;
pub const NWV_BLS_PK_INFINITY: i32 = 6;

pub const NWV_DAG_OK: i32 = 0;
pub const NWV_DAG_INVALID_EPOCH: i32 = 10;
pub const NWV_DAG_INVALID_HEADER_ID: i32 = 11;
pub const NWV_DAG_UNKNOWN_AUTHORITY: i32 = 12;
pub const NWV_DAG_MALFORMED_HEADER: i32 = 13;
pub const NWV_DAG_INVALID_SIGNATURE: i32 = 14;
pub const NWV_DAG_CERTIFICATE_REQUIRES_QUORUM: i32 = 15;
pub const NWV_DAG_INVALID_BITMAP: i32 = 16;

/// `nwv_committee` (config::Committee + the worker cache's worker ids, keys in BTreeMap order).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvCommittee {
    pub n: usize,
    pub keys: *const u8,
    pub stakes: *const u64,
    pub epoch: u64,
    pub n_workers: *const u32,
    pub worker_ids: *const *const u32,
}

/// `nwv_header` (types::Header, types/src/primary.rs:75-86).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvHeader {
    pub author: *const u8,
    pub round: u64,
    pub epoch: u64,
    pub n_payload: usize,
    pub payload_digests: *const u8,
    pub payload_workers: *const u32,
    pub n_parents: usize,
    pub parents: *const u8,
    pub id: *const u8,
    pub signature: *const u8,
}

/// `nwv_vote` (types::Vote, types/src/primary.rs:251-259).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvVote {
    pub id: *const u8,
    pub round: u64,
    pub epoch: u64,
    pub origin: *const u8,
    pub author: *const u8,
    pub signature: *const u8,
}

/// `nwv_certificate` (types::Certificate, types/src/primary.rs:388-395).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvCertificate {
    pub header: NwvHeader,
    pub n_signed: usize,
    pub signed_authorities: *const u32,
    pub n_sigs: usize,
    pub aggregated_signature: *const u8,
}

/// `nwv_bls_committee`: the committee under BLS12-381 (96-byte keys in BTreeMap order).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvBlsCommittee {
    pub n: usize,
    pub keys: *const u8,
    pub stakes: *const u64,
    pub epoch: u64,
    pub n_workers: *const u32,
    pub worker_ids: *const *const u32,
}

/// `nwv_bls_header` (types::Header with a 96-byte author and a 48-byte signature).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvBlsHeader {
    pub author: *const u8,
    pub round: u64,
    pub epoch: u64,
    pub n_payload: usize,
    pub payload_digests: *const u8,
    pub payload_workers: *const u32,
    pub n_parents: usize,
    pub parents: *const u8,
    pub id: *const u8,
    pub signature: *const u8,
}

/// `nwv_bls_vote` (types::Vote under BLS12-381).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvBlsVote {
    pub id: *const u8,
    pub round: u64,
    pub epoch: u64,
    pub origin: *const u8,
    pub author: *const u8,
    pub signature: *const u8,
}

/// `nwv_bls_certificate`: the aggregate is one 48-byte G1 point, or null for `sig: None`.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct NwvBlsCertificate {
    pub header: NwvBlsHeader,
    pub n_signed: usize,
    pub signed_authorities: *const u32,
    pub aggregated_signature: *const u8,
}

/// `nwv_done_fn`: completion callback of the batching service.
pub type NwvDoneFn = Option<unsafe extern "C" fn(user: *mut c_void, result: i32)>;

#[link(name = "nwv")]
extern "C" {
    // ---- lifecycle (include/nwv.h)
    pub fn nwv_init(out: *mut *mut NwvCtx, n_devices: c_int, flags: u32) -> c_int;
    pub fn nwv_init_device(out: *mut *mut NwvCtx, device_ordinal: c_int, flags: u32) -> c_int;
    pub fn nwv_free(ctx: *mut NwvCtx);
    pub fn nwv_device_count(ctx: *const NwvCtx) -> c_int;
    pub fn nwv_diag_counters(ctx: *const NwvCtx, out: *mut u64) -> c_int;
    pub fn nwv_device_ordinal(ctx: *const NwvCtx, i: c_int) -> c_int;
    pub fn nwv_abi_version() -> c_int;
    pub fn nwv_last_error() -> *const c_char;
    // ---- Ed25519 verification (include/nwv.h)
    pub fn nwv_ed25519_verify_each(
        ctx: *mut NwvCtx,
        n: usize,
        pk: *const u8,
        sig: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        verdict_bits: *mut u64,
    ) -> c_int;
    pub fn nwv_ed25519_verify_batch(
        ctx: *mut NwvCtx,
        n: usize,
        pk: *const u8,
        sig: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        seed32: *const u8,
        all_valid: *mut c_int,
        verdict_bits_or_null: *mut u64,
    ) -> c_int;
    pub fn nwv_ed25519_verify_batch_keyed(
        ctx: *mut NwvCtx,
        n_keys: usize,
        keys: *const u8,
        n: usize,
        key_idx: *const u32,
        sig: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        seed32: *const u8,
        all_valid: *mut c_int,
        verdict_bits_or_null: *mut u64,
    ) -> c_int;
    pub fn nwv_ed25519_verify_batch_keyed_digests(
        ctx: *mut NwvCtx,
        n_pre: usize,
        pre_base: *const u8,
        pre_off: *const u64,
        pre_len: *const u64,
        digests_out: *mut u8,
        n_keys: usize,
        keys: *const u8,
        n: usize,
        key_idx: *const u32,
        sig: *const u8,
        digest_idx: *const u32,
        seed32: *const u8,
        all_valid: *mut c_int,
        verdict_bits_or_null: *mut u64,
    ) -> c_int;
    // committee key cache (include/nwv.h): fill it with the committee's keys at epoch start
    pub fn nwv_keycache_register(ctx: *mut NwvCtx, n_keys: usize, keys: *const u8) -> c_int;
    // ---- fastcrypto trait surface: Verifier::verify, VerifyingKey::verify_batch_empty_fail, AggregateAuthenticator::{verify, batch_verify} (include/nwv.h)
    pub fn nwv_ed25519_pubkey_verify(
        ctx: *mut NwvCtx,
        pk: *const u8,
        msg: *const u8,
        msg_len: usize,
        sig: *const u8,
    ) -> c_int;
    pub fn nwv_ed25519_verify_batch_empty_fail(
        ctx: *mut NwvCtx,
        msg: *const u8,
        msg_len: usize,
        pks: *const u8,
        n_pks: usize,
        sigs: *const u8,
        n_sigs: usize,
        seed32: *const u8,
    ) -> c_int;
    pub fn nwv_ed25519_aggregate_verify(
        ctx: *mut NwvCtx,
        sigs: *const u8,
        n_sigs: usize,
        pks: *const u8,
        n_pks: usize,
        msg: *const u8,
        msg_len: usize,
        seed32: *const u8,
    ) -> c_int;
    pub fn nwv_ed25519_aggregate_batch_verify(
        ctx: *mut NwvCtx,
        n_aggs: usize,
        sigs: *const *const u8,
        n_sigs: *const usize,
        pks: *const *const u8,
        n_pks: *const usize,
        msgs: *const *const u8,
        msg_lens: *const usize,
        n_msgs: usize,
        seed32: *const u8,
    ) -> c_int;
    // ---- BLS12-381 min_sig, the reference's default scheme (include/nwv_bls.h)
    pub fn nwv_bls_verify_many(
        ctx: *mut NwvCtx,
        n_keys: usize,
        keys: *const u8,
        n: usize,
        sigs: *const u8,
        pk_off: *const u32,
        pk_cnt: *const u32,
        pk_idx: *const u32,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        dst: *const u8,
        dst_len: usize,
        status: *mut i32,
    ) -> c_int;
    pub fn nwv_bls_last_kernel_ms(ctx: *mut NwvCtx, out_ms: *mut f64) -> c_int;
    pub fn nwv_bls_last_path(ctx: *mut NwvCtx) -> c_int;
    pub fn nwv_bls_last_keys(ctx: *mut NwvCtx, out: *mut u64) -> c_int;
    pub fn nwv_bls_keycache_register(ctx: *mut NwvCtx, n_keys: usize, keys: *const u8) -> c_int;
    pub fn nwv_bls_keycache_reset(ctx: *mut NwvCtx) -> c_int;
    pub fn nwv_bls_keycache_size(ctx: *mut NwvCtx) -> c_int;
    pub fn nwv_bls_verify(
        ctx: *mut NwvCtx,
        pk: *const u8,
        msg: *const u8,
        msg_len: usize,
        sig: *const u8,
    ) -> c_int;
    pub fn nwv_bls_aggregate_verify(
        ctx: *mut NwvCtx,
        sig48_or_null: *const u8,
        pks: *const u8,
        n_pks: usize,
        msg: *const u8,
        msg_len: usize,
    ) -> c_int;
    pub fn nwv_bls_verify_batch_empty_fail(
        ctx: *mut NwvCtx,
        msg: *const u8,
        msg_len: usize,
        pks: *const u8,
        n_pks: usize,
        sigs: *const u8,
        n_sigs: usize,
    ) -> c_int;
    pub fn nwv_bls_aggregate_batch_verify(
        ctx: *mut NwvCtx,
        n_aggs: usize,
        sigs48: *const *const u8,
        pks: *const *const u8,
        n_pks: *const usize,
        msgs: *const *const u8,
        msg_lens: *const usize,
        n_msgs: usize,
    ) -> c_int;
    pub fn nwv_bls_aggregate(
        ctx: *mut NwvCtx,
        n: usize,
        sigs48: *const u8,
        out48: *mut u8,
        status_or_null: *mut i32,
    ) -> c_int;
    pub fn nwv_bls_keygen_many(ctx: *mut NwvCtx, n: usize, sks: *const u8, pks: *mut u8) -> c_int;
    pub fn nwv_bls_sign_many(
        ctx: *mut NwvCtx,
        n: usize,
        sks: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        dst: *const u8,
        dst_len: usize,
        sigs: *mut u8,
    ) -> c_int;
    pub fn nwv_bls_hash_to_g1_many(
        ctx: *mut NwvCtx,
        n: usize,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        dst: *const u8,
        dst_len: usize,
        out96: *mut u8,
    ) -> c_int;
    pub fn nwv_bls_pairing_many(
        ctx: *mut NwvCtx,
        n: usize,
        P96: *const u8,
        Q192: *const u8,
        out576: *mut u8,
    ) -> c_int;
    // ---- BLAKE2b-256: Batch::digest, serialized_batch_digest (include/nwv.h)
    pub fn nwv_blake2b256_many(
        ctx: *mut NwvCtx,
        n: usize,
        base: *const u8,
        off: *const u64,
        len: *const u64,
        out: *mut u8,
    ) -> c_int;
    pub fn nwv_batch_digest_serialized(
        ctx: *mut NwvCtx,
        n: usize,
        base: *const u8,
        off: *const u64,
        len: *const u64,
        out: *mut u8,
        err_offset: *mut i64,
    ) -> c_int;
    // ---- device-resident batches (include/nwv.h)
    pub fn nwv_stage_ed25519(
        ctx: *mut NwvCtx,
        device_index: c_int,
        n: usize,
        pk: *const u8,
        sig: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        out: *mut *mut NwvStaged,
    ) -> c_int;
    pub fn nwv_stage_ed25519_keyed(
        ctx: *mut NwvCtx,
        device_index: c_int,
        n_keys: usize,
        keys: *const u8,
        n: usize,
        key_idx: *const u32,
        sig: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        out: *mut *mut NwvStaged,
    ) -> c_int;
    pub fn nwv_staged_run(st: *mut NwvStaged, mode: c_int, seed32: *const u8) -> c_int;
    pub fn nwv_staged_sync(st: *mut NwvStaged) -> c_int;
    pub fn nwv_staged_fetch(st: *mut NwvStaged, verdict_bits: *mut u64, all_valid: *mut c_int) -> c_int;
    pub fn nwv_staged_kernel_ms(st: *mut NwvStaged, avg_ms: *mut f64, reset: c_int) -> c_int;
    pub fn nwv_staged_kernel_times(
        st: *mut NwvStaged,
        mode: c_int,
        cap: c_int,
        names: *mut *const c_char,
        avg_ms: *mut f64,
        reset: c_int,
    ) -> c_int;
    pub fn nwv_staged_msm_stats(st: *mut NwvStaged, out: *mut u64) -> c_int;
    pub fn nwv_staged_run_tally(st: *mut NwvStaged, out: *mut u64) -> c_int;
    pub fn nwv_staged_mark(st: *mut NwvStaged, slot: c_int) -> c_int;
    pub fn nwv_staged_mark_elapsed(
        a: *mut NwvStaged,
        slot_a: c_int,
        b: *mut NwvStaged,
        slot_b: c_int,
        ms: *mut f32,
    ) -> c_int;
    pub fn nwv_staged_free(st: *mut NwvStaged);
    // ---- synthetic signing, for workloads and tests (include/nwv.h)
    pub fn nwv_ed25519_sign_many(
        ctx: *mut NwvCtx,
        n: usize,
        seeds: *const u8,
        msg_base: *const u8,
        msg_off: *const u64,
        msg_len: *const u32,
        pk_out: *mut u8,
        sig_out: *mut u8,
    ) -> c_int;
    // ---- types layer: digests and Header / Vote / Certificate verification (include/nwv_types.h)
    pub fn nwv_header_digest(ctx: *mut NwvCtx, h: *const NwvHeader, out: *mut u8) -> c_int;
    pub fn nwv_vote_digest(ctx: *mut NwvCtx, v: *const NwvVote, out: *mut u8) -> c_int;
    pub fn nwv_certificate_digest(ctx: *mut NwvCtx, c: *const NwvCertificate, out: *mut u8) -> c_int;
    pub fn nwv_header_digest_many(ctx: *mut NwvCtx, n: usize, h: *const NwvHeader, out: *mut u8) -> c_int;
    pub fn nwv_vote_digest_many(ctx: *mut NwvCtx, n: usize, v: *const NwvVote, out: *mut u8) -> c_int;
    pub fn nwv_certificate_digest_many(
        ctx: *mut NwvCtx,
        n: usize,
        c: *const NwvCertificate,
        out: *mut u8,
    ) -> c_int;
    pub fn nwv_header_verify(ctx: *mut NwvCtx, committee: *const NwvCommittee, h: *const NwvHeader) -> c_int;
    pub fn nwv_vote_verify(ctx: *mut NwvCtx, committee: *const NwvCommittee, v: *const NwvVote) -> c_int;
    pub fn nwv_certificate_verify(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        c: *const NwvCertificate,
    ) -> c_int;
    pub fn nwv_header_verify_many(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        n: usize,
        h: *const NwvHeader,
        results: *mut i32,
    ) -> c_int;
    pub fn nwv_vote_verify_many(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        n: usize,
        v: *const NwvVote,
        results: *mut i32,
    ) -> c_int;
    pub fn nwv_certificate_verify_many(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        n: usize,
        c: *const NwvCertificate,
        results: *mut i32,
    ) -> c_int;
    pub fn nwv_verify_mixed_many(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        n_headers: usize,
        headers: *const NwvHeader,
        header_results: *mut i32,
        n_votes: usize,
        votes: *const NwvVote,
        vote_results: *mut i32,
        n_certs: usize,
        certs: *const NwvCertificate,
        cert_results: *mut i32,
    ) -> c_int;
    pub fn nwv_validate_certificates(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        n: usize,
        c: *const NwvCertificate,
        n_invalid: *mut usize,
        invalid_idx: *mut usize,
    ) -> c_int;
    pub fn nwv_certificate_new(
        committee: *const NwvCommittee,
        n_votes: usize,
        vote_pks: *const u8,
        vote_sigs: *const u8,
        check_stake: c_int,
        signed_out: *mut u32,
        n_signed: *mut usize,
        sigs_out: *mut u8,
        n_sigs: *mut usize,
    ) -> c_int;
    pub fn nwv_committee_quorum_threshold(committee: *const NwvCommittee) -> u64;
    // ---- the types layer under BLS12-381 (include/nwv_types.h)
    pub fn nwv_bls_header_digest_many(ctx: *mut NwvCtx, n: usize, h: *const NwvBlsHeader, out: *mut u8) -> c_int;
    pub fn nwv_bls_vote_digest_many(ctx: *mut NwvCtx, n: usize, v: *const NwvBlsVote, out: *mut u8) -> c_int;
    pub fn nwv_bls_certificate_digest_many(
        ctx: *mut NwvCtx,
        n: usize,
        c: *const NwvBlsCertificate,
        out: *mut u8,
    ) -> c_int;
    pub fn nwv_bls_verify_mixed_many(
        ctx: *mut NwvCtx,
        committee: *const NwvBlsCommittee,
        n_headers: usize,
        headers: *const NwvBlsHeader,
        header_results: *mut i32,
        n_votes: usize,
        votes: *const NwvBlsVote,
        vote_results: *mut i32,
        n_certs: usize,
        certs: *const NwvBlsCertificate,
        cert_results: *mut i32,
    ) -> c_int;
    pub fn nwv_bls_validate_certificates(
        ctx: *mut NwvCtx,
        committee: *const NwvBlsCommittee,
        n: usize,
        c: *const NwvBlsCertificate,
        n_invalid: *mut usize,
        invalid_idx: *mut usize,
    ) -> c_int;
    pub fn nwv_bls_certificate_new(
        ctx: *mut NwvCtx,
        committee: *const NwvBlsCommittee,
        n_votes: usize,
        vote_pks: *const u8,
        vote_sigs: *const u8,
        check_stake: c_int,
        signed_out: *mut u32,
        n_signed: *mut usize,
        agg_out: *mut u8,
        has_agg: *mut c_int,
    ) -> c_int;
    // ---- batching service in front of Core::sanitize_* (include/nwv_service.h)
    pub fn nwv_service_create(
        ctx: *mut NwvCtx,
        committee: *const NwvCommittee,
        max_batch: usize,
        max_wait_us: u32,
        out: *mut *mut NwvService,
    ) -> c_int;
    pub fn nwv_service_set_committee(svc: *mut NwvService, committee: *const NwvCommittee) -> c_int;
    pub fn nwv_service_submit_header(
        svc: *mut NwvService,
        h: *const NwvHeader,
        done: NwvDoneFn,
        user: *mut c_void,
    ) -> c_int;
    pub fn nwv_service_submit_vote(
        svc: *mut NwvService,
        v: *const NwvVote,
        done: NwvDoneFn,
        user: *mut c_void,
    ) -> c_int;
    pub fn nwv_service_submit_certificate(
        svc: *mut NwvService,
        c: *const NwvCertificate,
        done: NwvDoneFn,
        user: *mut c_void,
    ) -> c_int;
    pub fn nwv_service_verify_header(svc: *mut NwvService, h: *const NwvHeader, result: *mut i32) -> c_int;
    pub fn nwv_service_verify_vote(svc: *mut NwvService, v: *const NwvVote, result: *mut i32) -> c_int;
    pub fn nwv_service_verify_certificate(
        svc: *mut NwvService,
        c: *const NwvCertificate,
        result: *mut i32,
    ) -> c_int;
    // the same service over a BLS12-381 committee (nwv_bls_verify_mixed_many per flush)
    pub fn nwv_service_create_bls(
        ctx: *mut NwvCtx,
        committee: *const NwvBlsCommittee,
        max_batch: usize,
        max_wait_us: u32,
        out: *mut *mut NwvService,
    ) -> c_int;
    pub fn nwv_service_set_committee_bls(svc: *mut NwvService, committee: *const NwvBlsCommittee) -> c_int;
    pub fn nwv_service_submit_bls_header(
        svc: *mut NwvService,
        h: *const NwvBlsHeader,
        done: NwvDoneFn,
        user: *mut c_void,
    ) -> c_int;
    pub fn nwv_service_submit_bls_vote(
        svc: *mut NwvService,
        v: *const NwvBlsVote,
        done: NwvDoneFn,
        user: *mut c_void,
    ) -> c_int;
    pub fn nwv_service_submit_bls_certificate(
        svc: *mut NwvService,
        c: *const NwvBlsCertificate,
        done: NwvDoneFn,
        user: *mut c_void,
    ) -> c_int;
    pub fn nwv_service_verify_bls_header(svc: *mut NwvService, h: *const NwvBlsHeader, result: *mut i32) -> c_int;
    pub fn nwv_service_verify_bls_vote(svc: *mut NwvService, v: *const NwvBlsVote, result: *mut i32) -> c_int;
    pub fn nwv_service_verify_bls_certificate(
        svc: *mut NwvService,
        c: *const NwvBlsCertificate,
        result: *mut i32,
    ) -> c_int;
    pub fn nwv_service_set_idle(svc: *mut NwvService, idle_us: u32) -> c_int;
    pub fn nwv_service_flush(svc: *mut NwvService) -> c_int;
    pub fn nwv_service_stats(svc: *mut NwvService, out: *mut u64) -> c_int;
    pub fn nwv_service_free(svc: *mut NwvService);
}
