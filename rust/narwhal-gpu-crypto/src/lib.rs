//! GPU-backed Ed25519 scheme module for Narwhal's `crypto` crate.
//!
//! The reference selects its signature scheme with five type aliases
//! (`crypto/src/lib.rs:29-33`; swap rule `:19-27`); `crypto/src/bls12377/mod.rs:93-577` is the
//! in-tree template of a module implementing the fastcrypto 0.1.2 traits.  This module is that
//! template for Ed25519 with every *verification* routed to the MI355X engine (`libnwv`, C ABI in
//! `include/nwv.h`): keys, signing, serde and base64 stay fastcrypto's (`fastcrypto::ed25519`),
//! so the wire format is unchanged.  Swap the aliases to:
//!
//! ```ignore
//! pub type PublicKey = narwhal_gpu_crypto::GpuEd25519PublicKey;
//! pub type Signature = narwhal_gpu_crypto::GpuEd25519Signature;
//! pub type AggregateSignature = narwhal_gpu_crypto::GpuEd25519AggregateSignature;
//! pub type PrivateKey = narwhal_gpu_crypto::GpuEd25519PrivateKey;
//! pub type KeyPair = narwhal_gpu_crypto::GpuEd25519KeyPair;
//! ```
//!
//! Verdicts are ed25519-consensus 2.0.1 / ZIP-215 (the reference's Ed25519 backend,
//! `Cargo.lock:1428`), checked bit-exact against the engine's oracle in `tests/`.  Error
//! behaviour follows the reference: any failed check is the opaque `signature::Error::new()`
//! (`types/src/error.rs:154-155` maps it to `DagError::InvalidSignature`), length mismatches are
//! rejected before any crypto, and `verify_batch_empty_fail` returns the two fixed messages of
//! `crypto/src/bls12377/mod.rs:274-281`.  A runtime failure of the engine (no device, HIP error)
//! is never reported as valid.

pub mod bls;
pub mod core_drain;
pub mod ffi;

use std::ffi::CStr;
use std::fmt::{self, Display};
use std::str::FromStr;

use base64ct::{Base64, Encoding};
use eyre::eyre;
use fastcrypto::ed25519::{Ed25519KeyPair, Ed25519PrivateKey, Ed25519PublicKey, Ed25519Signature};
use fastcrypto::traits::{
    AggregateAuthenticator, Authenticator, EncodeDecodeBase64, KeyPair, SigningKey, ToFromBytes, VerifyingKey,
};
use once_cell::sync::{Lazy, OnceCell};
use rand::RngCore;
use serde::{Deserialize, Serialize};
use signature::{Signer, Verifier};

pub const PUBLIC_KEY_LENGTH: usize = 32;
pub const SIGNATURE_LENGTH: usize = 64;

// ------------------------------------------------------------------------- the engine --
/// Process-wide engine context over every visible gfx950 device, created on first use (the role
/// `Primary::spawn` plays for long-lived state).  The library is thread-safe
/// (a pool of lanes per device), so one context serves every tokio task.
struct Ctx(*mut ffi::NwvCtx);
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

static CTX: Lazy<Ctx> = Lazy::new(|| {
    let mut p = std::ptr::null_mut();
    let rc = unsafe { ffi::nwv_init(&mut p, 0, 0) };
    assert_eq!(rc, ffi::NWV_OK, "nwv_init failed: {}", last_error());
    Ctx(p)
});

fn ctx() -> *mut ffi::NwvCtx {
    CTX.0
}

/// Text of the calling thread's last engine error.
pub fn last_error() -> String {
    unsafe { CStr::from_ptr(ffi::nwv_last_error()) }.to_string_lossy().into_owned()
}

/// 32 bytes from the OS CSPRNG: the batch verifier's random coefficients (ed25519-consensus
/// draws them from its thread RNG).
fn seed() -> [u8; 32] {
    let mut s = [0u8; 32];
    rand::rngs::OsRng.fill_bytes(&mut s);
    s
}

fn sig_result(rc: i32) -> Result<(), signature::Error> {
    if rc == ffi::NWV_OK {
        Ok(())
    } else {
        Err(signature::Error::new())
    }
}

fn flat<'a, T: AsRef<[u8]> + 'a>(items: impl IntoIterator<Item = &'a T>) -> Vec<u8> {
    let mut v = Vec::new();
    for it in items {
        v.extend_from_slice(it.as_ref());
    }
    v
}

// -------------------------------------------------------------------------- signature --
#[derive(Debug, Clone, PartialEq, Eq, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuEd25519Signature(pub Ed25519Signature);

impl signature::Signature for GpuEd25519Signature {
    fn from_bytes(bytes: &[u8]) -> Result<Self, signature::Error> {
        <Ed25519Signature as signature::Signature>::from_bytes(bytes).map(GpuEd25519Signature)
    }
}
impl AsRef<[u8]> for GpuEd25519Signature {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl Default for GpuEd25519Signature {
    fn default() -> Self {
        GpuEd25519Signature(Ed25519Signature::default())
    }
}
impl Display for GpuEd25519Signature {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> Result<(), fmt::Error> {
        write!(f, "{}", Base64::encode_string(self.as_ref()))
    }
}
impl std::hash::Hash for GpuEd25519Signature {
    fn hash<H: std::hash::Hasher>(&self, state: &mut H) {
        self.as_ref().hash(state);
    }
}
impl Authenticator for GpuEd25519Signature {
    type PubKey = GpuEd25519PublicKey;
    type PrivKey = GpuEd25519PrivateKey;
    const LENGTH: usize = SIGNATURE_LENGTH;
}

// ------------------------------------------------------------------------- public key --
#[derive(Debug, Clone, PartialEq, Eq, Hash, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuEd25519PublicKey(pub Ed25519PublicKey);

impl AsRef<[u8]> for GpuEd25519PublicKey {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl ToFromBytes for GpuEd25519PublicKey {
    fn from_bytes(bytes: &[u8]) -> Result<Self, signature::Error> {
        Ed25519PublicKey::from_bytes(bytes).map(GpuEd25519PublicKey)
    }
}
impl Default for GpuEd25519PublicKey {
    fn default() -> Self {
        GpuEd25519PublicKey(Ed25519PublicKey::default())
    }
}
impl Display for GpuEd25519PublicKey {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> Result<(), fmt::Error> {
        write!(f, "{}", Base64::encode_string(self.as_ref()))
    }
}
// Committee keys are a BTreeMap ordered by key bytes (config/src/lib.rs:488-491): the bitmap
// index order of a certificate's signers.
impl PartialOrd for GpuEd25519PublicKey {
    fn partial_cmp(&self, other: &Self) -> Option<std::cmp::Ordering> {
        Some(self.cmp(other))
    }
}
impl Ord for GpuEd25519PublicKey {
    fn cmp(&self, other: &Self) -> std::cmp::Ordering {
        self.as_ref().cmp(other.as_ref())
    }
}
impl<'a> From<&'a GpuEd25519PrivateKey> for GpuEd25519PublicKey {
    fn from(secret: &'a GpuEd25519PrivateKey) -> Self {
        GpuEd25519PublicKey(Ed25519PublicKey::from(&secret.0))
    }
}

/// `Header::verify` (types/src/primary.rs:179-182) and `Vote::verify` (:325-327): one ZIP-215
/// verification on the GPU.
impl Verifier<GpuEd25519Signature> for GpuEd25519PublicKey {
    fn verify(&self, msg: &[u8], sig: &GpuEd25519Signature) -> Result<(), signature::Error> {
        let rc = unsafe {
            ffi::nwv_ed25519_pubkey_verify(ctx(), self.as_ref().as_ptr(), msg.as_ptr(), msg.len(), sig.as_ref().as_ptr())
        };
        sig_result(rc)
    }
}

impl VerifyingKey for GpuEd25519PublicKey {
    type PrivKey = GpuEd25519PrivateKey;
    type Sig = GpuEd25519Signature;
    const LENGTH: usize = PUBLIC_KEY_LENGTH;

    /// Contract of crypto/src/bls12377/mod.rs:269-290: empty -> Err, |pks| != |sigs| -> Err,
    /// both before any crypto, then one batch verification over the shared message.
    fn verify_batch_empty_fail(msg: &[u8], pks: &[Self], sigs: &[Self::Sig]) -> Result<(), eyre::Report> {
        if sigs.is_empty() {
            return Err(eyre!("Critical Error! This behavious can signal something dangerous, and that someone may be trying to bypass signature verification through providing empty batches."));
        }
        if sigs.len() != pks.len() {
            return Err(eyre!("Mismatch between number of signatures and public keys provided"));
        }
        let pk = flat(pks);
        let sg = flat(sigs);
        let s = seed();
        let rc = unsafe {
            ffi::nwv_ed25519_verify_batch_empty_fail(
                ctx(), msg.as_ptr(), msg.len(), pk.as_ptr(), pks.len(), sg.as_ptr(), sigs.len(), s.as_ptr(),
            )
        };
        match rc {
            ffi::NWV_OK => Ok(()),
            ffi::NWV_ERR_SIGNATURE => Err(eyre!("Signature verification failed")),
            _ => Err(eyre!("GPU verification error: {}", last_error())),
        }
    }
}

// ------------------------------------------------------------------------ private key --
#[derive(Debug, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuEd25519PrivateKey(pub Ed25519PrivateKey);

impl AsRef<[u8]> for GpuEd25519PrivateKey {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl ToFromBytes for GpuEd25519PrivateKey {
    fn from_bytes(bytes: &[u8]) -> Result<Self, signature::Error> {
        Ed25519PrivateKey::from_bytes(bytes).map(GpuEd25519PrivateKey)
    }
}
impl PartialEq for GpuEd25519PrivateKey {
    fn eq(&self, other: &Self) -> bool {
        self.as_ref() == other.as_ref()
    }
}
impl Eq for GpuEd25519PrivateKey {}
impl SigningKey for GpuEd25519PrivateKey {
    type PubKey = GpuEd25519PublicKey;
    type Sig = GpuEd25519Signature;
    const LENGTH: usize = 32;
}
/// Signing stays on the CPU, as in the reference (SignatureService, primary/src/primary.rs:256).
impl Signer<GpuEd25519Signature> for GpuEd25519PrivateKey {
    fn try_sign(&self, msg: &[u8]) -> Result<GpuEd25519Signature, signature::Error> {
        self.0.try_sign(msg).map(GpuEd25519Signature)
    }
}

// --------------------------------------------------------------------------- key pair --
#[derive(Debug, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuEd25519KeyPair(pub Ed25519KeyPair);

impl From<GpuEd25519PrivateKey> for GpuEd25519KeyPair {
    fn from(secret: GpuEd25519PrivateKey) -> Self {
        GpuEd25519KeyPair(Ed25519KeyPair::from(secret.0))
    }
}
impl EncodeDecodeBase64 for GpuEd25519KeyPair {
    fn encode_base64(&self) -> String {
        self.0.encode_base64()
    }
    fn decode_base64(value: &str) -> Result<Self, eyre::Report> {
        Ed25519KeyPair::decode_base64(value).map(GpuEd25519KeyPair)
    }
}
impl FromStr for GpuEd25519KeyPair {
    type Err = eyre::Report;
    fn from_str(s: &str) -> Result<Self, Self::Err> {
        Self::decode_base64(s)
    }
}
impl Signer<GpuEd25519Signature> for GpuEd25519KeyPair {
    fn try_sign(&self, msg: &[u8]) -> Result<GpuEd25519Signature, signature::Error> {
        self.0.try_sign(msg).map(GpuEd25519Signature)
    }
}
impl KeyPair for GpuEd25519KeyPair {
    type PubKey = GpuEd25519PublicKey;
    type PrivKey = GpuEd25519PrivateKey;
    type Sig = GpuEd25519Signature;

    fn public(&'_ self) -> &'_ Self::PubKey {
        // GpuEd25519PublicKey is #[repr(transparent)] over fastcrypto's key: same layout, so the
        // reference cast is sound
        let pk: &Ed25519PublicKey = self.0.public();
        unsafe { &*(pk as *const Ed25519PublicKey as *const GpuEd25519PublicKey) }
    }
    fn private(self) -> Self::PrivKey {
        GpuEd25519PrivateKey(self.0.private())
    }
    fn copy(&self) -> Self {
        GpuEd25519KeyPair(self.0.copy())
    }
    fn generate<R: rand::CryptoRng + rand::RngCore>(rng: &mut R) -> Self {
        GpuEd25519KeyPair(Ed25519KeyPair::generate(rng))
    }
}

// --------------------------------------------------------------- aggregate signature --
/// The Ed25519 aggregate of a certificate is the list of its signers' signatures in committee
/// order (Certificate::new_unsafe, types/src/primary.rs:427-485); verifying it is one batch
/// verification of Q signatures over the certificate digest (:531-534).
#[derive(Debug, Clone, Default, PartialEq, Eq, Serialize, Deserialize)]
pub struct GpuEd25519AggregateSignature {
    pub sigs: Vec<GpuEd25519Signature>,
    #[serde(skip)]
    bytes: OnceCell<Vec<u8>>,
}

impl AsRef<[u8]> for GpuEd25519AggregateSignature {
    fn as_ref(&self) -> &[u8] {
        self.bytes.get_or_init(|| flat(&self.sigs))
    }
}
impl Display for GpuEd25519AggregateSignature {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> Result<(), fmt::Error> {
        write!(f, "{}", Base64::encode_string(self.as_ref()))
    }
}

impl AggregateAuthenticator for GpuEd25519AggregateSignature {
    type Sig = GpuEd25519Signature;
    type PubKey = GpuEd25519PublicKey;
    type PrivKey = GpuEd25519PrivateKey;

    fn aggregate(signatures: Vec<Self::Sig>) -> Result<Self, signature::Error> {
        Ok(GpuEd25519AggregateSignature { sigs: signatures, bytes: OnceCell::new() })
    }
    fn add_signature(&mut self, signature: Self::Sig) -> Result<(), signature::Error> {
        self.sigs.push(signature);
        self.bytes = OnceCell::new();
        Ok(())
    }
    fn add_aggregate(&mut self, mut signature: Self) -> Result<(), signature::Error> {
        self.sigs.append(&mut signature.sigs);
        self.bytes = OnceCell::new();
        Ok(())
    }
    /// |pks| != |sigs| -> Err before any crypto; else one batch MSM on the GPU.
    fn verify(&self, pks: &[<Self::Sig as Authenticator>::PubKey], message: &[u8]) -> Result<(), signature::Error> {
        let pk = flat(pks);
        let sg = flat(&self.sigs);
        let s = seed();
        let rc = unsafe {
            ffi::nwv_ed25519_aggregate_verify(
                ctx(), sg.as_ptr(), self.sigs.len(), pk.as_ptr(), pks.len(), message.as_ptr(), message.len(), s.as_ptr(),
            )
        };
        sig_result(rc)
    }
    /// Contract of crypto/src/bls12377/mod.rs:548-576: every length mismatch -> Err; all the
    /// aggregates' signatures in ONE batch verification.
    fn batch_verify<'a>(
        signatures: &[&Self],
        pks: Vec<impl Iterator<Item = &'a Self::PubKey>>,
        messages: &[&[u8]],
    ) -> Result<(), signature::Error> {
        if pks.len() != messages.len() || messages.len() != signatures.len() {
            return Err(signature::Error::new());
        }
        let keys: Vec<Vec<u8>> = pks.into_iter().map(|it| flat(it.collect::<Vec<_>>())).collect();
        let sigs: Vec<Vec<u8>> = signatures.iter().map(|a| flat(&a.sigs)).collect();
        let n_pks: Vec<usize> = keys.iter().map(|k| k.len() / PUBLIC_KEY_LENGTH).collect();
        let n_sigs: Vec<usize> = signatures.iter().map(|a| a.sigs.len()).collect();
        let kp: Vec<*const u8> = keys.iter().map(|k| k.as_ptr()).collect();
        let sp: Vec<*const u8> = sigs.iter().map(|s| s.as_ptr()).collect();
        let mp: Vec<*const u8> = messages.iter().map(|m| m.as_ptr()).collect();
        let ml: Vec<usize> = messages.iter().map(|m| m.len()).collect();
        let s = seed();
        let rc = unsafe {
            ffi::nwv_ed25519_aggregate_batch_verify(
                ctx(), signatures.len(), sp.as_ptr(), n_sigs.as_ptr(), kp.as_ptr(), n_pks.as_ptr(), mp.as_ptr(),
                ml.as_ptr(), messages.len(), s.as_ptr(),
            )
        };
        sig_result(rc)
    }
}

// ------------------------------------------------------------------- worker digests --
/// `Batch::digest` (types/src/primary.rs:65-73) of many batches in one GPU call: `batches[i]` is
/// the concatenation of batch i's transactions.
pub fn blake2b256_many(batches: &[&[u8]]) -> Result<Vec<[u8; 32]>, String> {
    let mut base = Vec::new();
    let mut off = Vec::with_capacity(batches.len());
    let mut len = Vec::with_capacity(batches.len());
    for b in batches {
        off.push(base.len() as u64);
        len.push(b.len() as u64);
        base.extend_from_slice(b);
    }
    let mut out = vec![[0u8; 32]; batches.len()];
    let rc = unsafe {
        ffi::nwv_blake2b256_many(ctx(), batches.len(), base.as_ptr(), off.as_ptr(), len.as_ptr(), out.as_mut_ptr() as *mut u8)
    };
    if rc == ffi::NWV_OK {
        Ok(out)
    } else {
        Err(last_error())
    }
}

/// `serialized_batch_digest` (types/src/worker.rs:44-62) of bincode `WorkerMessage::Batch`
/// buffers: `Err(offset)` as `DigestError::InvalidArgumentError(offset)` for a malformed one.
pub fn serialized_batch_digests(bufs: &[&[u8]]) -> Vec<Result<[u8; 32], i64>> {
    let mut base = Vec::new();
    let mut off = Vec::with_capacity(bufs.len());
    let mut len = Vec::with_capacity(bufs.len());
    for b in bufs {
        off.push(base.len() as u64);
        len.push(b.len() as u64);
        base.extend_from_slice(b);
    }
    let mut out = vec![[0u8; 32]; bufs.len()];
    let mut err = vec![-1i64; bufs.len()];
    unsafe {
        ffi::nwv_batch_digest_serialized(
            ctx(), bufs.len(), base.as_ptr(), off.as_ptr(), len.as_ptr(), out.as_mut_ptr() as *mut u8, err.as_mut_ptr(),
        );
    }
    out.into_iter().zip(err).map(|(d, e)| if e < 0 { Ok(d) } else { Err(e) }).collect()
}

// ------------------------------------------------------------------------ types layer --
/// Codes of `include/nwv_types.h`: 0 or the DagError variant (types/src/error.rs) an item's
/// verify() returns.  The caller maps them to its `DagError` values.
pub type DagCode = i32;

/// Everything a Core loop iteration has queued (Core::sanitize_*, primary/src/core.rs:497-573),
/// verified in ONE call: one BLAKE2b launch for every digest, one batch MSM for every signature.
pub fn verify_mixed(
    committee: &ffi::NwvCommittee,
    headers: &[ffi::NwvHeader],
    votes: &[ffi::NwvVote],
    certs: &[ffi::NwvCertificate],
) -> Result<(Vec<DagCode>, Vec<DagCode>, Vec<DagCode>), String> {
    let mut rh = vec![0i32; headers.len()];
    let mut rv = vec![0i32; votes.len()];
    let mut rc = vec![0i32; certs.len()];
    let r = unsafe {
        ffi::nwv_verify_mixed_many(
            ctx(), committee, headers.len(), headers.as_ptr(), rh.as_mut_ptr(), votes.len(), votes.as_ptr(),
            rv.as_mut_ptr(), certs.len(), certs.as_ptr(), rc.as_mut_ptr(),
        )
    };
    if r == ffi::NWV_OK {
        Ok((rh, rv, rc))
    } else {
        Err(last_error())
    }
}

/// `CertificatesResponse::validate_certificates` (primary/src/block_synchronizer/responses.rs
/// :95-141): `Ok(())` or the exact indices of the invalid certificates.
pub fn validate_certificates(committee: &ffi::NwvCommittee, certs: &[ffi::NwvCertificate]) -> Result<(), Vec<usize>> {
    let mut n_invalid = 0usize;
    let mut idx = vec![0usize; certs.len()];
    let r = unsafe {
        ffi::nwv_validate_certificates(ctx(), committee, certs.len(), certs.as_ptr(), &mut n_invalid, idx.as_mut_ptr())
    };
    match r {
        ffi::NWV_OK => Ok(()),
        ffi::NWV_ERR_SIGNATURE => {
            idx.truncate(n_invalid);
            Err(idx)
        }
        // an engine failure is never "valid": every certificate is reported
        _ => Err((0..certs.len()).collect()),
    }
}

/// The batching service (include/nwv_service.h): many tasks call `verify_*` concurrently; the
/// library coalesces them into one engine call and hands each its own code.
pub struct VerificationService(*mut ffi::NwvService);
unsafe impl Send for VerificationService {}
unsafe impl Sync for VerificationService {}

impl VerificationService {
    pub fn new(committee: &ffi::NwvCommittee, max_batch: usize, max_wait_us: u32) -> Result<Self, String> {
        let mut p = std::ptr::null_mut();
        let rc = unsafe { ffi::nwv_service_create(ctx(), committee, max_batch, max_wait_us, &mut p) };
        if rc == ffi::NWV_OK {
            Ok(VerificationService(p))
        } else {
            Err(last_error())
        }
    }
    /// epoch change (Core::change_epoch, primary/src/core.rs:592-611)
    pub fn set_committee(&self, committee: &ffi::NwvCommittee) -> bool {
        unsafe { ffi::nwv_service_set_committee(self.0, committee) == ffi::NWV_OK }
    }
    /// burst flush: also flush once nothing was submitted for `idle_us` (0: off)
    pub fn set_idle(&self, idle_us: u32) -> bool {
        unsafe { ffi::nwv_service_set_idle(self.0, idle_us) == ffi::NWV_OK }
    }
    fn code(rc: i32, r: i32) -> Result<DagCode, String> {
        if rc == ffi::NWV_OK {
            Ok(r)
        } else {
            Err(last_error())
        }
    }
    /// blocking: call through `tokio::task::spawn_blocking` from async code
    pub fn verify_header(&self, h: &ffi::NwvHeader) -> Result<DagCode, String> {
        let mut r = 0i32;
        let rc = unsafe { ffi::nwv_service_verify_header(self.0, h, &mut r) };
        Self::code(rc, r)
    }
    pub fn verify_vote(&self, v: &ffi::NwvVote) -> Result<DagCode, String> {
        let mut r = 0i32;
        let rc = unsafe { ffi::nwv_service_verify_vote(self.0, v, &mut r) };
        Self::code(rc, r)
    }
    pub fn verify_certificate(&self, c: &ffi::NwvCertificate) -> Result<DagCode, String> {
        let mut r = 0i32;
        let rc = unsafe { ffi::nwv_service_verify_certificate(self.0, c, &mut r) };
        Self::code(rc, r)
    }
    pub fn flush(&self) {
        unsafe {
            ffi::nwv_service_flush(self.0);
        }
    }
}

impl Drop for VerificationService {
    fn drop(&mut self) {
        unsafe { ffi::nwv_service_free(self.0) }
    }
}
