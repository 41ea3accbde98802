//! GPU-backed BLS12-381 (min_sig) scheme module: the reference's DEFAULT signature scheme
//! (`crypto/src/lib.rs:29-33` aliases fastcrypto 0.1.2 `bls12381::*`, blst 0.3.10 underneath).
//! Keys, signing, aggregation bookkeeping, serde and base64 stay fastcrypto's, so the wire format
//! is unchanged; every *verification* runs on the MI355X engine (`include/nwv_bls.h`):
//!
//! ```ignore
//! pub type PublicKey = narwhal_gpu_crypto::bls::GpuBls12381PublicKey;
//! pub type Signature = narwhal_gpu_crypto::bls::GpuBls12381Signature;
//! pub type AggregateSignature = narwhal_gpu_crypto::bls::GpuBls12381AggregateSignature;
//! pub type PrivateKey = narwhal_gpu_crypto::bls::GpuBls12381PrivateKey;
//! pub type KeyPair = narwhal_gpu_crypto::bls::GpuBls12381KeyPair;
//! ```
//!
//! Verdicts are blst's `fast_aggregate_verify` (decode, subgroup checks, key sum, hash to G1 under
//! fastcrypto's DST, the pairing equation), checked against the engine's oracle and the
//! reference's own BLS key fixtures in `tests/`.  Errors follow the reference: any failed check is
//! the opaque `signature::Error::new()`; `verify_batch_empty_fail` returns the two fixed messages
//! of `crypto/src/bls12377/mod.rs:274-281`; an engine failure is never reported as valid.

use std::fmt::{self, Display};
use std::str::FromStr;

use eyre::eyre;
use fastcrypto::bls12381::{
    BLS12381AggregateSignature, BLS12381KeyPair, BLS12381PrivateKey, BLS12381PublicKey, BLS12381Signature,
};
use fastcrypto::traits::{
    AggregateAuthenticator, Authenticator, EncodeDecodeBase64, KeyPair, SigningKey, ToFromBytes, VerifyingKey,
};
use serde::{Deserialize, Serialize};
use signature::{Signer, Verifier};

use crate::{ctx, ffi, flat, last_error, sig_result};

pub const BLS_PUBLIC_KEY_LENGTH: usize = 96;
pub const BLS_SIGNATURE_LENGTH: usize = 48;

// -------------------------------------------------------------------------- signature --
#[derive(Debug, Clone, PartialEq, Eq, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuBls12381Signature(pub BLS12381Signature);

impl signature::Signature for GpuBls12381Signature {
    fn from_bytes(bytes: &[u8]) -> Result<Self, signature::Error> {
        <BLS12381Signature as signature::Signature>::from_bytes(bytes).map(GpuBls12381Signature)
    }
}
impl AsRef<[u8]> for GpuBls12381Signature {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl Default for GpuBls12381Signature {
    fn default() -> Self {
        GpuBls12381Signature(BLS12381Signature::default())
    }
}
impl Display for GpuBls12381Signature {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> Result<(), fmt::Error> {
        write!(f, "{}", self.0)
    }
}
impl std::hash::Hash for GpuBls12381Signature {
    fn hash<H: std::hash::Hasher>(&self, state: &mut H) {
        self.as_ref().hash(state);
    }
}
impl Authenticator for GpuBls12381Signature {
    type PubKey = GpuBls12381PublicKey;
    type PrivKey = GpuBls12381PrivateKey;
    const LENGTH: usize = BLS_SIGNATURE_LENGTH;
}

// ------------------------------------------------------------------------- public key --
#[derive(Debug, Clone, PartialEq, Eq, Hash, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuBls12381PublicKey(pub BLS12381PublicKey);

impl AsRef<[u8]> for GpuBls12381PublicKey {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl ToFromBytes for GpuBls12381PublicKey {
    fn from_bytes(bytes: &[u8]) -> Result<Self, signature::Error> {
        BLS12381PublicKey::from_bytes(bytes).map(GpuBls12381PublicKey)
    }
}
impl Default for GpuBls12381PublicKey {
    fn default() -> Self {
        GpuBls12381PublicKey(BLS12381PublicKey::default())
    }
}
impl Display for GpuBls12381PublicKey {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> Result<(), fmt::Error> {
        write!(f, "{}", self.0)
    }
}
// committee order: by key bytes (config/src/lib.rs:488-491)
impl PartialOrd for GpuBls12381PublicKey {
    fn partial_cmp(&self, other: &Self) -> Option<std::cmp::Ordering> {
        Some(self.cmp(other))
    }
}
impl Ord for GpuBls12381PublicKey {
    fn cmp(&self, other: &Self) -> std::cmp::Ordering {
        self.as_ref().cmp(other.as_ref())
    }
}
impl<'a> From<&'a GpuBls12381PrivateKey> for GpuBls12381PublicKey {
    fn from(secret: &'a GpuBls12381PrivateKey) -> Self {
        GpuBls12381PublicKey(BLS12381PublicKey::from(&secret.0))
    }
}

/// `Header::verify` (types/src/primary.rs:179-182) and `Vote::verify` (:325-327): one
/// fast_aggregate_verify with one key, on the GPU.
impl Verifier<GpuBls12381Signature> for GpuBls12381PublicKey {
    fn verify(&self, msg: &[u8], sig: &GpuBls12381Signature) -> Result<(), signature::Error> {
        let rc = unsafe {
            ffi::nwv_bls_verify(ctx(), self.as_ref().as_ptr(), msg.as_ptr(), msg.len(), sig.as_ref().as_ptr())
        };
        sig_result(rc)
    }
}

impl VerifyingKey for GpuBls12381PublicKey {
    type PrivKey = GpuBls12381PrivateKey;
    type Sig = GpuBls12381Signature;
    const LENGTH: usize = BLS_PUBLIC_KEY_LENGTH;

    /// crypto/src/bls12377/mod.rs:269-290: empty -> Err, |pks| != |sigs| -> Err, both before any
    /// crypto; then the signatures' sum verified against the keys' sum.
    fn verify_batch_empty_fail(msg: &[u8], pks: &[Self], sigs: &[Self::Sig]) -> Result<(), eyre::Report> {
        if sigs.is_empty() {
            return Err(eyre!("Critical Error! This behavious can signal something dangerous, and that someone may be trying to bypass signature verification through providing empty batches."));
        }
        if sigs.len() != pks.len() {
            return Err(eyre!("Mismatch between number of signatures and public keys provided"));
        }
        let pk = flat(pks);
        let sg = flat(sigs);
        let rc = unsafe {
            ffi::nwv_bls_verify_batch_empty_fail(
                ctx(), msg.as_ptr(), msg.len(), pk.as_ptr(), pks.len(), sg.as_ptr(), sigs.len(),
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
pub struct GpuBls12381PrivateKey(pub BLS12381PrivateKey);

impl AsRef<[u8]> for GpuBls12381PrivateKey {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl ToFromBytes for GpuBls12381PrivateKey {
    fn from_bytes(bytes: &[u8]) -> Result<Self, signature::Error> {
        BLS12381PrivateKey::from_bytes(bytes).map(GpuBls12381PrivateKey)
    }
}
impl PartialEq for GpuBls12381PrivateKey {
    fn eq(&self, other: &Self) -> bool {
        self.as_ref() == other.as_ref()
    }
}
impl Eq for GpuBls12381PrivateKey {}
impl SigningKey for GpuBls12381PrivateKey {
    type PubKey = GpuBls12381PublicKey;
    type Sig = GpuBls12381Signature;
    const LENGTH: usize = 32;
}
/// Signing stays on the CPU, as in the reference (SignatureService, primary/src/primary.rs:256).
impl Signer<GpuBls12381Signature> for GpuBls12381PrivateKey {
    fn try_sign(&self, msg: &[u8]) -> Result<GpuBls12381Signature, signature::Error> {
        self.0.try_sign(msg).map(GpuBls12381Signature)
    }
}

// --------------------------------------------------------------------------- key pair --
#[derive(Debug, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuBls12381KeyPair(pub BLS12381KeyPair);

impl From<GpuBls12381PrivateKey> for GpuBls12381KeyPair {
    fn from(secret: GpuBls12381PrivateKey) -> Self {
        GpuBls12381KeyPair(BLS12381KeyPair::from(secret.0))
    }
}
impl EncodeDecodeBase64 for GpuBls12381KeyPair {
    fn encode_base64(&self) -> String {
        self.0.encode_base64()
    }
    fn decode_base64(value: &str) -> Result<Self, eyre::Report> {
        BLS12381KeyPair::decode_base64(value).map(GpuBls12381KeyPair)
    }
}
impl FromStr for GpuBls12381KeyPair {
    type Err = eyre::Report;
    fn from_str(s: &str) -> Result<Self, Self::Err> {
        Self::decode_base64(s)
    }
}
impl Signer<GpuBls12381Signature> for GpuBls12381KeyPair {
    fn try_sign(&self, msg: &[u8]) -> Result<GpuBls12381Signature, signature::Error> {
        self.0.try_sign(msg).map(GpuBls12381Signature)
    }
}
impl KeyPair for GpuBls12381KeyPair {
    type PubKey = GpuBls12381PublicKey;
    type PrivKey = GpuBls12381PrivateKey;
    type Sig = GpuBls12381Signature;

    fn public(&'_ self) -> &'_ Self::PubKey {
        // #[repr(transparent)] over fastcrypto's key: same layout, so the reference cast is sound
        let pk: &BLS12381PublicKey = self.0.public();
        unsafe { &*(pk as *const BLS12381PublicKey as *const GpuBls12381PublicKey) }
    }
    fn private(self) -> Self::PrivKey {
        GpuBls12381PrivateKey(self.0.private())
    }
    fn copy(&self) -> Self {
        GpuBls12381KeyPair(self.0.copy())
    }
    fn generate<R: rand::CryptoRng + rand::RngCore>(rng: &mut R) -> Self {
        GpuBls12381KeyPair(BLS12381KeyPair::generate(rng))
    }
}

// --------------------------------------------------------------- aggregate signature --
/// A certificate's aggregate (Certificate::new_unsafe, types/src/primary.rs:427-485): fastcrypto's
/// own type (the sum of the votes' G1 signatures, `None` when empty), so it serializes as before;
/// verification on the GPU.
#[derive(Debug, Clone, Default, PartialEq, Eq, Serialize, Deserialize)]
#[serde(transparent)]
#[repr(transparent)]
pub struct GpuBls12381AggregateSignature(pub BLS12381AggregateSignature);

impl AsRef<[u8]> for GpuBls12381AggregateSignature {
    fn as_ref(&self) -> &[u8] {
        self.0.as_ref()
    }
}
impl Display for GpuBls12381AggregateSignature {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> Result<(), fmt::Error> {
        write!(f, "{}", self.0)
    }
}

impl GpuBls12381AggregateSignature {
    /// the 48-byte aggregate, or None for an aggregate holding no signature
    fn bytes48(&self) -> Option<&[u8]> {
        let b = self.as_ref();
        if b.len() == BLS_SIGNATURE_LENGTH {
            Some(b)
        } else {
            None
        }
    }
}

impl AggregateAuthenticator for GpuBls12381AggregateSignature {
    type Sig = GpuBls12381Signature;
    type PubKey = GpuBls12381PublicKey;
    type PrivKey = GpuBls12381PrivateKey;

    fn aggregate(signatures: Vec<Self::Sig>) -> Result<Self, signature::Error> {
        BLS12381AggregateSignature::aggregate(signatures.into_iter().map(|s| s.0).collect())
            .map(GpuBls12381AggregateSignature)
    }
    fn add_signature(&mut self, signature: Self::Sig) -> Result<(), signature::Error> {
        self.0.add_signature(signature.0)
    }
    fn add_aggregate(&mut self, signature: Self) -> Result<(), signature::Error> {
        self.0.add_aggregate(signature.0)
    }
    /// Certificate::verify (types/src/primary.rs:531-534): fast_aggregate_verify on the GPU
    fn verify(&self, pks: &[<Self::Sig as Authenticator>::PubKey], message: &[u8]) -> Result<(), signature::Error> {
        let sig = match self.bytes48() {
            Some(b) => b.as_ptr(),
            None => std::ptr::null(),
        };
        let pk = flat(pks);
        let rc = unsafe { ffi::nwv_bls_aggregate_verify(ctx(), sig, pk.as_ptr(), pks.len(), message.as_ptr(), message.len()) };
        sig_result(rc)
    }
    /// crypto/src/bls12377/mod.rs:548-576: every length mismatch -> Err; all the aggregates in
    /// ONE engine call (one batch pairing check over the call's items)
    fn batch_verify<'a>(
        signatures: &[&Self],
        pks: Vec<impl Iterator<Item = &'a Self::PubKey>>,
        messages: &[&[u8]],
    ) -> Result<(), signature::Error> {
        if pks.len() != messages.len() || messages.len() != signatures.len() {
            return Err(signature::Error::new());
        }
        let keys: Vec<Vec<u8>> = pks.into_iter().map(|it| flat(it.collect::<Vec<_>>())).collect();
        let n_pks: Vec<usize> = keys.iter().map(|k| k.len() / BLS_PUBLIC_KEY_LENGTH).collect();
        let kp: Vec<*const u8> = keys.iter().map(|k| k.as_ptr()).collect();
        let mut sp: Vec<*const u8> = Vec::with_capacity(signatures.len());
        for s in signatures {
            match s.bytes48() {
                Some(b) => sp.push(b.as_ptr()),
                None => return Err(signature::Error::new()), // an aggregate holding no signature
            }
        }
        let mp: Vec<*const u8> = messages.iter().map(|m| m.as_ptr()).collect();
        let ml: Vec<usize> = messages.iter().map(|m| m.len()).collect();
        let rc = unsafe {
            ffi::nwv_bls_aggregate_batch_verify(
                ctx(), signatures.len(), sp.as_ptr(), kp.as_ptr(), n_pks.as_ptr(), mp.as_ptr(), ml.as_ptr(),
                messages.len(),
            )
        };
        sig_result(rc)
    }
}

/// `CertificatesResponse::validate_certificates` (primary/src/block_synchronizer/responses.rs
/// :95-141) for BLS certificates: per-item statuses (`include/nwv_bls.h` NWV_BLS_*) of many
/// fast_aggregate_verify items over one key table (the committee) in ONE engine call.  item i:
/// aggregate `sigs[i]` over `msgs[i]` by the keys `keys[key_lists[i][..]]`.
pub fn verify_many(
    keys: &[GpuBls12381PublicKey],
    sigs: &[[u8; BLS_SIGNATURE_LENGTH]],
    key_lists: &[&[u32]],
    msgs: &[&[u8]],
) -> Result<Vec<i32>, String> {
    let n = sigs.len();
    if key_lists.len() != n || msgs.len() != n {
        return Err("length mismatch".into());
    }
    let kb = flat(keys);
    let mut off = Vec::with_capacity(n);
    let mut cnt = Vec::with_capacity(n);
    let mut idx: Vec<u32> = Vec::new();
    let mut mb: Vec<u8> = Vec::new();
    let mut moff = Vec::with_capacity(n);
    let mut mlen = Vec::with_capacity(n);
    for i in 0..n {
        off.push(idx.len() as u32);
        cnt.push(key_lists[i].len() as u32);
        idx.extend_from_slice(key_lists[i]);
        moff.push(mb.len() as u64);
        mlen.push(msgs[i].len() as u32);
        mb.extend_from_slice(msgs[i]);
    }
    mb.push(0);
    idx.push(0);
    let mut status = vec![0i32; n];
    let rc = unsafe {
        ffi::nwv_bls_verify_many(
            ctx(), keys.len(), kb.as_ptr(), n, sigs.as_ptr() as *const u8, off.as_ptr(), cnt.as_ptr(), idx.as_ptr(),
            mb.as_ptr(), moff.as_ptr(), mlen.as_ptr(), std::ptr::null(), 0, status.as_mut_ptr(),
        )
    };
    if rc == ffi::NWV_OK {
        Ok(status)
    } else {
        Err(last_error())
    }
}
