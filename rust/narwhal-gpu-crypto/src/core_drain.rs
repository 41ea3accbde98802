//! Core-side coalescer: the primary's Core verifies one message at a time inside one tokio task
//! (`Core::run`, primary/src/core.rs:614-714, calling `sanitize_header` / `sanitize_vote` /
//! `sanitize_certificate` :497-573), so a per-message GPU call sees batches of 1 (header, vote) or
//! 1 + Q (certificate) signatures and pays a full batch latency for each.  Verification depends
//! only on the committee, never on Core's state, so the loop can verify ahead:
//!
//! ```ignore
//! Some(first) = self.rx_primaries.recv() => {
//!     let batch = core_drain::drain(&mut self.rx_primaries, first, &self.drain_policy).await;
//!     let views: Vec<_> = batch.iter().map(|m| m.as_item(&mut self.arena)).collect(); // C views
//!     let codes = core_drain::verify_items(&self.nwv_committee, &views)?;          // ONE GPU call
//!     for (message, code) in batch.into_iter().zip(codes) {
//!         // sanitize_*'s state checks (epoch, gc round, expected vote) exactly as before, then
//!         // the pre-computed verification verdict in place of header.verify(..) / vote.verify(..)
//!         // / certificate.verify(..), then process_* -- per message, in arrival order
//!     }
//! }
//! ```
//!
//! A drained batch is verified against the committee current at drain time; `sanitize_*` rejects
//! an item of another epoch (InvalidEpoch) before its verdict is consulted, so an epoch change
//! inside a batch changes no outcome.

use std::time::Duration;

use tokio::sync::mpsc::{error::TryRecvError, Receiver};

use crate::{ffi, last_error, DagCode};

/// When to stop draining: `max_items` messages taken; or the channel is empty and either
/// `min_items` are already taken and nothing more arrives within `idle` (zero: at once -- a burst
/// still arriving is taken whole, a batch with nothing behind it goes without waiting) or
/// `max_wait` has elapsed since the first message.
#[derive(Clone, Copy, Debug)]
pub struct DrainPolicy {
    pub max_items: usize,
    pub min_items: usize,
    pub max_wait: Duration,
    pub idle: Duration,
}

impl Default for DrainPolicy {
    /// 512 messages, 64, 1 ms, no idle wait: a 100-node round (100 headers, 100 certificates, 99
    /// votes) fits one flush, a burst of 64+ goes at once, and a trickle waits at most 1 ms (about
    /// two coalesced verifications of such a round).  `idle` of 50 us takes a fast burst whole
    /// (one call instead of two: 0.79 -> 0.69 ms a round from native threads) but costs the
    /// overlap with a slow producer
    fn default() -> Self {
        DrainPolicy { max_items: 512, min_items: 64, max_wait: Duration::from_micros(1000), idle: Duration::ZERO }
    }
}

/// `first` plus whatever `rx` already holds or receives before the deadline, at most
/// `policy.max_items` messages, in arrival order.  Never waits once the channel is closed.
pub async fn drain<T>(rx: &mut Receiver<T>, first: T, policy: &DrainPolicy) -> Vec<T> {
    let mut out = vec![first];
    let deadline = tokio::time::Instant::now() + policy.max_wait;
    while out.len() < policy.max_items {
        match rx.try_recv() {
            Ok(m) => out.push(m),
            Err(TryRecvError::Disconnected) => break,
            Err(TryRecvError::Empty) if out.len() >= policy.min_items && policy.idle.is_zero() => break,
            Err(TryRecvError::Empty) => {
                let mut until = deadline;
                if out.len() >= policy.min_items {
                    until = until.min(tokio::time::Instant::now() + policy.idle);
                }
                match tokio::time::timeout_at(until, rx.recv()).await {
                    Ok(Some(m)) => out.push(m),
                    Ok(None) | Err(_) => break, // closed, or the deadline / idle gap passed
                }
            }
        }
    }
    out
}

/// One message as the C views of its fields (`include/nwv_types.h`); the views borrow the
/// message's buffers, which must outlive the `verify_items` call.
#[derive(Clone, Copy)]
pub enum Item {
    Header(ffi::NwvHeader),
    Vote(ffi::NwvVote),
    Certificate(ffi::NwvCertificate),
}

/// Every item verified in ONE engine call (`nwv_verify_mixed_many`: one digest launch, one batch
/// MSM); the codes (0 = Ok, else the DagError variant of `include/nwv_types.h`) come back in the
/// items' order.  An engine failure is an `Err` -- never a valid verdict.
pub fn verify_items(committee: &ffi::NwvCommittee, items: &[Item]) -> Result<Vec<DagCode>, String> {
    let (mut hs, mut vs, mut cs) = (Vec::new(), Vec::new(), Vec::new());
    let (mut hi, mut vi, mut ci) = (Vec::new(), Vec::new(), Vec::new());
    for (i, it) in items.iter().enumerate() {
        match it {
            Item::Header(h) => {
                hs.push(*h);
                hi.push(i)
            }
            Item::Vote(v) => {
                vs.push(*v);
                vi.push(i)
            }
            Item::Certificate(c) => {
                cs.push(*c);
                ci.push(i)
            }
        }
    }
    let mut rh = vec![0i32; hs.len()];
    let mut rv = vec![0i32; vs.len()];
    let mut rc = vec![0i32; cs.len()];
    let r = unsafe {
        ffi::nwv_verify_mixed_many(
            crate::ctx(), committee, hs.len(), hs.as_ptr(), rh.as_mut_ptr(), vs.len(), vs.as_ptr(), rv.as_mut_ptr(),
            cs.len(), cs.as_ptr(), rc.as_mut_ptr(),
        )
    };
    if r != ffi::NWV_OK {
        return Err(last_error());
    }
    let mut codes = vec![0i32; items.len()];
    for (pos, res) in [(&hi, &rh), (&vi, &rv), (&ci, &rc)] {
        for (j, &i) in pos.iter().enumerate() {
            codes[i] = res[j];
        }
    }
    Ok(codes)
}

/// One message under BLS12-381, the reference's default scheme (`crypto/src/lib.rs:29-33`): the
/// C views of `include/nwv_types.h`'s `nwv_bls_*` structs.
#[derive(Clone, Copy)]
pub enum BlsItem {
    Header(ffi::NwvBlsHeader),
    Vote(ffi::NwvBlsVote),
    Certificate(ffi::NwvBlsCertificate),
}

/// `verify_items` under BLS12-381: every item in ONE engine call (`nwv_bls_verify_mixed_many`:
/// one digest launch, one BLS verification call -- single-key checks for headers and votes, one
/// fast_aggregate_verify per certificate), codes in the items' order.
pub fn verify_bls_items(committee: &ffi::NwvBlsCommittee, items: &[BlsItem]) -> Result<Vec<DagCode>, String> {
    let (mut hs, mut vs, mut cs) = (Vec::new(), Vec::new(), Vec::new());
    let (mut hi, mut vi, mut ci) = (Vec::new(), Vec::new(), Vec::new());
    for (i, it) in items.iter().enumerate() {
        match it {
            BlsItem::Header(h) => {
                hs.push(*h);
                hi.push(i)
            }
            BlsItem::Vote(v) => {
                vs.push(*v);
                vi.push(i)
            }
            BlsItem::Certificate(c) => {
                cs.push(*c);
                ci.push(i)
            }
        }
    }
    let mut rh = vec![0i32; hs.len()];
    let mut rv = vec![0i32; vs.len()];
    let mut rc = vec![0i32; cs.len()];
    let r = unsafe {
        ffi::nwv_bls_verify_mixed_many(
            crate::ctx(), committee, hs.len(), hs.as_ptr(), rh.as_mut_ptr(), vs.len(), vs.as_ptr(), rv.as_mut_ptr(),
            cs.len(), cs.as_ptr(), rc.as_mut_ptr(),
        )
    };
    if r != ffi::NWV_OK {
        return Err(last_error());
    }
    let mut codes = vec![0i32; items.len()];
    for (pos, res) in [(&hi, &rh), (&vi, &rv), (&ci, &rc)] {
        for (j, &i) in pos.iter().enumerate() {
            codes[i] = res[j];
        }
    }
    Ok(codes)
}

/// Running counters of a Core loop's drains (engine calls, items, largest flush).
#[derive(Default, Debug, Clone, Copy)]
pub struct DrainStats {
    pub calls: u64,
    pub items: u64,
    pub largest: usize,
}

impl DrainStats {
    pub fn record(&mut self, n: usize) {
        self.calls += 1;
        self.items += n as u64;
        self.largest = self.largest.max(n);
    }
}
