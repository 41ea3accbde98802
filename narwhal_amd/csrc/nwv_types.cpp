// nwv_types.cpp -- Narwhal Header / Vote / Certificate verification over the GPU engine
// (include/nwv_types.h).  Host-side control flow mirrors types/src/primary.rs check by check;
// every digest and every signature goes to the device through the C ABI of include/nwv.h, with
// the *_many forms batching a whole call into one BLAKE2b launch and one batch MSM.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/nwv_types.h"

namespace {

// NWV_HOST_TRACE=1: host-side phase timestamps of the mixed-batch path on stderr (diagnostics)
void htrace(const char* what) {
    static const bool on = std::getenv("NWV_HOST_TRACE") != nullptr;
    if (!on) return;
    const double us = std::chrono::duration<double, std::micro>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "nwv-trace %.1f %s\n", us, what);
}

void put(std::vector<uint8_t>& b, const uint8_t* p, size_t n) { b.insert(b.end(), p, p + n); }
// little-endian integers at a write cursor (the host is little-endian: x86-64 / aarch64)
uint8_t* at_le64(uint8_t* w, uint64_t v) {
    std::memcpy(w, &v, 8);
    return w + 8;
}
uint8_t* at_le32(uint8_t* w, uint32_t v) {
    std::memcpy(w, &v, 4);
    return w + 4;
}
uint8_t* at_bytes(uint8_t* w, const uint8_t* p, size_t n) {
    if (n) std::memcpy(w, p, n);
    return w + n;
}

// Header::digest preimage (types/src/primary.rs:209-227): author || round_le || epoch_le ||
// (batch digest || worker id_le)* in payload order || parent digests in BTreeSet order.  The
// arena grows once per preimage and the fields are copied in.
void header_preimage(const nwv_header& h, std::vector<uint8_t>& b) {
    const size_t at = b.size();
    b.resize(at + 48 + 36 * h.n_payload + 32 * h.n_parents);
    uint8_t* w = at_bytes(b.data() + at, h.author, 32);
    w = at_le64(w, h.round);
    w = at_le64(w, h.epoch);
    for (size_t i = 0; i < h.n_payload; i++) {
        w = at_bytes(w, h.payload_digests + 32 * i, 32);
        w = at_le32(w, h.payload_workers[i]);
    }
    at_bytes(w, h.parents, 32 * h.n_parents);  // contiguous, already in BTreeSet order
}
// Vote::digest (:351-364) and Certificate::digest (:594-607): id || round_le || epoch_le || origin
void id_round_epoch_origin(const uint8_t* id, uint64_t round, uint64_t epoch, const uint8_t* origin,
                           std::vector<uint8_t>& b) {
    const size_t at = b.size();
    b.resize(at + 80);
    uint8_t* w = at_bytes(b.data() + at, id, 32);
    w = at_le64(w, round);
    w = at_le64(w, epoch);
    at_bytes(w, origin, 32);
}

// Preimages appended to one arena, hashed in one nwv_blake2b256_many launch.  The batches of a
// call live in thread_local storage (reset per call): fresh multi-100 KB vectors per call would be
// page-faulted in every time, which costs more host time than the GPU work of a committee round.
struct DigestBatch {
    std::vector<uint8_t> arena;
    std::vector<uint64_t> off, len;
    void reset() {
        arena.clear();
        off.clear();
        len.clear();
    }
    size_t add_begin() {
        off.push_back(arena.size());
        return off.size() - 1;
    }
    void add_end() { len.push_back(arena.size() - off.back()); }
    int run(nwv_ctx* ctx, std::vector<uint8_t>& out) {
        out.assign(32 * off.size(), 0);
        if (off.empty()) return NWV_OK;
        arena.resize(arena.size() + 16);
        return nwv_blake2b256_many(ctx, off.size(), arena.data(), off.data(), len.data(), out.data());
    }
};

long committee_index(const nwv_committee& c, const uint8_t* pk);

// Committee lookups (keys sorted by bytes, as the BTreeMap)
long committee_index(const nwv_committee& c, const uint8_t* pk) {
    size_t lo = 0, hi = c.n;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        const int r = std::memcmp(c.keys + 32 * mid, pk, 32);
        if (r == 0) return (long)mid;
        if (r < 0) lo = mid + 1;
        else hi = mid;
    }
    return -1;
}
uint64_t committee_stake(const nwv_committee& c, const uint8_t* pk) {
    const long i = committee_index(c, pk);
    return i < 0 ? 0 : c.stakes[i];
}
// WorkerCache::worker(author, id) succeeds
bool worker_known(const nwv_committee& c, const uint8_t* author, uint32_t id) {
    const long i = committee_index(c, author);
    if (i < 0 || !c.n_workers) return false;
    for (uint32_t k = 0; k < c.n_workers[i]; k++)
        if (c.worker_ids[i][k] == id) return true;
    return false;
}
uint64_t quorum_threshold(const nwv_committee& c) {
    uint64_t total = 0;
    for (size_t i = 0; i < c.n; i++) total += c.stakes[i];
    return 2 * total / 3 + 1;
}
bool is_zero32(const uint8_t* p) {
    for (int i = 0; i < 32; i++)
        if (p[i]) return false;
    return true;
}
// Certificate::genesis(committee).contains(self): PartialEq (:615-623) compares header id,
// round, epoch and origin against the genesis certificates (default header of every authority)
bool is_genesis(const nwv_committee& c, const nwv_certificate& cert) {
    return is_zero32(cert.header.id) && cert.header.round == 0 && cert.header.epoch == c.epoch &&
           committee_index(c, cert.header.author) >= 0;
}

// Host-side checks of Header::verify before its digest and signature (:150-176); the digest
// comparison and worker ids are evaluated in reference order by the caller.
struct HeaderPlan {
    int pre = NWV_DAG_OK;   // epoch
    long digest = -1;       // index in the digest batch
    long sig = -1;          // index in the signature batch
    int post = NWV_DAG_OK;  // authority / worker checks (after the id check)
};

void plan_header(const nwv_committee& c, const nwv_header& h, DigestBatch& db, HeaderPlan& p) {
    if (h.epoch != c.epoch) {
        p.pre = NWV_DAG_INVALID_EPOCH;
        return;
    }
    p.digest = (long)db.add_begin();
    header_preimage(h, db.arena);
    db.add_end();
    if (committee_stake(c, h.author) == 0) {
        p.post = NWV_DAG_UNKNOWN_AUTHORITY;
        return;
    }
    for (size_t i = 0; i < h.n_payload; i++)
        if (!worker_known(c, h.author, h.payload_workers[i])) {
            p.post = NWV_DAG_MALFORMED_HEADER;
            return;
        }
}

bool valid_args(const nwv_committee* c) {
    return c && (c->n == 0 || (c->keys && c->stakes));
}

}  // namespace

extern "C" {

uint64_t nwv_committee_quorum_threshold(const nwv_committee* committee) {
    return committee ? quorum_threshold(*committee) : 0;
}

// ------------------------------------------------------------------ digests ------------
int nwv_header_digest_many(nwv_ctx* ctx, size_t n, const nwv_header* h, uint8_t* out) {
    if (!ctx || (n && (!h || !out))) return NWV_ERR_ARG;
    DigestBatch db;
    for (size_t i = 0; i < n; i++) {
        db.add_begin();
        header_preimage(h[i], db.arena);
        db.add_end();
    }
    std::vector<uint8_t> d;
    int rc = db.run(ctx, d);
    if (rc) return rc;
    if (n) std::memcpy(out, d.data(), 32 * n);
    return NWV_OK;
}
int nwv_vote_digest_many(nwv_ctx* ctx, size_t n, const nwv_vote* v, uint8_t* out) {
    if (!ctx || (n && (!v || !out))) return NWV_ERR_ARG;
    DigestBatch db;
    for (size_t i = 0; i < n; i++) {
        db.add_begin();
        id_round_epoch_origin(v[i].id, v[i].round, v[i].epoch, v[i].origin, db.arena);
        db.add_end();
    }
    std::vector<uint8_t> d;
    int rc = db.run(ctx, d);
    if (rc) return rc;
    if (n) std::memcpy(out, d.data(), 32 * n);
    return NWV_OK;
}
int nwv_certificate_digest_many(nwv_ctx* ctx, size_t n, const nwv_certificate* c, uint8_t* out) {
    if (!ctx || (n && (!c || !out))) return NWV_ERR_ARG;
    DigestBatch db;
    for (size_t i = 0; i < n; i++) {
        db.add_begin();
        id_round_epoch_origin(c[i].header.id, c[i].header.round, c[i].header.epoch, c[i].header.author,
                              db.arena);
        db.add_end();
    }
    std::vector<uint8_t> d;
    int rc = db.run(ctx, d);
    if (rc) return rc;
    if (n) std::memcpy(out, d.data(), 32 * n);
    return NWV_OK;
}
int nwv_header_digest(nwv_ctx* ctx, const nwv_header* h, uint8_t out[32]) {
    return nwv_header_digest_many(ctx, 1, h, out);
}
int nwv_vote_digest(nwv_ctx* ctx, const nwv_vote* v, uint8_t out[32]) { return nwv_vote_digest_many(ctx, 1, v, out); }
int nwv_certificate_digest(nwv_ctx* ctx, const nwv_certificate* c, uint8_t out[32]) {
    return nwv_certificate_digest_many(ctx, 1, c, out);
}

// ------------------------------------------------------------------ mixed batches ------
// Headers, votes and certificates of one call (Core::sanitize_header / sanitize_vote /
// sanitize_certificate, primary/src/core.rs:497-573, and CertificatesResponse::
// validate_certificates, responses.rs:95-141): every digest of the call in one BLAKE2b launch,
// every signature in one keyed batch MSM, then each item's verdict in the reference's check
// order (Header::verify :150-183, Vote::verify :307-328, Certificate::verify :487-537).
}  // extern "C"
namespace {
// Signatures of a mixed call, each over one of the call's digests (by index): the digests are
// hashed and the signatures verified by ONE engine call with no host round trip in between
// (nwv_ed25519_verify_batch_keyed_digests).  A header's signature is checked over its computed
// digest: whenever that verdict is used the id equals the digest (else InvalidHeaderId comes
// first), so the bytes are the ones the reference verifies.
struct DigestSigBatch {
    const nwv_committee* c = nullptr;
    std::vector<uint8_t> keys, sig, ok;
    std::vector<uint32_t> kidx, didx;
    std::vector<uint64_t> bits;
    void reset(const nwv_committee* cm) {
        c = cm;
        keys.clear();
        sig.clear();
        kidx.clear();
        didx.clear();
        if (c && c->n) keys.assign(c->keys, c->keys + 32 * c->n);
    }
    size_t add_run(const size_t* ks, size_t q, const uint8_t* s, size_t digest) {
        const size_t first = kidx.size();
        for (size_t k = 0; k < q; k++) kidx.push_back((uint32_t)ks[k]);
        put(sig, s, 64 * q);
        didx.insert(didx.end(), q, (uint32_t)digest);
        return first;
    }
    size_t add(const uint8_t* p, const uint8_t* s, size_t digest) {
        long k = committee_index(*c, p);
        if (k < 0) {  // not reached by the verify paths (unknown authors fail first); kept total
            k = (long)(keys.size() / 32);
            put(keys, p, 32);
        }
        const size_t kk = (size_t)k;
        return add_run(&kk, 1, s, digest);
    }
    int run(nwv_ctx* ctx, DigestBatch& db, std::vector<uint8_t>& dig) {
        const size_t n = kidx.size(), m = db.off.size();
        ok.assign(n, 1);
        dig.assign(32 * m, 0);
        if (m == 0) return NWV_OK;
        db.arena.resize(db.arena.size() + 16);
        bits.assign((n + 63) / 64 + 1, 0);
        int all = 0;
        // the committee registered on the devices (a no-op after an epoch's first call): a call of
        // at most 64 signatures by its members -- a certificate, a header, a vote -- then takes
        // the one-launch path (k_ed_tiny) inside the engine call below
        int rc = (c && c->n) ? nwv_keycache_register(ctx, c->n, c->keys) : NWV_OK;
        if (rc) return rc;
        rc = nwv_ed25519_verify_batch_keyed_digests(ctx, m, db.arena.data(), db.off.data(), db.len.data(),
                                                        dig.data(), keys.size() / 32, keys.data(), n, kidx.data(),
                                                        sig.data(), didx.data(), nullptr, &all, bits.data());
        if (rc) return rc;
        for (size_t i = 0; i < n; i++) ok[i] = (uint8_t)((bits[i >> 6] >> (i & 63)) & 1);
        return NWV_OK;
    }
};

// Header::verify up to its signature, once the digest is known (epoch, id, authority / workers)
int header_checks(const nwv_header& h, const HeaderPlan& p, const std::vector<uint8_t>& dig) {
    if (p.pre) return p.pre;
    if (std::memcmp(dig.data() + 32 * p.digest, h.id, 32) != 0) return NWV_DAG_INVALID_HEADER_ID;
    return p.post;
}

int verify_mixed(nwv_ctx* ctx, const nwv_committee& c, size_t nh, const nwv_header* h, int32_t* hres,
                 size_t nv, const nwv_vote* v, int32_t* vres, size_t nc, const nwv_certificate* cs,
                 int32_t* cres) {
    const uint64_t quorum = quorum_threshold(c);
    htrace("mixed:start");
    // phase 1 (host only): every preimage, and every signature a verdict may depend on, over
    // the index of the digest it signs
    thread_local DigestBatch db;
    thread_local DigestSigBatch sb;
    db.reset();
    sb.reset(&c);
    std::vector<HeaderPlan> hplan(nh), cplan(nc);
    for (size_t i = 0; i < nh; i++) {
        plan_header(c, h[i], db, hplan[i]);
        if (!hplan[i].pre && !hplan[i].post) hplan[i].sig = (long)sb.add(h[i].author, h[i].signature, hplan[i].digest);
    }
    htrace("mixed:headers");
    std::vector<long> vsig(nv, -1);
    for (size_t i = 0; i < nv; i++) {
        const size_t dg = db.add_begin();
        id_round_epoch_origin(v[i].id, v[i].round, v[i].epoch, v[i].origin, db.arena);
        db.add_end();
        if (v[i].epoch != c.epoch) vres[i] = NWV_DAG_INVALID_EPOCH;
        else if (committee_stake(c, v[i].author) == 0) vres[i] = NWV_DAG_UNKNOWN_AUTHORITY;
        else {
            vres[i] = NWV_DAG_OK;
            vsig[i] = (long)sb.add(v[i].author, v[i].signature, dg);
        }
    }
    htrace("mixed:votes");
    std::vector<uint8_t> done(nc, 0);
    std::vector<long> agg_first(nc, -1), agg_count(nc, 0);
    std::vector<int32_t> after_header(nc, NWV_DAG_OK);
    std::vector<size_t> pks;
    for (size_t i = 0; i < nc; i++) {
        const nwv_certificate& x = cs[i];
        cres[i] = NWV_DAG_OK;
        if (x.header.epoch != c.epoch) {  // Certificate::verify's own epoch check
            cres[i] = NWV_DAG_INVALID_EPOCH;
            done[i] = 1;
            continue;
        }
        if (is_genesis(c, x)) {  // genesis certificates are always valid
            done[i] = 1;
            continue;
        }
        HeaderPlan& hp = cplan[i];
        plan_header(c, x.header, db, hp);
        const size_t cdig = db.add_begin();
        id_round_epoch_origin(x.header.id, x.header.round, x.header.epoch, x.header.author, db.arena);
        db.add_end();
        if (hp.pre || hp.post) continue;  // the header's own error decides
        hp.sig = (long)sb.add(x.header.author, x.header.signature, hp.digest);
        // bitmap -> pks in committee order, as the filter at :505-520
        uint64_t weight = 0;
        size_t it = 0;
        pks.clear();
        for (size_t a = 0; a < c.n; a++) {
            if (it < x.n_signed && x.signed_authorities[it] == (uint32_t)a) {
                weight += c.stakes[a];
                it++;
                pks.push_back(a);
            }
        }
        if (weight < quorum) {
            after_header[i] = NWV_DAG_CERTIFICATE_REQUIRES_QUORUM;
            continue;
        }
        // Ed25519AggregateSignature::verify: |pks| != |sigs| -> Err before any crypto
        if (pks.size() != x.n_sigs) {
            after_header[i] = NWV_DAG_INVALID_SIGNATURE;
            continue;
        }
        agg_first[i] = (long)sb.add_run(pks.data(), pks.size(), x.aggregated_signature, cdig);
        agg_count[i] = (long)pks.size();
    }
    htrace("mixed:batch");
    // phase 2: one engine call (digests, then the signatures over them, on the device)
    thread_local std::vector<uint8_t> dig;
    int rc = sb.run(ctx, db, dig);
    if (rc) return rc;
    htrace("mixed:verified");
    const std::vector<uint8_t>& ok = sb.ok;
    // phase 3: verdicts in the reference's check order
    for (size_t i = 0; i < nh; i++) {
        hres[i] = header_checks(h[i], hplan[i], dig);
        if (hres[i] == NWV_DAG_OK && hplan[i].sig >= 0 && !ok[hplan[i].sig]) hres[i] = NWV_DAG_INVALID_SIGNATURE;
    }
    for (size_t i = 0; i < nv; i++)
        if (vsig[i] >= 0 && !ok[vsig[i]]) vres[i] = NWV_DAG_INVALID_SIGNATURE;
    for (size_t i = 0; i < nc; i++) {
        if (done[i]) continue;
        const int hr = header_checks(cs[i].header, cplan[i], dig);
        if (hr) {
            cres[i] = hr;
            continue;
        }
        if (cplan[i].sig >= 0 && !ok[cplan[i].sig]) {  // Header::verify's signature comes first
            cres[i] = NWV_DAG_INVALID_SIGNATURE;
            continue;
        }
        if (after_header[i]) {
            cres[i] = after_header[i];
            continue;
        }
        for (long k = 0; k < agg_count[i]; k++)
            if (!ok[agg_first[i] + k]) {
                cres[i] = NWV_DAG_INVALID_SIGNATURE;
                break;
            }
    }
    return NWV_OK;
}
}  // namespace
extern "C" {

int nwv_verify_mixed_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n_headers,
                          const nwv_header* headers, int32_t* header_results, size_t n_votes,
                          const nwv_vote* votes, int32_t* vote_results, size_t n_certs,
                          const nwv_certificate* certs, int32_t* cert_results) {
    if (!ctx || !valid_args(committee) || (n_headers && (!headers || !header_results)) ||
        (n_votes && (!votes || !vote_results)) || (n_certs && (!certs || !cert_results)))
        return NWV_ERR_ARG;
    return verify_mixed(ctx, *committee, n_headers, headers, header_results, n_votes, votes, vote_results,
                        n_certs, certs, cert_results);
}

// ------------------------------------------------------------------ Header::verify -----
int nwv_header_verify_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n, const nwv_header* h,
                           int32_t* results) {
    return nwv_verify_mixed_many(ctx, committee, n, h, results, 0, nullptr, nullptr, 0, nullptr, nullptr);
}
int nwv_header_verify(nwv_ctx* ctx, const nwv_committee* committee, const nwv_header* h) {
    int32_t r = 0;
    int rc = nwv_header_verify_many(ctx, committee, 1, h, &r);
    return rc ? rc : r;
}

// ------------------------------------------------------------------ Vote::verify -------
int nwv_vote_verify_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n, const nwv_vote* v,
                         int32_t* results) {
    return nwv_verify_mixed_many(ctx, committee, 0, nullptr, nullptr, n, v, results, 0, nullptr, nullptr);
}
int nwv_vote_verify(nwv_ctx* ctx, const nwv_committee* committee, const nwv_vote* v) {
    int32_t r = 0;
    int rc = nwv_vote_verify_many(ctx, committee, 1, v, &r);
    return rc ? rc : r;
}

// ------------------------------------------------------------------ Certificate::verify -
int nwv_certificate_verify_many(nwv_ctx* ctx, const nwv_committee* committee, size_t n,
                                const nwv_certificate* cs, int32_t* results) {
    return nwv_verify_mixed_many(ctx, committee, 0, nullptr, nullptr, 0, nullptr, nullptr, n, cs, results);
}
int nwv_certificate_verify(nwv_ctx* ctx, const nwv_committee* committee, const nwv_certificate* c) {
    int32_t r = 0;
    int rc = nwv_certificate_verify_many(ctx, committee, 1, c, &r);
    return rc ? rc : r;
}

int nwv_validate_certificates(nwv_ctx* ctx, const nwv_committee* committee, size_t n,
                              const nwv_certificate* c, size_t* n_invalid, size_t* invalid_idx) {
    if (!n_invalid || (n && !invalid_idx)) return NWV_ERR_ARG;
    *n_invalid = 0;
    if (n == 0) return NWV_OK;  // "No certificates are able to be served": Ok(vec![])
    std::vector<int32_t> r(n);
    int rc = nwv_certificate_verify_many(ctx, committee, n, c, r.data());
    if (rc) return rc;
    for (size_t i = 0; i < n; i++)
        if (r[i] != NWV_DAG_OK) invalid_idx[(*n_invalid)++] = i;
    return *n_invalid ? NWV_ERR_SIGNATURE : NWV_OK;
}

// ------------------------------------------------------------------ Certificate::new ----
int nwv_certificate_new(const nwv_committee* committee, size_t n_votes, const uint8_t* vote_pks,
                        const uint8_t* vote_sigs, int check_stake, uint32_t* signed_out,
                        size_t* n_signed, uint8_t* sigs_out, size_t* n_sigs) {
    if (!valid_args(committee) || !n_signed || !n_sigs || (n_votes && (!vote_pks || !vote_sigs)))
        return NWV_ERR_ARG;
    const nwv_committee& c = *committee;
    // votes.sort_by_key(pk) (stable), then walk the committee keys in order
    std::vector<size_t> order(n_votes);
    for (size_t i = 0; i < n_votes; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return std::memcmp(vote_pks + 32 * a, vote_pks + 32 * b, 32) < 0;
    });
    auto same_vote = [&](size_t a, size_t b) {
        return std::memcmp(vote_pks + 32 * a, vote_pks + 32 * b, 32) == 0 &&
               std::memcmp(vote_sigs + 64 * a, vote_sigs + 64 * b, 64) == 0;
    };
    size_t front = 0, ns = 0;
    uint64_t weight = 0;
    std::vector<size_t> taken;
    for (size_t k = 0; k < c.n; k++) {
        if (front < n_votes && std::memcmp(c.keys + 32 * k, vote_pks + 32 * order[front], 32) == 0) {
            taken.push_back(order[front++]);
            weight += c.stakes[k];
            while (front < n_votes && same_vote(order[front], taken.back())) front++;  // repeats
            if (signed_out) signed_out[ns] = (uint32_t)k;
            ns++;
        }
    }
    if (front < n_votes) return NWV_DAG_UNKNOWN_AUTHORITY;
    if (check_stake && weight < quorum_threshold(c)) return NWV_DAG_CERTIFICATE_REQUIRES_QUORUM;
    *n_signed = ns;
    *n_sigs = taken.size();
    if (sigs_out)
        for (size_t k = 0; k < taken.size(); k++) std::memcpy(sigs_out + 64 * k, vote_sigs + 64 * taken[k], 64);
    return NWV_DAG_OK;
}

}  // extern "C"

// ====================================================================================== BLS
// The types layer under the reference's default scheme, BLS12-381 (crypto/src/lib.rs:29-33).  The
// control flow is the Ed25519 layer's, check by check (types/src/primary.rs); what differs is the
// key length in the digests (96-byte authors / origins) and the signature checks: a header's or a
// vote's signature is Verifier::verify (one key), a certificate's aggregate is ONE
// fast_aggregate_verify over its signers' keys (blst; no |pks| = |sigs| check: the aggregate is
// a single G1 point), an aggregate holding no signature fails (sig: None).  All of a call's
// signature checks go to the GPU as one nwv_bls_verify_many call over the committee's keys, which
// are registered in the device's BLS key cache.
#include "../../include/nwv_bls.h"

namespace {
constexpr size_t BK = 96;  // BLS public key bytes
constexpr size_t BS = 48;  // BLS signature bytes

void bls_header_preimage(const nwv_bls_header& h, std::vector<uint8_t>& b) {
    const size_t at = b.size();
    b.resize(at + BK + 16 + 36 * h.n_payload + 32 * h.n_parents);
    uint8_t* w = at_bytes(b.data() + at, h.author, BK);
    w = at_le64(w, h.round);
    w = at_le64(w, h.epoch);
    for (size_t i = 0; i < h.n_payload; i++) {
        w = at_bytes(w, h.payload_digests + 32 * i, 32);
        w = at_le32(w, h.payload_workers[i]);
    }
    at_bytes(w, h.parents, 32 * h.n_parents);
}
void bls_id_round_epoch_origin(const uint8_t* id, uint64_t round, uint64_t epoch, const uint8_t* origin,
                               std::vector<uint8_t>& b) {
    const size_t at = b.size();
    b.resize(at + 48 + BK);
    uint8_t* w = at_bytes(b.data() + at, id, 32);
    w = at_le64(w, round);
    w = at_le64(w, epoch);
    at_bytes(w, origin, BK);
}
long bls_index(const nwv_bls_committee& c, const uint8_t* pk) {
    size_t lo = 0, hi = c.n;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        const int r = std::memcmp(c.keys + BK * mid, pk, BK);
        if (r == 0) return (long)mid;
        if (r < 0) lo = mid + 1;
        else hi = mid;
    }
    return -1;
}
uint64_t bls_stake(const nwv_bls_committee& c, const uint8_t* pk) {
    const long i = bls_index(c, pk);
    return i < 0 ? 0 : c.stakes[i];
}
bool bls_worker_known(const nwv_bls_committee& c, const uint8_t* author, uint32_t id) {
    const long i = bls_index(c, author);
    if (i < 0 || !c.n_workers) return false;
    for (uint32_t k = 0; k < c.n_workers[i]; k++)
        if (c.worker_ids[i][k] == id) return true;
    return false;
}
uint64_t bls_quorum(const nwv_bls_committee& c) {
    uint64_t total = 0;
    for (size_t i = 0; i < c.n; i++) total += c.stakes[i];
    return 2 * total / 3 + 1;
}
bool bls_is_genesis(const nwv_bls_committee& c, const nwv_bls_certificate& cert) {
    return is_zero32(cert.header.id) && cert.header.round == 0 && cert.header.epoch == c.epoch &&
           bls_index(c, cert.header.author) >= 0;
}
void bls_plan_header(const nwv_bls_committee& c, const nwv_bls_header& h, DigestBatch& db, HeaderPlan& p) {
    if (h.epoch != c.epoch) {
        p.pre = NWV_DAG_INVALID_EPOCH;
        return;
    }
    p.digest = (long)db.add_begin();
    bls_header_preimage(h, db.arena);
    db.add_end();
    if (bls_stake(c, h.author) == 0) {
        p.post = NWV_DAG_UNKNOWN_AUTHORITY;
        return;
    }
    for (size_t i = 0; i < h.n_payload; i++)
        if (!bls_worker_known(c, h.author, h.payload_workers[i])) {
            p.post = NWV_DAG_MALFORMED_HEADER;
            return;
        }
}
bool bls_valid_args(const nwv_bls_committee* c) { return c && (c->n == 0 || (c->keys && c->stakes)); }

// The signature checks of one call as nwv_bls_verify_many items over the committee's keys: item =
// (signature, signer indices, message).  A header's signature is checked over its id (when that
// verdict is used, id == digest: InvalidHeaderId comes first), a vote's and a certificate's over
// the digest computed by the call.
struct BlsItems {
    std::vector<uint8_t> sig, msg;
    std::vector<uint32_t> off, cnt, idx, mlen;
    std::vector<uint64_t> moff;
    std::vector<int32_t> st;
    void reset() {
        sig.clear();
        msg.clear();
        off.clear();
        cnt.clear();
        idx.clear();
        mlen.clear();
        moff.clear();
    }
    long add(const uint8_t* s, const uint32_t* keys, size_t nk, const uint8_t* m) {
        put(sig, s, BS);
        off.push_back((uint32_t)idx.size());
        cnt.push_back((uint32_t)nk);
        idx.insert(idx.end(), keys, keys + nk);
        moff.push_back(msg.size());
        mlen.push_back(32);
        put(msg, m, 32);
        return (long)off.size() - 1;
    }
    int run(nwv_ctx* ctx, const nwv_bls_committee& c) {
        st.assign(off.size(), 0);
        if (off.empty()) return NWV_OK;
        msg.resize(msg.size() + 8);
        return nwv_bls_verify_many(ctx, c.n, c.keys, off.size(), sig.data(), off.data(), cnt.data(),
                                   idx.empty() ? nullptr : idx.data(), msg.data(), moff.data(), mlen.data(), nullptr, 0,
                                   st.data());
    }
};

int bls_verify_mixed(nwv_ctx* ctx, const nwv_bls_committee& c, size_t nh, const nwv_bls_header* h, int32_t* hres,
                     size_t nv, const nwv_bls_vote* v, int32_t* vres, size_t nc, const nwv_bls_certificate* cs,
                     int32_t* cres) {
    const uint64_t quorum = bls_quorum(c);
    thread_local DigestBatch db;
    thread_local BlsItems items;
    db.reset();
    items.reset();
    // phase 1 (host): every preimage; the signature checks are listed once the digests are known
    std::vector<HeaderPlan> hplan(nh), cplan(nc);
    for (size_t i = 0; i < nh; i++) bls_plan_header(c, h[i], db, hplan[i]);
    std::vector<long> vdig(nv, -1);
    for (size_t i = 0; i < nv; i++) {
        vdig[i] = (long)db.add_begin();
        bls_id_round_epoch_origin(v[i].id, v[i].round, v[i].epoch, v[i].origin, db.arena);
        db.add_end();
    }
    std::vector<uint8_t> done(nc, 0);
    std::vector<long> cdig(nc, -1);
    for (size_t i = 0; i < nc; i++) {
        const nwv_bls_certificate& x = cs[i];
        if (x.header.epoch != c.epoch || bls_is_genesis(c, x)) {
            done[i] = 1;
            continue;
        }
        bls_plan_header(c, x.header, db, cplan[i]);
        cdig[i] = (long)db.add_begin();
        bls_id_round_epoch_origin(x.header.id, x.header.round, x.header.epoch, x.header.author, db.arena);
        db.add_end();
    }
    // phase 2: the digests (one BLAKE2b launch), then every signature check (one BLS call)
    std::vector<uint8_t> dig;
    int rc = db.run(ctx, dig);
    if (rc) return rc;
    std::vector<long> hsig(nh, -1), vsig(nv, -1), csig(nc, -1), asig(nc, -1);
    std::vector<int32_t> after_header(nc, NWV_DAG_OK);
    for (size_t i = 0; i < nh; i++) {
        const HeaderPlan& p = hplan[i];
        if (p.pre || p.post || std::memcmp(dig.data() + 32 * p.digest, h[i].id, 32) != 0) continue;
        const uint32_t a = (uint32_t)bls_index(c, h[i].author);
        hsig[i] = items.add(h[i].signature, &a, 1, h[i].id);
    }
    for (size_t i = 0; i < nv; i++) {
        if (v[i].epoch != c.epoch || bls_stake(c, v[i].author) == 0) continue;
        const uint32_t a = (uint32_t)bls_index(c, v[i].author);
        vsig[i] = items.add(v[i].signature, &a, 1, dig.data() + 32 * vdig[i]);
    }
    std::vector<uint32_t> pks;
    for (size_t i = 0; i < nc; i++) {
        if (done[i]) continue;
        const nwv_bls_certificate& x = cs[i];
        const HeaderPlan& p = cplan[i];
        if (p.pre || p.post || std::memcmp(dig.data() + 32 * p.digest, x.header.id, 32) != 0) continue;
        const uint32_t a = (uint32_t)bls_index(c, x.header.author);
        csig[i] = items.add(x.header.signature, &a, 1, x.header.id);
        // bitmap -> pks in committee order (:505-520), quorum, then the aggregate
        uint64_t weight = 0;
        size_t it = 0;
        pks.clear();
        for (size_t k = 0; k < c.n; k++)
            if (it < x.n_signed && x.signed_authorities[it] == (uint32_t)k) {
                weight += c.stakes[k];
                it++;
                pks.push_back((uint32_t)k);
            }
        if (weight < quorum) {
            after_header[i] = NWV_DAG_CERTIFICATE_REQUIRES_QUORUM;
            continue;
        }
        if (!x.aggregated_signature) {  // sig: None -> signature::Error
            after_header[i] = NWV_DAG_INVALID_SIGNATURE;
            continue;
        }
        asig[i] = items.add(x.aggregated_signature, pks.data(), pks.size(), dig.data() + 32 * cdig[i]);
    }
    if ((rc = nwv_bls_keycache_register(ctx, c.n, c.keys))) return rc;  // no-op once registered
    if ((rc = items.run(ctx, c))) return rc;
    auto bad = [&](long k) { return k >= 0 && items.st[k] != NWV_BLS_OK; };
    // phase 3: verdicts in the reference's check order
    for (size_t i = 0; i < nh; i++) {
        const HeaderPlan& p = hplan[i];
        if (p.pre) hres[i] = p.pre;
        else if (std::memcmp(dig.data() + 32 * p.digest, h[i].id, 32) != 0) hres[i] = NWV_DAG_INVALID_HEADER_ID;
        else if (p.post) hres[i] = p.post;
        else hres[i] = bad(hsig[i]) ? NWV_DAG_INVALID_SIGNATURE : NWV_DAG_OK;
    }
    for (size_t i = 0; i < nv; i++) {
        if (v[i].epoch != c.epoch) vres[i] = NWV_DAG_INVALID_EPOCH;
        else if (bls_stake(c, v[i].author) == 0) vres[i] = NWV_DAG_UNKNOWN_AUTHORITY;
        else vres[i] = bad(vsig[i]) ? NWV_DAG_INVALID_SIGNATURE : NWV_DAG_OK;
    }
    for (size_t i = 0; i < nc; i++) {
        const nwv_bls_certificate& x = cs[i];
        if (x.header.epoch != c.epoch) {
            cres[i] = NWV_DAG_INVALID_EPOCH;
            continue;
        }
        if (done[i]) {  // genesis
            cres[i] = NWV_DAG_OK;
            continue;
        }
        const HeaderPlan& p = cplan[i];
        if (p.pre) cres[i] = p.pre;
        else if (std::memcmp(dig.data() + 32 * p.digest, x.header.id, 32) != 0) cres[i] = NWV_DAG_INVALID_HEADER_ID;
        else if (p.post) cres[i] = p.post;
        else if (bad(csig[i])) cres[i] = NWV_DAG_INVALID_SIGNATURE;
        else if (after_header[i]) cres[i] = after_header[i];
        else cres[i] = bad(asig[i]) ? NWV_DAG_INVALID_SIGNATURE : NWV_DAG_OK;
    }
    return NWV_OK;
}
template <class T, class F>
int bls_digest_many(nwv_ctx* ctx, size_t n, const T* x, uint8_t* out, F pre) {
    if (!ctx || (n && (!x || !out))) return NWV_ERR_ARG;
    DigestBatch db;
    for (size_t i = 0; i < n; i++) {
        db.add_begin();
        pre(x[i], db.arena);
        db.add_end();
    }
    std::vector<uint8_t> d;
    int rc = db.run(ctx, d);
    if (rc) return rc;
    if (n) std::memcpy(out, d.data(), 32 * n);
    return NWV_OK;
}
}  // namespace

extern "C" {

int nwv_bls_header_digest_many(nwv_ctx* ctx, size_t n, const nwv_bls_header* h, uint8_t* out) {
    return bls_digest_many(ctx, n, h, out, [](const nwv_bls_header& x, std::vector<uint8_t>& b) { bls_header_preimage(x, b); });
}
int nwv_bls_vote_digest_many(nwv_ctx* ctx, size_t n, const nwv_bls_vote* v, uint8_t* out) {
    return bls_digest_many(ctx, n, v, out, [](const nwv_bls_vote& x, std::vector<uint8_t>& b) {
        bls_id_round_epoch_origin(x.id, x.round, x.epoch, x.origin, b);
    });
}
int nwv_bls_certificate_digest_many(nwv_ctx* ctx, size_t n, const nwv_bls_certificate* c, uint8_t* out) {
    return bls_digest_many(ctx, n, c, out, [](const nwv_bls_certificate& x, std::vector<uint8_t>& b) {
        bls_id_round_epoch_origin(x.header.id, x.header.round, x.header.epoch, x.header.author, b);
    });
}

int nwv_bls_verify_mixed_many(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t n_headers,
                              const nwv_bls_header* headers, int32_t* header_results, size_t n_votes,
                              const nwv_bls_vote* votes, int32_t* vote_results, size_t n_certs,
                              const nwv_bls_certificate* certs, int32_t* cert_results) {
    if (!ctx || !bls_valid_args(committee) || (n_headers && (!headers || !header_results)) ||
        (n_votes && (!votes || !vote_results)) || (n_certs && (!certs || !cert_results)))
        return NWV_ERR_ARG;
    return bls_verify_mixed(ctx, *committee, n_headers, headers, header_results, n_votes, votes, vote_results,
                            n_certs, certs, cert_results);
}

int nwv_bls_validate_certificates(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t n,
                                  const nwv_bls_certificate* c, size_t* n_invalid, size_t* invalid_idx) {
    if (!n_invalid || (n && !invalid_idx)) return NWV_ERR_ARG;
    *n_invalid = 0;
    if (n == 0) return NWV_OK;
    std::vector<int32_t> r(n);
    int rc = nwv_bls_verify_mixed_many(ctx, committee, 0, nullptr, nullptr, 0, nullptr, nullptr, n, c, r.data());
    if (rc) return rc;
    for (size_t i = 0; i < n; i++)
        if (r[i] != NWV_DAG_OK) invalid_idx[(*n_invalid)++] = i;
    return *n_invalid ? NWV_ERR_SIGNATURE : NWV_OK;
}

int nwv_bls_certificate_new(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t n_votes,
                            const uint8_t* vote_pks, const uint8_t* vote_sigs, int check_stake,
                            uint32_t* signed_out, size_t* n_signed, uint8_t* agg_out, int* has_agg) {
    if (!ctx || !bls_valid_args(committee) || !n_signed || !has_agg || !agg_out ||
        (n_votes && (!vote_pks || !vote_sigs)))
        return NWV_ERR_ARG;
    const nwv_bls_committee& c = *committee;
    std::vector<size_t> order(n_votes);
    for (size_t i = 0; i < n_votes; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return std::memcmp(vote_pks + BK * a, vote_pks + BK * b, BK) < 0;
    });
    auto same_vote = [&](size_t a, size_t b) {
        return std::memcmp(vote_pks + BK * a, vote_pks + BK * b, BK) == 0 &&
               std::memcmp(vote_sigs + BS * a, vote_sigs + BS * b, BS) == 0;
    };
    size_t front = 0, ns = 0;
    uint64_t weight = 0;
    std::vector<uint8_t> kept;
    for (size_t k = 0; k < c.n; k++) {
        if (front < n_votes && std::memcmp(c.keys + BK * k, vote_pks + BK * order[front], BK) == 0) {
            const size_t t = order[front++];
            put(kept, vote_sigs + BS * t, BS);
            weight += c.stakes[k];
            while (front < n_votes && same_vote(order[front], t)) front++;
            if (signed_out) signed_out[ns] = (uint32_t)k;
            ns++;
        }
    }
    if (front < n_votes) return NWV_DAG_UNKNOWN_AUTHORITY;
    if (check_stake && weight < bls_quorum(c)) return NWV_DAG_CERTIFICATE_REQUIRES_QUORUM;
    *n_signed = ns;
    *has_agg = 0;
    if (kept.empty()) return NWV_DAG_OK;  // AggregateSignature::default()
    const int rc = nwv_bls_aggregate(ctx, kept.size() / BS, kept.data(), agg_out, nullptr);
    if (rc == NWV_ERR_SIGNATURE) return NWV_DAG_INVALID_SIGNATURE;  // AggregateSignature::aggregate fails
    if (rc) return rc;
    *has_agg = 1;
    return NWV_DAG_OK;
}

}  // extern "C"
