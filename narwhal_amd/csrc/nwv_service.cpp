// nwv_service.cpp -- batching verification service (include/nwv_service.h).
//
// Submitters (any threads) enqueue deep copies of headers / votes / certificates; flusher threads
// coalesce what is pending into one nwv_verify_mixed_many call (include/nwv_types.h: one BLAKE2b
// launch, one batch MSM on the GPU) and complete every item with its own DagError code, in the
// role of the Core loop's per-message sanitize_* calls (primary/src/core.rs:497-573, loop
// :614-714).  Plain host C++ over the C ABI; no GPU code here.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <thread>
#include <vector>

#include "../../include/nwv_service.h"

namespace {

using Clock = std::chrono::steady_clock;

// committee (config/src/lib.rs:488-551) owned by the service; items keep the one current at
// their submission.  Ed25519 committees hold 32-byte keys, BLS12-381 ones 96-byte keys (the two
// C structs differ only in that).
struct OwnedCommittee {
    std::vector<uint8_t> keys;
    std::vector<uint64_t> stakes;
    std::vector<uint32_t> n_workers;
    std::vector<std::vector<uint32_t>> ids;
    std::vector<const uint32_t*> id_ptr;
    nwv_committee view{};
    nwv_bls_committee bview{};

    OwnedCommittee(size_t n, const uint8_t* k, size_t key_bytes, const uint64_t* st, uint64_t epoch,
                   const uint32_t* nw, const uint32_t* const* wid)
        : keys(k, k + key_bytes * n), stakes(st, st + n), ids(n), id_ptr(n, nullptr) {
        n_workers.assign(n, 0);
        for (size_t i = 0; i < n; i++) {
            const uint32_t c = nw ? nw[i] : 0;
            n_workers[i] = c;
            if (c && wid && wid[i]) ids[i].assign(wid[i], wid[i] + c);
            id_ptr[i] = ids[i].empty() ? nullptr : ids[i].data();
        }
        view = nwv_committee{n, keys.data(), stakes.data(), epoch, n_workers.data(), id_ptr.data()};
        bview = nwv_bls_committee{n, keys.data(), stakes.data(), epoch, n_workers.data(), id_ptr.data()};
    }
    explicit OwnedCommittee(const nwv_committee& c)
        : OwnedCommittee(c.n, c.keys, 32, c.stakes, c.epoch, c.n_workers, c.worker_ids) {}
    explicit OwnedCommittee(const nwv_bls_committee& c)
        : OwnedCommittee(c.n, c.keys, 96, c.stakes, c.epoch, c.n_workers, c.worker_ids) {}
};

enum Kind { HEADER = 0, VOTE = 1, CERT = 2 };

// an uninitialised buffer (every byte of an item's copy is written by the copy itself: a vector's
// zero fill doubled the memory traffic of a submission)
template <class T>
struct RawBuf {
    std::unique_ptr<T[]> p;
    void resize(size_t n) { p.reset(n ? new T[n] : nullptr); }
    T* data() { return p.get(); }
};

// one submitted message, deep-copied: the views point into bytes / words
struct Item {
    Kind kind;
    RawBuf<uint8_t> bytes;
    RawBuf<uint32_t> words;
    nwv_header h{};
    nwv_vote v{};
    nwv_certificate c{};
    nwv_bls_header bh{};  // BLS12-381 services
    nwv_bls_vote bv{};
    nwv_bls_certificate bc{};
    nwv_done_fn done = nullptr;
    void* user = nullptr;
    Clock::time_point t;
    uint64_t seq = 0;
    std::shared_ptr<const OwnedCommittee> com;
};

size_t header_bytes(const nwv_header& h) { return 32 + 32 * h.n_payload + 32 * h.n_parents + 32 + 64; }

// copies h into it->bytes / words starting at byte `at` / word `wat`; it->h views the copy
void copy_header(Item* it, const nwv_header& h, size_t at, size_t wat, nwv_header& out) {
    uint8_t* b = it->bytes.data() + at;
    auto put = [&](const uint8_t* src, size_t n) {
        if (n && src) std::memcpy(b, src, n);
        else if (n) std::memset(b, 0, n);
        const uint8_t* r = b;
        b += n;
        return r;
    };
    out = h;
    out.author = put(h.author, 32);
    out.payload_digests = put(h.payload_digests, 32 * h.n_payload);
    out.parents = put(h.parents, 32 * h.n_parents);
    out.id = put(h.id, 32);
    out.signature = put(h.signature, 64);
    uint32_t* w = it->words.data() + wat;
    if (h.n_payload && h.payload_workers) std::memcpy(w, h.payload_workers, 4 * h.n_payload);
    out.payload_workers = h.n_payload ? w : nullptr;
    if (!h.n_payload) out.payload_digests = nullptr;
    if (!h.n_parents) out.parents = nullptr;
}

// the BLS12-381 header layout (96-byte author, 48-byte signature)
size_t bls_header_bytes(const nwv_bls_header& h) { return 96 + 32 * h.n_payload + 32 * h.n_parents + 32 + 48; }
void copy_bls_header(Item* it, const nwv_bls_header& h, size_t at, size_t wat, nwv_bls_header& out) {
    uint8_t* b = it->bytes.data() + at;
    auto put = [&](const uint8_t* src, size_t n) {
        if (n && src) std::memcpy(b, src, n);
        else if (n) std::memset(b, 0, n);
        const uint8_t* r = b;
        b += n;
        return r;
    };
    out = h;
    out.author = put(h.author, 96);
    out.payload_digests = put(h.payload_digests, 32 * h.n_payload);
    out.parents = put(h.parents, 32 * h.n_parents);
    out.id = put(h.id, 32);
    out.signature = put(h.signature, 48);
    uint32_t* w = it->words.data() + wat;
    if (h.n_payload && h.payload_workers) std::memcpy(w, h.payload_workers, 4 * h.n_payload);
    out.payload_workers = h.n_payload ? w : nullptr;
    if (!h.n_payload) out.payload_digests = nullptr;
    if (!h.n_parents) out.parents = nullptr;
}

template <class H>
bool header_ok(const H* h) {
    return h && h->author && h->id && h->signature && (!h->n_payload || (h->payload_digests && h->payload_workers)) &&
           (!h->n_parents || h->parents);
}

struct Waiter {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    int32_t r = 0;
};
void waiter_done(void* user, int32_t r) {
    auto* w = static_cast<Waiter*>(user);
    {
        std::lock_guard<std::mutex> g(w->m);
        w->r = r;
        w->done = true;
    }
    w->cv.notify_one();
}

// The service whose completion callbacks this thread is running (null outside callbacks).  A
// callback may submit asynchronously, but a blocking call on THAT service (nwv_service_verify_*,
// nwv_service_flush) would wait for batches that this very thread -- or, with both flushers inside
// callbacks, no thread -- would ever verify: such calls return NWV_ERR_REENTRANT instead of
// deadlocking.  Blocking calls on another service are refused only when they would close a cycle
// of such waits (WaitEdge below).  Set and restored by an RAII guard, so a callback that unwinds
// cannot leave it set.
thread_local const nwv_service* tl_cb_svc = nullptr;
struct CallbackScope {
    const nwv_service* prev;
    explicit CallbackScope(const nwv_service* s) : prev(tl_cb_svc) { tl_cb_svc = s; }
    ~CallbackScope() { tl_cb_svc = prev; }
};

// Blocking calls made from callbacks across services: while a callback of service A waits on
// service B, the edge A -> B is in a process-wide waits-for graph.  A wait that would close a
// cycle (B's callbacks already wait, directly or through other services, on A) is refused with
// NWV_ERR_REENTRANT: with every flusher of each service inside such a callback, none of them
// would ever verify the batch another one waits for.
std::mutex g_wait_mu;
std::multiset<std::pair<const nwv_service*, const nwv_service*>> g_wait_edges;
bool waits_reach(const nwv_service* from, const nwv_service* to) {  // g_wait_mu held
    std::vector<const nwv_service*> stack{from};
    std::set<const nwv_service*> seen;
    while (!stack.empty()) {
        const nwv_service* x = stack.back();
        stack.pop_back();
        if (x == to) return true;
        if (!seen.insert(x).second) continue;
        for (auto it = g_wait_edges.lower_bound({x, nullptr}); it != g_wait_edges.end() && it->first == x; ++it)
            stack.push_back(it->second);
    }
    return false;
}
// registers the edge (callback's service -> target) for the duration of a blocking call
struct WaitEdge {
    const nwv_service* from = nullptr;
    const nwv_service* to = nullptr;
    int rc = NWV_OK;
    explicit WaitEdge(const nwv_service* target) {
        if (!tl_cb_svc || !target) return;  // not inside a callback: nothing can wait on this thread
        if (tl_cb_svc == target) {
            rc = NWV_ERR_REENTRANT;
            return;
        }
        std::lock_guard<std::mutex> g(g_wait_mu);
        if (waits_reach(target, tl_cb_svc)) {
            rc = NWV_ERR_REENTRANT;
            return;
        }
        from = tl_cb_svc;
        to = target;
        g_wait_edges.insert({from, to});
    }
    ~WaitEdge() {
        if (!from) return;
        std::lock_guard<std::mutex> g(g_wait_mu);
        g_wait_edges.erase(g_wait_edges.find({from, to}));
    }
};

template <class Submit>
int verify_blocking(const nwv_service* svc, Submit submit, int32_t* result) {
    if (!result) return NWV_ERR_ARG;
    WaitEdge edge(svc);
    if (edge.rc) return edge.rc;
    Waiter w;
    const int rc = submit(&w);
    if (rc) return rc;
    std::unique_lock<std::mutex> lk(w.m);
    w.cv.wait(lk, [&] { return w.done; });
    *result = w.r;
    return w.r < 0 ? w.r : NWV_OK;
}

}  // namespace

struct nwv_service {
    nwv_ctx* ctx = nullptr;
    bool bls = false;  // BLS12-381 service (nwv_service_create_bls): one nwv_bls_verify_mixed_many per flush
    size_t max_batch = 1;
    std::chrono::microseconds max_wait{0};
    std::chrono::microseconds idle{0};  // nwv_service_set_idle: flush once no item arrived for this long (0: off)
    Clock::time_point last_submit{};
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<std::unique_ptr<Item>> pending;
    std::set<uint64_t> open;  // sequence numbers submitted and not yet completed
    std::shared_ptr<const OwnedCommittee> com;
    uint64_t next_seq = 0, flush_upto = 0;
    bool stop = false;
    uint64_t stats[6] = {0, 0, 0, 0, 0, 0};
    std::vector<std::thread> workers;

    void run();
    int submit(std::unique_ptr<Item> it, nwv_done_fn done, void* user);
};

// flusher: waits for a full batch, the oldest item's deadline, a flush request or stop; takes the
// pending items that share the front item's committee; verifies them in one engine call
void nwv_service::run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
        if (pending.empty()) {
            if (stop) return;
            cv_work.wait(lk);
            continue;
        }
        const Item& front = *pending.front();
        int reason = -1;
        if (pending.size() >= max_batch) reason = 3;
        else if (stop || flush_upto > front.seq) reason = 5;
        else {
            // a burst has ended (no arrival for `idle`) or the oldest item has waited max_wait
            const auto now = Clock::now();
            auto due = front.t + max_wait;
            if (idle.count() > 0) due = std::min(due, last_submit + idle);
            if (now >= due) reason = 4;
        }
        if (reason < 0) {
            auto due = front.t + max_wait;
            if (idle.count() > 0) due = std::min(due, last_submit + idle);
            cv_work.wait_until(lk, due);
            continue;
        }
        // take up to 8 batches' worth: under a backlog one larger call beats several small ones
        std::vector<std::unique_ptr<Item>> batch;
        const auto com_b = pending.front()->com;
        while (!pending.empty() && batch.size() < 8 * max_batch && pending.front()->com == com_b) {
            batch.push_back(std::move(pending.front()));
            pending.pop_front();
        }
        if (!pending.empty()) cv_work.notify_one();  // the rest may be another flusher's
        lk.unlock();
        size_t nh = 0, nv = 0, nc = 0;
        for (auto& it : batch) (it->kind == HEADER ? nh : it->kind == VOTE ? nv : nc)++;
        std::vector<int32_t> rh(nh), rv(nv), rc(nc);
        int rc_call;
        if (bls) {
            std::vector<nwv_bls_header> H;
            std::vector<nwv_bls_vote> V;
            std::vector<nwv_bls_certificate> C;
            for (auto& it : batch) {
                if (it->kind == HEADER) H.push_back(it->bh);
                else if (it->kind == VOTE) V.push_back(it->bv);
                else C.push_back(it->bc);
            }
            rc_call = nwv_bls_verify_mixed_many(ctx, &com_b->bview, nh, H.data(), rh.data(), nv, V.data(), rv.data(),
                                                nc, C.data(), rc.data());
        } else {
            std::vector<nwv_header> H;
            std::vector<nwv_vote> V;
            std::vector<nwv_certificate> C;
            for (auto& it : batch) {
                if (it->kind == HEADER) H.push_back(it->h);
                else if (it->kind == VOTE) V.push_back(it->v);
                else C.push_back(it->c);
            }
            rc_call = nwv_verify_mixed_many(ctx, &com_b->view, nh, H.data(), rh.data(), nv, V.data(), rv.data(), nc,
                                            C.data(), rc.data());
        }
        // the call's statistics before its callbacks: a submitter woken by its verdict sees them
        lk.lock();
        stats[0]++;
        stats[1] += batch.size();
        stats[2] = std::max<uint64_t>(stats[2], batch.size());
        stats[reason]++;
        lk.unlock();
        size_t ih = 0, iv = 0, ic = 0;
        {
            CallbackScope scope(this);
            for (auto& it : batch) {
                int32_t r = rc_call;
                if (rc_call == 0) r = it->kind == HEADER ? rh[ih++] : it->kind == VOTE ? rv[iv++] : rc[ic++];
                if (it->done) it->done(it->user, r);
            }
        }
        lk.lock();
        for (auto& it : batch) open.erase(it->seq);
        cv_done.notify_all();
    }
}

int nwv_service::submit(std::unique_ptr<Item> it, nwv_done_fn done, void* user) {
    it->done = done;
    it->user = user;
    std::lock_guard<std::mutex> g(mu);
    if (stop) return NWV_ERR_ARG;
    it->com = com;
    it->seq = next_seq++;
    it->t = Clock::now();
    last_submit = it->t;
    open.insert(it->seq);
    pending.push_back(std::move(it));
    if (pending.size() == 1 || pending.size() >= max_batch) cv_work.notify_one();
    return NWV_OK;
}

extern "C" {

}  // extern "C"

namespace {
template <class Committee>
int service_create(nwv_ctx* ctx, const Committee* committee, size_t max_batch, uint32_t max_wait_us, bool bls,
                   nwv_service** out) {
    if (!out) return NWV_ERR_ARG;
    *out = nullptr;
    if (!ctx || !committee || !committee->keys || !committee->stakes || max_batch == 0) return NWV_ERR_ARG;
    auto* s = new (std::nothrow) nwv_service;
    if (!s) return NWV_ERR_OOM;
    try {
        s->ctx = ctx;
        s->bls = bls;
        s->max_batch = max_batch;
        s->max_wait = std::chrono::microseconds(max_wait_us);
        s->com = std::make_shared<const OwnedCommittee>(*committee);
        // two flushers: one builds and verifies a batch while the other's is on the GPU (the
        // engine's per-device lanes let the calls overlap)
        for (int k = 0; k < 2; k++) s->workers.emplace_back([s] { s->run(); });
    } catch (...) {
        {
            std::lock_guard<std::mutex> g(s->mu);
            s->stop = true;
        }
        s->cv_work.notify_all();
        for (auto& t : s->workers) t.join();
        delete s;
        return NWV_ERR_OOM;
    }
    *out = s;
    return NWV_OK;
}
template <class Committee>
int set_committee(nwv_service* svc, const Committee* committee, bool bls) {
    if (!svc || !committee || !committee->keys || !committee->stakes || svc->bls != bls) return NWV_ERR_ARG;
    try {
        auto c = std::make_shared<const OwnedCommittee>(*committee);
        std::lock_guard<std::mutex> g(svc->mu);
        svc->com = std::move(c);
    } catch (...) {
        return NWV_ERR_OOM;
    }
    return NWV_OK;
}
}  // namespace

extern "C" {

int nwv_service_create(nwv_ctx* ctx, const nwv_committee* committee, size_t max_batch, uint32_t max_wait_us,
                       nwv_service** out) {
    return service_create(ctx, committee, max_batch, max_wait_us, false, out);
}
int nwv_service_create_bls(nwv_ctx* ctx, const nwv_bls_committee* committee, size_t max_batch, uint32_t max_wait_us,
                           nwv_service** out) {
    return service_create(ctx, committee, max_batch, max_wait_us, true, out);
}
int nwv_service_set_committee(nwv_service* svc, const nwv_committee* committee) {
    return set_committee(svc, committee, false);
}
int nwv_service_set_committee_bls(nwv_service* svc, const nwv_bls_committee* committee) {
    return set_committee(svc, committee, true);
}

int nwv_service_submit_header(nwv_service* svc, const nwv_header* h, nwv_done_fn done, void* user) {
    if (!svc || svc->bls || !header_ok(h)) return NWV_ERR_ARG;
    try {
        auto it = std::make_unique<Item>();
        it->kind = HEADER;
        it->bytes.resize(header_bytes(*h));
        it->words.resize(h->n_payload);
        copy_header(it.get(), *h, 0, 0, it->h);
        return svc->submit(std::move(it), done, user);
    } catch (...) {
        return NWV_ERR_OOM;
    }
}

int nwv_service_submit_vote(nwv_service* svc, const nwv_vote* v, nwv_done_fn done, void* user) {
    if (!svc || svc->bls || !v || !v->id || !v->origin || !v->author || !v->signature) return NWV_ERR_ARG;
    try {
        auto it = std::make_unique<Item>();
        it->kind = VOTE;
        it->bytes.resize(32 * 3 + 64);
        uint8_t* b = it->bytes.data();
        std::memcpy(b, v->id, 32);
        std::memcpy(b + 32, v->origin, 32);
        std::memcpy(b + 64, v->author, 32);
        std::memcpy(b + 96, v->signature, 64);
        it->v = nwv_vote{b, v->round, v->epoch, b + 32, b + 64, b + 96};
        return svc->submit(std::move(it), done, user);
    } catch (...) {
        return NWV_ERR_OOM;
    }
}

int nwv_service_submit_certificate(nwv_service* svc, const nwv_certificate* c, nwv_done_fn done, void* user) {
    if (!svc || svc->bls || !c || !header_ok(&c->header) || (c->n_signed && !c->signed_authorities) ||
        (c->n_sigs && !c->aggregated_signature))
        return NWV_ERR_ARG;
    try {
        auto it = std::make_unique<Item>();
        it->kind = CERT;
        const size_t hb = header_bytes(c->header);
        it->bytes.resize(hb + 64 * c->n_sigs);
        it->words.resize(c->header.n_payload + c->n_signed);
        copy_header(it.get(), c->header, 0, 0, it->c.header);
        uint32_t* sa = it->words.data() + c->header.n_payload;
        if (c->n_signed) std::memcpy(sa, c->signed_authorities, 4 * c->n_signed);
        uint8_t* sg = it->bytes.data() + hb;
        if (c->n_sigs) std::memcpy(sg, c->aggregated_signature, 64 * c->n_sigs);
        it->c.n_signed = c->n_signed;
        it->c.signed_authorities = c->n_signed ? sa : nullptr;
        it->c.n_sigs = c->n_sigs;
        it->c.aggregated_signature = c->n_sigs ? sg : nullptr;
        return svc->submit(std::move(it), done, user);
    } catch (...) {
        return NWV_ERR_OOM;
    }
}

// ---- BLS12-381 items (96-byte keys, 48-byte signatures; a certificate's aggregate is one
// 48-byte G1 point or NULL for AggregateSignature::default())
int nwv_service_submit_bls_header(nwv_service* svc, const nwv_bls_header* h, nwv_done_fn done, void* user) {
    if (!svc || !svc->bls || !header_ok(h)) return NWV_ERR_ARG;
    try {
        auto it = std::make_unique<Item>();
        it->kind = HEADER;
        it->bytes.resize(bls_header_bytes(*h));
        it->words.resize(h->n_payload);
        copy_bls_header(it.get(), *h, 0, 0, it->bh);
        return svc->submit(std::move(it), done, user);
    } catch (...) {
        return NWV_ERR_OOM;
    }
}

int nwv_service_submit_bls_vote(nwv_service* svc, const nwv_bls_vote* v, nwv_done_fn done, void* user) {
    if (!svc || !svc->bls || !v || !v->id || !v->origin || !v->author || !v->signature) return NWV_ERR_ARG;
    try {
        auto it = std::make_unique<Item>();
        it->kind = VOTE;
        it->bytes.resize(32 + 96 + 96 + 48);
        uint8_t* b = it->bytes.data();
        std::memcpy(b, v->id, 32);
        std::memcpy(b + 32, v->origin, 96);
        std::memcpy(b + 128, v->author, 96);
        std::memcpy(b + 224, v->signature, 48);
        it->bv = nwv_bls_vote{b, v->round, v->epoch, b + 32, b + 128, b + 224};
        return svc->submit(std::move(it), done, user);
    } catch (...) {
        return NWV_ERR_OOM;
    }
}

int nwv_service_submit_bls_certificate(nwv_service* svc, const nwv_bls_certificate* c, nwv_done_fn done,
                                       void* user) {
    if (!svc || !svc->bls || !c || !header_ok(&c->header) || (c->n_signed && !c->signed_authorities))
        return NWV_ERR_ARG;
    try {
        auto it = std::make_unique<Item>();
        it->kind = CERT;
        const size_t hb = bls_header_bytes(c->header);
        it->bytes.resize(hb + 48);
        it->words.resize(c->header.n_payload + c->n_signed);
        copy_bls_header(it.get(), c->header, 0, 0, it->bc.header);
        uint32_t* sa = it->words.data() + c->header.n_payload;
        if (c->n_signed) std::memcpy(sa, c->signed_authorities, 4 * c->n_signed);
        uint8_t* sg = it->bytes.data() + hb;
        if (c->aggregated_signature) std::memcpy(sg, c->aggregated_signature, 48);
        it->bc.n_signed = c->n_signed;
        it->bc.signed_authorities = c->n_signed ? sa : nullptr;
        it->bc.aggregated_signature = c->aggregated_signature ? sg : nullptr;
        return svc->submit(std::move(it), done, user);
    } catch (...) {
        return NWV_ERR_OOM;
    }
}

int nwv_service_verify_bls_header(nwv_service* svc, const nwv_bls_header* h, int32_t* result) {
    return verify_blocking(svc, [&](Waiter* w) { return nwv_service_submit_bls_header(svc, h, waiter_done, w); },
                           result);
}
int nwv_service_verify_bls_vote(nwv_service* svc, const nwv_bls_vote* v, int32_t* result) {
    return verify_blocking(svc, [&](Waiter* w) { return nwv_service_submit_bls_vote(svc, v, waiter_done, w); },
                           result);
}
int nwv_service_verify_bls_certificate(nwv_service* svc, const nwv_bls_certificate* c, int32_t* result) {
    return verify_blocking(svc, [&](Waiter* w) { return nwv_service_submit_bls_certificate(svc, c, waiter_done, w); },
                           result);
}

int nwv_service_verify_header(nwv_service* svc, const nwv_header* h, int32_t* result) {
    return verify_blocking(svc, [&](Waiter* w) { return nwv_service_submit_header(svc, h, waiter_done, w); }, result);
}
int nwv_service_verify_vote(nwv_service* svc, const nwv_vote* v, int32_t* result) {
    return verify_blocking(svc, [&](Waiter* w) { return nwv_service_submit_vote(svc, v, waiter_done, w); }, result);
}
int nwv_service_verify_certificate(nwv_service* svc, const nwv_certificate* c, int32_t* result) {
    return verify_blocking(svc, [&](Waiter* w) { return nwv_service_submit_certificate(svc, c, waiter_done, w); },
                           result);
}

int nwv_service_flush(nwv_service* svc) {
    if (!svc) return NWV_ERR_ARG;
    WaitEdge edge(svc);
    if (edge.rc) return edge.rc;
    std::unique_lock<std::mutex> lk(svc->mu);
    const uint64_t upto = svc->next_seq;
    svc->flush_upto = std::max(svc->flush_upto, upto);
    svc->cv_work.notify_all();
    svc->cv_done.wait(lk, [&] { return svc->open.empty() || *svc->open.begin() >= upto; });
    return NWV_OK;
}

int nwv_service_set_idle(nwv_service* svc, uint32_t idle_us) {
    if (!svc) return NWV_ERR_ARG;
    {
        std::lock_guard<std::mutex> g(svc->mu);
        svc->idle = std::chrono::microseconds(idle_us);
    }
    svc->cv_work.notify_all();
    return NWV_OK;
}

int nwv_service_stats(nwv_service* svc, uint64_t out[6]) {
    if (!svc || !out) return NWV_ERR_ARG;
    std::lock_guard<std::mutex> g(svc->mu);
    std::memcpy(out, svc->stats, sizeof(svc->stats));
    return NWV_OK;
}

void nwv_service_free(nwv_service* svc) {
    if (!svc) return;
    {
        std::lock_guard<std::mutex> g(svc->mu);
        svc->stop = true;
    }
    svc->cv_work.notify_all();
    for (auto& t : svc->workers) t.join();
    delete svc;
}

}  // extern "C"
