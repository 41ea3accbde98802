// svcbench.cpp -- native drivers of the C5 service leg (bench.py configs.C5.service): the batching
// service (include/nwv_service.h) and the Core loop's drain-then-verify consumer, timed from C++
// threads as a Rust caller runs them (rust/narwhal-gpu-crypto/src/core_drain.rs, Core::run
// primary/src/core.rs:614-714), so the figures carry no Python queue or ctypes cost.
// Bench tooling, not product: built as tools/libsvcbench.so against narwhal_amd/lib/libnwv.so.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../include/nwv.h"
#include "../include/nwv_service.h"
#include "../include/nwv_types.h"

namespace {
using clk = std::chrono::steady_clock;
double ms_since(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

struct Msgs {
    size_t nh, nv, nc;
    const nwv_header* h;
    const nwv_vote* v;
    const nwv_certificate* c;
    size_t n() const { return nh + nv + nc; }
};

struct Done {
    std::atomic<size_t> left{0};
    std::vector<clk::time_point> t_done;
    std::vector<int32_t> code;
    std::mutex mu;
    std::condition_variable cv;
};
struct Slot {
    Done* d;
    size_t i;
};
void on_done(void* user, int32_t result) {
    Slot* s = static_cast<Slot*>(user);
    s->d->t_done[s->i] = clk::now();
    s->d->code[s->i] = result;
    if (s->d->left.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(s->d->mu);
        s->d->cv.notify_all();
    }
}
}  // namespace

extern "C" {

// rounds + 1 rounds (the first warms up): `threads` submitter threads hand every message of the
// round to one service (message i by thread i % threads, asynchronously), and the round ends when
// every completion has fired.  round_ms[rounds]; submit_ms[rounds] (until every submit returned);
// lat_ms[rounds * n] (submission -> own completion); stats[6] = nwv_service_stats after the run.  Returns 0, or the first nonzero
// result code / negative error seen.
int svcbench_service(nwv_ctx* ctx, const nwv_committee* com, size_t nh, const nwv_header* h, size_t nv,
                     const nwv_vote* v, size_t nc, const nwv_certificate* c, int threads, int rounds,
                     size_t max_batch, uint32_t max_wait_us, uint32_t idle_us, double* round_ms, double* submit_ms,
                     double* lat_ms, uint64_t* stats) {
    const Msgs m{nh, nv, nc, h, v, c};
    const size_t n = m.n();
    nwv_service* svc = nullptr;
    int rc = nwv_service_create(ctx, com, max_batch, max_wait_us, &svc);
    if (rc) return rc;
    if (idle_us) nwv_service_set_idle(svc, idle_us);
    Done d;
    d.t_done.resize(n);
    d.code.resize(n);
    std::vector<Slot> slots(n);
    for (size_t i = 0; i < n; i++) slots[i] = Slot{&d, i};
    std::vector<clk::time_point> t_sub(n);
    // persistent submitter threads, released together at the start of every round
    std::mutex gm;
    std::condition_variable gcv, jcv;
    int round_go = -1, joined = 0;
    bool quit = false;
    std::atomic<int> err{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++)
        ts.emplace_back([&, t] {
            for (int r = 0;; r++) {
                {
                    std::unique_lock<std::mutex> g(gm);
                    gcv.wait(g, [&] { return round_go >= r || quit; });
                    if (quit) return;
                }
                for (size_t i = (size_t)t; i < n; i += (size_t)threads) {
                    t_sub[i] = clk::now();
                    int e;
                    if (i < nh) e = nwv_service_submit_header(svc, &h[i], on_done, &slots[i]);
                    else if (i < nh + nv) e = nwv_service_submit_vote(svc, &v[i - nh], on_done, &slots[i]);
                    else e = nwv_service_submit_certificate(svc, &c[i - nh - nv], on_done, &slots[i]);
                    if (e) {
                        err = e;
                        on_done(&slots[i], e);
                    }
                }
                std::lock_guard<std::mutex> g(gm);
                if (++joined == threads) jcv.notify_all();
            }
        });
    int bad = 0;
    for (int r = 0; r <= rounds && !bad; r++) {
        d.left = n;
        const auto t0 = clk::now();
        {
            std::lock_guard<std::mutex> g(gm);
            joined = 0;
            round_go = r;
        }
        gcv.notify_all();
        clk::time_point ts_end;
        {
            std::unique_lock<std::mutex> g(gm);
            jcv.wait(g, [&] { return joined == threads; });
            ts_end = clk::now();
        }
        {
            std::unique_lock<std::mutex> g(d.mu);
            d.cv.wait(g, [&] { return d.left.load() == 0; });
        }
        const auto t1 = clk::now();
        if (err) bad = err;
        for (size_t i = 0; i < n && !bad; i++)
            if (d.code[i]) bad = d.code[i];
        if (r) {
            round_ms[r - 1] = ms_since(t0, t1);
            submit_ms[r - 1] = ms_since(t0, ts_end);
            for (size_t i = 0; i < n; i++) lat_ms[(size_t)(r - 1) * n + i] = ms_since(t_sub[i], d.t_done[i]);
        }
    }
    {
        std::lock_guard<std::mutex> g(gm);
        quit = true;
    }
    gcv.notify_all();
    for (auto& th : ts) th.join();
    nwv_service_stats(svc, stats);
    nwv_service_free(svc);
    return bad;
}

// rounds + 1 rounds (the first warms up) of the Core loop's drain pattern (core_drain.rs): a
// producer thread delivers the round's messages one at a time into a channel; the consumer (the
// calling thread) takes a message, then whatever else is queued -- at most max_items, waiting until
// max_wait_us after the first while fewer than min_items are taken, then at most idle_us for each
// next one (0: none) -- and verifies the lot with ONE nwv_verify_mixed_many call.  round_ms[rounds]; lat_ms[rounds * n] (enqueue -> the
// verdict of its call); calls[rounds], largest[rounds] engine calls and largest flush per round.
int svcbench_drain(nwv_ctx* ctx, const nwv_committee* com, size_t nh, const nwv_header* h, size_t nv,
                   const nwv_vote* v, size_t nc, const nwv_certificate* c, int rounds, size_t max_items,
                   uint32_t max_wait_us, size_t min_items, uint32_t idle_us, double* round_ms, double* lat_ms,
                   uint32_t* calls, uint32_t* largest) {
    const size_t n = nh + nv + nc;
    if (max_items < 1) return NWV_ERR_ARG;
    struct Item {
        clk::time_point t;
        size_t i;
    };
    std::deque<Item> q;
    std::mutex mu;
    std::condition_variable cv, go_cv;
    int go_round = -1;
    bool stop = false;
    std::thread prod([&] {
        for (int r = 0; r <= rounds; r++) {
            {
                std::unique_lock<std::mutex> g(mu);
                go_cv.wait(g, [&] { return go_round >= r || stop; });
                if (stop) return;
            }
            for (size_t i = 0; i < n; i++) {
                {
                    std::lock_guard<std::mutex> g(mu);
                    q.push_back(Item{clk::now(), i});
                }
                cv.notify_one();
            }
        }
    });
    std::vector<nwv_header> bh;
    std::vector<nwv_vote> bv;
    std::vector<nwv_certificate> bc;
    std::vector<int32_t> rh, rv, rcv;
    std::vector<Item> batch;
    int bad = 0;
    for (int r = 0; r <= rounds && !bad; r++) {
        const auto t0 = clk::now();
        {
            std::lock_guard<std::mutex> g(mu);
            go_round = r;
        }
        go_cv.notify_all();
        size_t seen = 0;
        uint32_t ncall = 0, big = 0;
        while (seen < n && !bad) {
            batch.clear();
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return !q.empty(); });
                batch.push_back(q.front());
                q.pop_front();
                const auto deadline = clk::now() + std::chrono::microseconds(max_wait_us);
                while (batch.size() < max_items) {
                    if (!q.empty()) {
                        batch.push_back(q.front());
                        q.pop_front();
                        continue;
                    }
                    // below min_items wait until the deadline; past it at most idle_us for more
                    auto until = deadline;
                    if (batch.size() >= min_items) until = std::min(until, clk::now() + std::chrono::microseconds(idle_us));
                    if (clk::now() >= until) break;
                    if (!cv.wait_until(g, until, [&] { return !q.empty(); })) break;
                }
            }
            bh.clear();
            bv.clear();
            bc.clear();
            for (const Item& it : batch) {
                if (it.i < nh) bh.push_back(h[it.i]);
                else if (it.i < nh + nv) bv.push_back(v[it.i - nh]);
                else bc.push_back(c[it.i - nh - nv]);
            }
            rh.assign(bh.size(), -1);
            rv.assign(bv.size(), -1);
            rcv.assign(bc.size(), -1);
            const int e = nwv_verify_mixed_many(ctx, com, bh.size(), bh.data(), rh.data(), bv.size(), bv.data(),
                                                rv.data(), bc.size(), bc.data(), rcv.data());
            const auto t1 = clk::now();
            if (e) bad = e;
            for (int32_t x : rh) bad = bad ? bad : x;
            for (int32_t x : rv) bad = bad ? bad : x;
            for (int32_t x : rcv) bad = bad ? bad : x;
            if (r)
                for (const Item& it : batch) lat_ms[(size_t)(r - 1) * n + it.i] = ms_since(it.t, t1);
            seen += batch.size();
            ncall++;
            big = std::max(big, (uint32_t)batch.size());
        }
        if (r) {
            round_ms[r - 1] = ms_since(t0, clk::now());
            calls[r - 1] = ncall;
            largest[r - 1] = big;
        }
    }
    {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
    }
    go_cv.notify_all();
    prod.join();
    return bad;
}

}  // extern "C"
