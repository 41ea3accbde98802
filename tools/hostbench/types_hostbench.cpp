// Host-side cost of nwv_verify_mixed_many (the types layer's C++ around the GPU calls) on a C5
// round (100-node committee: 100 headers with 67 parents, 100 certificates x (1 + 67)
// signatures, 99 votes).  The two engine calls are stubbed (a 32-byte FNV-style digest and an
// all-valid batch verdict), so this measures only the host work; no GPU is needed.
//   g++ -O2 -std=c++17 -o /tmp/types_hostbench tools/hostbench/types_hostbench.cpp narwhal_amd/csrc/nwv_types.cpp
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/nwv_types.h"

extern "C" int nwv_blake2b256_many(nwv_ctx*, size_t n, const uint8_t* base, const uint64_t* off,
                                   const uint64_t* len, uint8_t* out) {
    for (size_t i = 0; i < n; i++) {
        uint64_t h = 1469598103934665603ull;  // cheap stand-in: 8 bytes per step
        for (uint64_t k = 0; k + 8 <= len[i]; k += 8) {
            uint64_t w;
            std::memcpy(&w, base + off[i] + k, 8);
            h = (h ^ w) * 1099511628211ull;
        }
        for (uint64_t k = len[i] & ~7ull; k < len[i]; k++) h = (h ^ base[off[i] + k]) * 1099511628211ull;
        for (int w = 0; w < 4; w++) std::memcpy(out + 32 * i + 8 * w, &(h += w), 8);
    }
    return NWV_OK;
}
extern "C" int nwv_ed25519_verify_batch_keyed_digests(nwv_ctx* ctx, size_t n_pre, const uint8_t* base,
                                                      const uint64_t* off, const uint64_t* len, uint8_t* dig,
                                                      size_t, const uint8_t*, size_t n, const uint32_t*,
                                                      const uint8_t*, const uint32_t*, const uint8_t*,
                                                      int* all_valid, uint64_t* bits) {
    nwv_blake2b256_many(ctx, n_pre, base, off, len, dig);
    *all_valid = 1;
    if (bits) std::memset(bits, 0xff, 8 * ((n + 63) / 64));
    return NWV_OK;
}

// the BLS12-381 layer's engine calls (nwv_types.cpp links them; this bench times the Ed25519 path)
extern "C" int nwv_bls_keycache_register(nwv_ctx*, size_t, const uint8_t*) { return NWV_OK; }
extern "C" int nwv_keycache_register(nwv_ctx*, size_t, const uint8_t*) { return NWV_OK; }
extern "C" int nwv_bls_verify_many(nwv_ctx*, size_t, const uint8_t*, size_t n, const uint8_t*, const uint32_t*,
                                   const uint32_t*, const uint32_t*, const uint8_t*, const uint64_t*, const uint32_t*,
                                   const uint8_t*, size_t, int32_t* status) {
    std::memset(status, 0, 4 * n);
    return NWV_OK;
}
extern "C" int nwv_bls_aggregate(nwv_ctx*, size_t, const uint8_t*, uint8_t out48[48], int32_t*) {
    std::memset(out48, 0, 48);
    return NWV_OK;
}

int main() {
    const size_t N = 100, Q = 67;
    static int dummy;
    nwv_ctx* ctx = reinterpret_cast<nwv_ctx*>(&dummy);  // opaque, never dereferenced by the stubs
    std::vector<uint8_t> keys(32 * N);
    for (size_t i = 0; i < N; i++) keys[32 * i] = (uint8_t)i, keys[32 * i + 1] = 7;
    std::vector<uint64_t> stakes(N, 1);
    std::vector<uint32_t> nw(N, 4), wids = {0, 1, 2, 3};
    std::vector<const uint32_t*> wp(N, wids.data());
    nwv_committee c{};
    c.n = N;
    c.keys = keys.data();
    c.stakes = stakes.data();
    c.epoch = 0;
    c.n_workers = nw.data();
    c.worker_ids = wp.data();
    std::vector<uint8_t> parents(32 * Q), pay(32), sig(64, 1), sigs(64 * Q, 2);
    for (size_t i = 0; i < parents.size(); i++) parents[i] = (uint8_t)(i * 13);
    std::vector<uint32_t> pw = {0};
    std::vector<std::vector<uint8_t>> ids(N, std::vector<uint8_t>(32));
    std::vector<nwv_header> hs(N);
    for (size_t a = 0; a < N; a++) {
        nwv_header& h = hs[a];
        std::memset(&h, 0, sizeof h);
        h.author = keys.data() + 32 * a;
        h.round = 1;
        h.n_payload = 1;
        h.payload_digests = pay.data();
        h.payload_workers = pw.data();
        h.n_parents = Q;
        h.parents = parents.data();
        h.signature = sig.data();
        h.id = ids[a].data();
        nwv_header_digest(ctx, &h, ids[a].data());
    }
    std::vector<uint32_t> signers(Q);
    std::vector<nwv_certificate> cs(N);
    for (size_t a = 0; a < N; a++) {
        std::memset(&cs[a], 0, sizeof cs[a]);
        cs[a].header = hs[a];
        for (size_t k = 0; k < Q; k++) signers[k] = (uint32_t)k;
        cs[a].n_signed = Q;
        cs[a].signed_authorities = signers.data();
        cs[a].n_sigs = Q;
        cs[a].aggregated_signature = sigs.data();
    }
    std::vector<nwv_vote> vs(N - 1);
    for (size_t v = 0; v + 1 < N; v++) {
        std::memset(&vs[v], 0, sizeof vs[v]);
        vs[v].id = ids[0].data();
        vs[v].round = 1;
        vs[v].origin = keys.data();
        vs[v].author = keys.data() + 32 * (v + 1);
        vs[v].signature = sig.data();
    }
    std::vector<int32_t> hr(N), vr(N), cr(N);
    double best = 1e9, sum = 0;
    const int reps = 200;
    for (int r = 0; r < reps + 5; r++) {
        auto t0 = std::chrono::steady_clock::now();
        int rc = nwv_verify_mixed_many(ctx, &c, N, hs.data(), hr.data(), N - 1, vs.data(), vr.data(), N, cs.data(),
                                       cr.data());
        auto t1 = std::chrono::steady_clock::now();
        if (rc) return std::printf("rc %d\n", rc), 1;
        for (size_t i = 0; i < N; i++)
            if (hr[i] || cr[i] || (i + 1 < N && vr[i])) return std::printf("verdict %zu: %d %d\n", i, hr[i], cr[i]), 1;
        const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
        if (r >= 5) { best = std::min(best, us); sum += us; }
    }
    std::printf("{\"host_us_per_round_mean\": %.1f, \"host_us_per_round_min\": %.1f}\n", sum / reps, best);
    return 0;
}
