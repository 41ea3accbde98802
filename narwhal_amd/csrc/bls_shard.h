// bls_shard.h -- BLS12-381 calls over a multi-device context (host code, SURVEY §8 e).
//
// The reference verifies certificates independently (validate_certificates,
// primary/src/block_synchronizer/responses.rs:115-129; the Core's queued headers and votes), so a
// nwv_bls_verify_many call splits its items by index into contiguous ranges, one per device, and
// every range's statuses land at their own indices: no cross-device exchange, exactly as the
// Ed25519 calls shard (nwv_host.hip for_shards).  Small calls stay on one device: each item's
// pairing check is latency-bound on one wave, so spreading 100 items over 8 devices buys nothing
// and costs a host thread per device.
#pragma once
#include <cstddef>
#include <thread>
#include <utility>
#include <vector>

namespace nwv {

// [lo, hi) item ranges over at most ndev devices, near-equal, each of at least min_per items (so a
// call of n < 2 min_per items is one range on device 0); range k goes to device k
inline std::vector<std::pair<size_t, size_t>> bls_shard_ranges(size_t n, size_t ndev, size_t min_per) {
    std::vector<std::pair<size_t, size_t>> r;
    if (n == 0) return r;
    if (min_per == 0) min_per = 1;
    size_t k = n / min_per;
    if (k > ndev) k = ndev;
    if (k == 0) k = 1;
    for (size_t j = 0; j < k; j++) r.push_back({n * j / k, n * (j + 1) / k});
    return r;
}

// fn(k, lo, hi) for every range, range k on its own host thread (range 0 on the caller's); the
// first nonzero return code in range order
template <class Fn>
int bls_for_ranges(const std::vector<std::pair<size_t, size_t>>& ranges, Fn fn) {
    std::vector<int> rcs(ranges.size(), 0);
    std::vector<std::thread> th;
    for (size_t k = 1; k < ranges.size(); k++) {
        auto run = [&, k]() { rcs[k] = fn(k, ranges[k].first, ranges[k].second); };
        try {
            th.emplace_back(run);
        } catch (...) {  // no host thread: run this range inline (never throw across the C ABI)
            run();
        }
    }
    if (!ranges.empty()) rcs[0] = fn(0, ranges[0].first, ranges[0].second);
    for (auto& t : th) t.join();
    for (int rc : rcs)
        if (rc) return rc;
    return 0;
}

}  // namespace nwv
