// shard.h -- how an Ed25519 / BLAKE2b call splits over a multi-device context (host code,
// SURVEY §8 e).
//
// The reference verifies signatures independently of one another (ed25519-consensus batches are
// a random linear combination per call; validate_certificates checks each certificate,
// primary/src/block_synchronizer/responses.rs:115-138), so a call over several devices splits its
// items by index into contiguous ranges, one per device, and each range's verdict lands at its own
// indices: no cross-device exchange.  Two rules beyond that:
//   * Ed25519 ranges start on multiples of 64, so every range owns whole 64-bit verdict words
//     (verdict_bits + lo / 64) and no two host threads ever write the same word;
//   * a range holds at least min_per items.  A batch MSM's tail is a latency-bound chain of
//     ~0.12 ms whatever the batch size, so eight 128-signature MSMs on eight devices (plus their
//     host threads) are slower than one 1,024-signature MSM on one: a call of fewer than
//     2 min_per items stays on device 0.
#pragma once
#include <cstddef>
#include <thread>
#include <utility>
#include <vector>

namespace nwv {

// [lo, hi) ranges over at most ndev devices: contiguous, in order, near-equal (counted in units of
// `align` items), every start a multiple of align, each range at least min_per items (except that a
// call of n < 2 min_per items is one range).  Range k runs on device k.
inline std::vector<std::pair<size_t, size_t>> shard_ranges(size_t n, size_t ndev, size_t min_per, size_t align) {
    std::vector<std::pair<size_t, size_t>> r;
    if (n == 0) return r;
    if (ndev == 0) ndev = 1;
    if (min_per == 0) min_per = 1;
    if (align == 0) align = 1;
    const size_t units = (n + align - 1) / align;
    size_t k = n / min_per;
    if (k > ndev) k = ndev;
    if (k > units) k = units;
    if (k == 0) k = 1;
    for (size_t j = 0; j < k; j++) {
        const size_t lo = (units * j / k) * align, hi = (units * (j + 1) / k) * align;
        r.push_back({lo < n ? lo : n, hi < n ? hi : n});
    }
    return r;
}

// Ed25519 calls: 64-aligned ranges (whole verdict words per range)
inline std::vector<std::pair<size_t, size_t>> ed_shard_ranges(size_t n, size_t ndev, size_t min_per) {
    return shard_ranges(n, ndev, min_per, 64);
}

// fn(k, lo, hi) for every range; range 0 on the calling thread, every other range on a host thread
// of its own.  Returns the first nonzero return code in range order.
template <class Fn>
int for_ranges(const std::vector<std::pair<size_t, size_t>>& ranges, Fn fn) {
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
