// The split of a BLS call over a multi-device context (narwhal_amd/csrc/bls_shard.h) with a stub
// per-device verifier: tests/test_bls_shard.py checks the ranges, that every range runs on its own
// device with its own item slice, and that the statuses land in item order.
#include <atomic>
#include <cstdint>
#include <mutex>
#include <set>
#include <thread>

#include "../../narwhal_amd/csrc/bls_shard.h"
#include "../../narwhal_amd/csrc/shard.h"

extern "C" {

// ranges of n items over ndev devices; returns the count, [lo, hi) pairs in out (2 x max_out)
int bst_ranges(uint64_t n, uint64_t ndev, uint64_t min_per, uint64_t* out, int max_out) {
    const auto r = nwv::bls_shard_ranges(n, ndev, min_per);
    for (size_t k = 0; k < r.size() && (int)k < max_out; k++) {
        out[2 * k] = r[k].first;
        out[2 * k + 1] = r[k].second;
    }
    return (int)r.size();
}

// a "verify_many" of n items over ndev stub devices: device k writes, for each item of its slice,
// status = item's value x 3 + 1 (from its slice pointer, as the real call's sigs + lo / status + lo)
// and dev[i] = k; keys_registered[k] counts the key registrations each device received (one per
// device, all devices, as nwv_bls_keycache_register).  Returns the number of distinct host threads
// that ran ranges, or -1 on a wrong rc propagation (fail_dev >= 0 makes that device return 7).
int bst_run(uint64_t n, uint64_t ndev, uint64_t min_per, const int32_t* items, int32_t* status, int32_t* dev,
            int32_t* keys_registered, int fail_dev) {
    std::vector<std::pair<size_t, size_t>> all;
    for (size_t k = 0; k < ndev; k++) all.push_back({k, k + 1});
    nwv::bls_for_ranges(all, [&](size_t k, size_t, size_t) {
        keys_registered[k] += 1;
        return 0;
    });
    std::mutex mu;
    std::set<std::thread::id> ids;
    const auto r = nwv::bls_shard_ranges(n, ndev, min_per);
    const int rc = nwv::bls_for_ranges(r, [&](size_t k, size_t lo, size_t hi) -> int {
        {
            std::lock_guard<std::mutex> g(mu);
            ids.insert(std::this_thread::get_id());
        }
        const int32_t* it = items + lo;
        int32_t* st = status + lo;
        for (size_t i = 0; i < hi - lo; i++) {
            st[i] = it[i] * 3 + 1;
            dev[lo + i] = (int32_t)k;
        }
        return (int)k == fail_dev ? 7 : 0;
    });
    const bool fail_expected = fail_dev >= 0 && (size_t)fail_dev < r.size();
    if ((rc != 0) != fail_expected || (fail_expected && rc != 7)) return -1;
    return (int)ids.size();
}

// Ed25519 split (shard.h, nwv_host.hip for_shards): ranges of n signatures over ndev devices
int bst_ed_ranges(uint64_t n, uint64_t ndev, uint64_t min_per, uint64_t* out, int max_out) {
    const auto r = nwv::ed_shard_ranges(n, ndev, min_per);
    for (size_t k = 0; k < r.size() && (int)k < max_out; k++) {
        out[2 * k] = r[k].first;
        out[2 * k + 1] = r[k].second;
    }
    return (int)r.size();
}

// The verdict-word merge of a sharded Ed25519 call, as batch_on_device does it for a shard: each
// range clears its own words at bits + lo / 64 (memset of (hi - lo + 63) / 64 words, as after an
// accepted MSM), then sets bit i for every index of its range whose valid[i] is set, with
// plain (non-atomic) word stores, all ranges on their own host threads at once.  Returns the
// number of ranges, or -1 if any range's start is not on a word boundary.
int bst_ed_merge(uint64_t n, uint64_t ndev, uint64_t min_per, const uint8_t* valid, uint64_t* bits, int reps) {
    const auto r = nwv::ed_shard_ranges(n, ndev, min_per);
    for (auto& x : r)
        if (x.first % 64) return -1;
    for (int rep = 0; rep < reps; rep++) {
        nwv::for_ranges(r, [&](size_t, size_t lo, size_t hi) -> int {
            uint64_t* w = bits + lo / 64;
            const size_t words = (hi - lo + 63) / 64;
            for (size_t j = 0; j < words; j++) w[j] = 0;
            for (size_t i = lo; i < hi; i++)
                if (valid[i]) w[(i - lo) >> 6] |= 1ULL << ((i - lo) & 63);
            return 0;
        });
    }
    return (int)r.size();
}

}  // extern "C"
