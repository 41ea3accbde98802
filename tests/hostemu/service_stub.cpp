// Test infrastructure: a stand-in for the engine's nwv_verify_mixed_many so that the batching
// service (narwhal_amd/csrc/nwv_service.cpp) can be tested on the CPU.  Rule: an item is
// NWV_DAG_INVALID_EPOCH if its epoch differs from the committee's, NWV_DAG_INVALID_SIGNATURE if
// the first byte of its (header) signature is 0xFF, else NWV_DAG_OK.  Records the batch sizes.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>

#include "../../include/nwv_service.h"

static std::atomic<long> g_calls{0}, g_items{0}, g_max{0}, g_delay_us{0}, g_fail{0};

extern "C" {

int nwv_verify_mixed_many(nwv_ctx*, const nwv_committee* c, size_t nh, const nwv_header* h, int32_t* rh, size_t nv,
                          const nwv_vote* v, int32_t* rv, size_t nc, const nwv_certificate* cs, int32_t* rc) {
    g_calls++;
    const long n = (long)(nh + nv + nc);
    g_items += n;
    long m = g_max.load();
    while (n > m && !g_max.compare_exchange_weak(m, n)) {
    }
    if (g_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(g_delay_us.load()));
    if (g_fail) return NWV_ERR_HIP;
    auto code = [&](uint64_t epoch, const uint8_t* sig) {
        if (epoch != c->epoch) return NWV_DAG_INVALID_EPOCH;
        return sig[0] == 0xFF ? NWV_DAG_INVALID_SIGNATURE : NWV_DAG_OK;
    };
    for (size_t i = 0; i < nh; i++) rh[i] = code(h[i].epoch, h[i].signature);
    for (size_t i = 0; i < nv; i++) rv[i] = code(v[i].epoch, v[i].signature);
    for (size_t i = 0; i < nc; i++) rc[i] = code(cs[i].header.epoch, cs[i].header.signature);
    return NWV_OK;
}

// the BLS12-381 layer's stand-in, same rule (a certificate's code from its header's signature;
// an aggregate holding no signature -> InvalidSignature)
int nwv_bls_verify_mixed_many(nwv_ctx*, const nwv_bls_committee* c, size_t nh, const nwv_bls_header* h, int32_t* rh,
                              size_t nv, const nwv_bls_vote* v, int32_t* rv, size_t nc, const nwv_bls_certificate* cs,
                              int32_t* rc) {
    g_calls++;
    const long n = (long)(nh + nv + nc);
    g_items += n;
    long m = g_max.load();
    while (n > m && !g_max.compare_exchange_weak(m, n)) {
    }
    if (g_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(g_delay_us.load()));
    if (g_fail) return NWV_ERR_HIP;
    auto code = [&](uint64_t epoch, const uint8_t* sig) {
        if (epoch != c->epoch) return NWV_DAG_INVALID_EPOCH;
        return sig[0] == 0xFF ? NWV_DAG_INVALID_SIGNATURE : NWV_DAG_OK;
    };
    for (size_t i = 0; i < nh; i++) rh[i] = code(h[i].epoch, h[i].signature);
    for (size_t i = 0; i < nv; i++) rv[i] = code(v[i].epoch, v[i].signature);
    for (size_t i = 0; i < nc; i++)
        rc[i] = cs[i].aggregated_signature ? code(cs[i].header.epoch, cs[i].header.signature) : NWV_DAG_INVALID_SIGNATURE;
    return NWV_OK;
}

void stub_reset(long delay_us, long fail) {
    g_calls = 0;
    g_items = 0;
    g_max = 0;
    g_delay_us = delay_us;
    g_fail = fail;
}
void stub_counts(long* out) {
    out[0] = g_calls;
    out[1] = g_items;
    out[2] = g_max;
}
}
