// stage_args.h -- small host-to-device staging through kernel arguments (gfx950).
//
// A per-call path's inputs are a few hundred bytes to a few KB (a certificate's signatures and
// preimages, one BLS verification's signature, message and key index).  hipMemcpyAsync sends them
// through a copy engine, and the first kernel then waits on the hand-off from that engine to the
// compute queue (~30 us between a 4 us copy and the next kernel in the single-verify trace).  A
// kernel whose arguments carry the bytes puts them in place on the compute queue itself: the
// runtime writes the arguments with the dispatch, so there is no copy engine on the path.
// NWV_NO_ARG_STAGE=1 keeps the async copy (A/B).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace nwv_stage {

constexpr size_t STAGE_ARG_BYTES = 3584;  // HIP kernel arguments are limited to 4 KB
struct StageArgs {
    uint8_t* dst;
    uint32_t bytes;
    uint32_t pad_;
    uint32_t w[STAGE_ARG_BYTES / 4];
};

// dst[0, bytes) <- the argument words (dst 4-byte aligned; the last partial word byte by byte)
static __global__ void __launch_bounds__(256) k_stage_args(StageArgs a) {
    const uint32_t nw = a.bytes >> 2;
    uint32_t* d = reinterpret_cast<uint32_t*>(a.dst);
    const uint32_t* s = a.w;
    for (uint32_t i = threadIdx.x; i < nw; i += 256) d[i] = s[i];
    const uint32_t tail = a.bytes & 3u;
    if (threadIdx.x < tail) a.dst[4 * nw + threadIdx.x] = (uint8_t)(s[nw] >> (8 * threadIdx.x));
}

inline bool arg_stage_on() {
    static const bool on = [] {
        const char* e = std::getenv("NWV_NO_ARG_STAGE");
        return !(e && std::atoi(e) != 0);
    }();
    return on;
}

// dst <- src[0, bytes) on `stream`, in stream order: through k_stage_args when the bytes fit its
// arguments, else one hipMemcpyAsync (src must then stay valid until the copy has run, as for any
// async copy; the argument form copies src at the call)
inline hipError_t stage_h2d(void* dst, const void* src, size_t bytes, hipStream_t stream) {
    if (!bytes) return hipSuccess;
    if (bytes <= STAGE_ARG_BYTES && arg_stage_on() && (reinterpret_cast<uintptr_t>(dst) & 3u) == 0) {
        StageArgs a;
        a.dst = static_cast<uint8_t*>(dst);
        a.bytes = (uint32_t)bytes;
        a.pad_ = 0;
        if (bytes & 3u) a.w[bytes >> 2] = 0;
        std::memcpy(a.w, src, bytes);
        hipLaunchKernelGGL(k_stage_args, dim3(1), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream);
}

}  // namespace nwv_stage
