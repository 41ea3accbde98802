// ubench_row.hip -- latency of the row-parallel point doubling (fe_row.h) on one wave: the DPP
// operand form against the LDS operand form of the 16-lane field multiply.  Both must give the
// same limbs.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../narwhal_amd/csrc/fe_row.h"

using namespace nwv;

__global__ void __launch_bounds__(64) k_rowdbl(uint32_t* out, long long* cyc, int iters, int use_lds) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ uint32_t sc[192];
    rowf::RowConsts k = rowf::row_consts();
    k.sc = use_lds ? sc : nullptr;
    const uint32_t limb = __lane_id() & 15;
    // a valid-looking starting point: small limbs
    rowf::RowP3 d{limb * 7u + 3u, limb * 5u + 11u, limb == 0 ? 1u : 0u, limb * 3u + 1u};
    const long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < iters; i++) d = rowf::row_dbl(d, k);
    const long long t1 = clock64();
    if (__lane_id() < 16) {
        out[__lane_id()] = d.X;
        out[16 + __lane_id()] = d.Y;
        out[32 + __lane_id()] = d.Z;
    }
    if (__lane_id() == 0) *cyc = t1 - t0;
#endif
}

int main() {
    uint32_t* out;
    long long* cyc;
    hipMalloc(&out, 2 * 64 * 4);
    hipMalloc(&cyc, 2 * 8);
    const int iters = 2048;
    uint32_t h[2][48];
    long long c[2];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms[2];
    for (int v = 0; v < 2; v++) {
        hipLaunchKernelGGL(k_rowdbl, dim3(1), dim3(64), 0, 0, out + 64 * v, cyc + v, 16, v);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_rowdbl, dim3(1), dim3(64), 0, 0, out + 64 * v, cyc + v, iters, v);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[v], e0, e1);
        hipMemcpy(h[v], out + 64 * v, 48 * 4, hipMemcpyDeviceToHost);
        hipMemcpy(&c[v], cyc + v, 8, hipMemcpyDeviceToHost);
    }
    const bool same = std::memcmp(h[0], h[1], sizeof(h[0])) == 0;
    printf("{\"iters\": %d, \"dpp_us_per_dbl\": %.4f, \"lds_us_per_dbl\": %.4f, \"dpp_cycles_per_dbl\": %.1f, "
           "\"lds_cycles_per_dbl\": %.1f, \"same_limbs\": %s}\n",
           iters, ms[0] * 1e3 / iters, ms[1] * 1e3 / iters, (double)c[0] / iters, (double)c[1] / iters,
           same ? "true" : "false");
    return same ? 0 : 1;
}
