// ubench_row.hip -- latency of the row-parallel point doubling (fe_row.h) on one wave: the DPP
// operand form against the LDS operand form of the 16-lane field multiply.  Both must give the
// same limbs.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <unistd.h>
#include "../narwhal_amd/csrc/fe_row.h"
#include "../narwhal_amd/csrc/msm.h"

using namespace nwv;

template <int FORM>
__global__ void __launch_bounds__(64) k_rowdbl(uint32_t* out, long long* cyc, int iters) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ uint32_t sc[192];
    rowf::RowConsts k = rowf::row_consts();
    k.sc = FORM == 1 ? sc : nullptr;
    k.rot = FORM >= 2 ? FORM - 1 : 0;
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

// one wave, 4 rows each squaring its own element (the decompression power's loop, k_msm_prep's
// row form); nwaves > 1 puts that many such waves in one workgroup
template <int FORM>
__global__ void __launch_bounds__(256) k_rowsq(uint32_t* out, long long* cyc, int iters) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ uint32_t sc[4][192];
    rowf::RowConsts k = rowf::row_consts();
    k.sc = FORM == 1 ? sc[threadIdx.x >> 6] : nullptr;
    k.rot = FORM >= 2 ? FORM - 1 : 0;
    const uint32_t limb = __lane_id() & 15;
    uint32_t x = limb * 7u + 3u + (threadIdx.x >> 4);
    const long long t0 = clock64();
    x = rowf::row_sqn(x, iters, k);
    const long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) *cyc = t1 - t0;
#endif
}

// k_msm_prep's row decompression (msm_points_rows_block) on one wave, with cycle stamps after
// the lane-local prelude, the row power and the postlude
__global__ void __launch_bounds__(64) k_rowdec(uint32_t* out, long long* cyc, int target) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ uint32_t sh[64];
    if ((int)blockIdx.x != target) return;  // one working block; the others land on other CUs
    const int lane = threadIdx.x;
    const long long t0 = clock64();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t w[8];
    for (int i = 0; i < 8; i++) w[i] = 0x66666666u + (lane & 3) * 0x1111u;
    if (lane < 4) fe_to_limbs16(ge_decompress_pre(w), sh + 16 * lane);
    rowf::lds_order();
    const long long t1 = clock64();
    rowf::RowConsts k = rowf::row_consts();
    k.rot = 1;
    const uint32_t pw = rowf::row_pow_p58(sh[lane], k);
    rowf::lds_order();
    sh[lane] = pw;
    rowf::lds_order();
    const long long t2 = clock64();
    if (lane < 4) {
        ge_p3 P;
        const bool ok = ge_decompress_post(w, fe_from_limbs16(sh + 16 * lane), P);
        msm_store_point(out + 32 * lane, P);
        out[32 * lane + 31] = ok;
    }
    const long long t3 = clock64();
    const unsigned long long r3 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t2 - t1;
        cyc[2] = t3 - t2;
        cyc[3] = (long long)(r3 - r0);  // 100 MHz ticks
    }
#endif
}

int main() {
    uint32_t* out;
    long long* cyc;
    hipMalloc(&out, 4 * 64 * 4 + 512);
    hipMalloc(&cyc, 8 * 8);
    const int iters = 2048;
    uint32_t h[4][48];
    long long c[4];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms[4];
    for (int v = 0; v < 4; v++) {
        auto kern = v == 0 ? k_rowdbl<0> : v == 1 ? k_rowdbl<1> : v == 2 ? k_rowdbl<2> : k_rowdbl<3>;
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out + 64 * v, cyc + v, 16);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out + 64 * v, cyc + v, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[v], e0, e1);
        hipMemcpy(h[v], out + 64 * v, 48 * 4, hipMemcpyDeviceToHost);
        hipMemcpy(&c[v], cyc + v, 8, hipMemcpyDeviceToHost);
    }
    // squaring loops: 1 wave and 4 waves per workgroup (one per SIMD), rotation and LDS forms
    for (int v = 0; v < 4; v++) {
        const int nthr = (v & 1) ? 256 : 64;
        auto kern = v < 2 ? k_rowsq<2> : k_rowsq<1>;
        hipLaunchKernelGGL(kern, dim3(1), dim3(nthr), 0, 0, out, cyc, 16);
        hipDeviceSynchronize();
        float t;
        long long cc;
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(1), dim3(nthr), 0, 0, out, cyc, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&t, e0, e1);
        hipMemcpy(&cc, cyc, 8, hipMemcpyDeviceToHost);
        printf("{\"sq_form\": \"%s\", \"waves\": %d, \"us_per_sq\": %.4f, \"cycles_per_sq\": %.1f}\n",
               v < 2 ? "ror" : "lds", nthr / 64, t * 1e3 / iters, (double)cc / iters);
    }
    // (a) the same CU twice (warm instruction cache), (b) a block index the kernel never ran on
    // before: with 2,048 blocks it lands on a CU whose instruction cache holds none of this code
    for (int idle = 0; idle < 4; idle++) {
        long long cc[4];
        const int target = idle < 2 ? 0 : 1000 + 37 * idle;
        if (idle < 2) hipLaunchKernelGGL(k_rowdec, dim3(2048), dim3(64), 0, 0, out, cyc, target);
        hipDeviceSynchronize();
        if (idle == 1) usleep(20000);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_rowdec, dim3(2048), dim3(64), 0, 0, out, cyc, target);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float t;
        hipEventElapsedTime(&t, e0, e1);
        hipMemcpy(cc, cyc, 32, hipMemcpyDeviceToHost);
        const long long tot = cc[0] + cc[1] + cc[2];
        printf("{\"rowdec_case\": \"%s\", \"cycles\": {\"prelude\": %lld, \"power\": %lld, \"postlude\": %lld}, "
               "\"in_kernel_us\": %.2f, \"clock_ghz\": %.3f, \"event_us\": %.2f}\n",
               idle == 0 ? "warm" : idle == 1 ? "warm_after_20ms_idle" : "fresh_cu", cc[0], cc[1], cc[2],
               cc[3] * 0.01, tot / (cc[3] * 10.0), t * 1e3);
    }
    const bool same = std::memcmp(h[0], h[1], sizeof(h[0])) == 0 && std::memcmp(h[0], h[2], sizeof(h[0])) == 0 &&
                      std::memcmp(h[0], h[3], sizeof(h[0])) == 0;
    printf("{\"iters\": %d, \"dpp_us_per_dbl\": %.4f, \"lds_us_per_dbl\": %.4f, \"ror_us_per_dbl\": %.4f, \"ror2_us_per_dbl\": %.4f, "
           "\"dpp_cycles_per_dbl\": %.1f, \"lds_cycles_per_dbl\": %.1f, \"ror_cycles_per_dbl\": %.1f, \"ror2_cycles_per_dbl\": %.1f, \"same_limbs\": %s}\n",
           iters, ms[0] * 1e3 / iters, ms[1] * 1e3 / iters, ms[2] * 1e3 / iters, ms[3] * 1e3 / iters, (double)c[0] / iters,
           (double)c[1] / iters, (double)c[2] / iters, (double)c[3] / iters, same ? "true" : "false");
    return same ? 0 : 1;
}
