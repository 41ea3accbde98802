// ubench_field.hip -- throughput of the field squaring / multiplication (fe25519.h) as a function
// of waves per SIMD and independent chains per lane: how much latency hiding the VALU-bound
// kernels need (k_msm_points runs 2 waves per SIMD with one chain per lane at 65,536 signatures).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../narwhal_amd/csrc/fe25519.h"

using namespace nwv;

template <int ILP>
__global__ void __launch_bounds__(256) k_sq(uint32_t* out, int iters) {
    fe f[ILP];
#pragma unroll
    for (int c = 0; c < ILP; c++)
        for (int i = 0; i < 10; i++) f[c].v[i] = (threadIdx.x * 7 + i * 13 + c) & M25;
#pragma unroll 1
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < ILP; c++) fe_pin(f[c]);
#pragma unroll
        for (int c = 0; c < ILP; c++) f[c] = fe_sq(f[c]);
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < ILP; c++)
        for (int i = 0; i < 10; i++) s ^= f[c].v[i];
    if (s == 0x12345u) out[0] = s;
}
template <int ILP>
__global__ void __launch_bounds__(256) k_mul(uint32_t* out, int iters) {
    fe f[ILP], g;
    for (int i = 0; i < 10; i++) g.v[i] = (threadIdx.x * 5 + i * 11) & M25;
#pragma unroll
    for (int c = 0; c < ILP; c++)
        for (int i = 0; i < 10; i++) f[c].v[i] = (threadIdx.x * 7 + i * 13 + c) & M25;
#pragma unroll 1
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < ILP; c++) fe_pin(f[c]);
#pragma unroll
        for (int c = 0; c < ILP; c++) f[c] = fe_mul(f[c], g);
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < ILP; c++)
        for (int i = 0; i < 10; i++) s ^= f[c].v[i];
    if (s == 0x12345u) out[0] = s;
}

template <class K>
double rate(K kern, uint32_t* out, int iters, int blocks, int ilp) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 8);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    return (double)blocks * 256 * iters * ilp / (best * 1e-3);
}

int main() {
    uint32_t* out;
    hipMalloc(&out, 64);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int iters = 4096;
    for (int w : {1, 2, 3, 4, 6, 8}) {
        const int blocks = cus * w;  // 256-thread blocks: one wave per SIMD per block
        printf("{\"waves_per_simd\": %d, \"sq_ilp1\": %.4e, \"sq_ilp2\": %.4e, \"mul_ilp1\": %.4e, \"mul_ilp2\": %.4e}\n", w,
               rate(k_sq<1>, out, iters, blocks, 1), rate(k_sq<2>, out, iters, blocks, 2),
               rate(k_mul<1>, out, iters, blocks, 1), rate(k_mul<2>, out, iters, blocks, 2));
        fflush(stdout);
    }
    return 0;
}
