// ubench_valu.hip -- measures the peak rate of the VALU instructions the Ed25519 kernels are
// built from (roofline denominator): v_mad_u64_u32 (32x32->64 multiply-add),
// v_add_u32 and v_mul_lo_u32, with many independent chains per lane and full occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH 8
__global__ void __launch_bounds__(256) k_mad(void* outp, uint32_t a0, int iters) {
    uint32_t a = a0 + threadIdx.x, b = a0 * 3 + blockIdx.x;
    uint64_t acc[CH];
    for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint64_t r;
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(acc[c]) : "vcc");
            acc[c] = r;
        }
    }
    uint64_t s = 0;
    for (int c = 0; c < CH; c++) s ^= acc[c];
    if (s == 0x1234567) ((decltype(s)*)outp)[0] = s;
}
__global__ void __launch_bounds__(256) k_add(void* outp, uint32_t a0, int iters) {
    uint32_t acc[CH];
    for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
    uint32_t b = a0 + blockIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_add_u32 %0, %1, %0" : "+v"(acc[c]) : "v"(b));
    }
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= acc[c];
    if (s == 0x1234567) ((decltype(s)*)outp)[0] = s;
}
__global__ void __launch_bounds__(256) k_mullo(void* outp, uint32_t a0, int iters) {
    uint32_t acc[CH];
    for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x + 1;
    uint32_t b = a0 + blockIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(acc[c]) : "v"(b));
    }
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= acc[c];
    if (s == 0x1234567) ((decltype(s)*)outp)[0] = s;
}

// gfx950 64-bit integer forms used by the field and SHA-512 code (SQ_INSTS_VALU_INT64 class)
__global__ void __launch_bounds__(256) k_add64(void* outp, uint32_t a0, int iters) {
    uint64_t acc[CH];
    for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x;
    const uint64_t b = a0 + blockIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"(b));
    }
    uint64_t s = 0;
    for (int c = 0; c < CH; c++) s ^= acc[c];
    if (s == 0x1234567) ((decltype(s)*)outp)[0] = s;
}
__global__ void __launch_bounds__(256) k_shr64(void* outp, uint32_t a0, int iters) {
    uint64_t acc[CH];
    for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x + ((uint64_t)a0 << 40);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc[c]));
    }
    uint64_t s = 0;
    for (int c = 0; c < CH; c++) s ^= acc[c];
    if (s == 0x1234567) ((decltype(s)*)outp)[0] = s;
}
__global__ void __launch_bounds__(256) k_alignbit(void* outp, uint32_t a0, int iters) {
    uint32_t acc[CH];
    for (int c = 0; c < CH; c++) acc[c] = c + threadIdx.x + 1;
    uint32_t b = a0 + blockIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_alignbit_b32 %0, %1, %0, 7" : "+v"(acc[c]) : "v"(b));
    }
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= acc[c];
    if (s == 0x1234567) ((decltype(s)*)outp)[0] = s;
}

template <class K>
double rate(K kern, void* out, int iters, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 3u, 16);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 3u, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)blocks * 256 * iters * CH;
    return ops / (ms * 1e-3);
}

int main() {
    void* out;
    hipMalloc(&out, 64);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * 8;
    const int iters = 1 << 14;
    double mad = 0, add = 0, mul = 0, add64 = 0, shr64 = 0, alb = 0;
    for (int r = 0; r < 3; r++) {
        mad = std::max(mad, rate(k_mad, out, iters, blocks));
        add = std::max(add, rate(k_add, out, iters, blocks));
        mul = std::max(mul, rate(k_mullo, out, iters, blocks));
        add64 = std::max(add64, rate(k_add64, out, iters, blocks));
        shr64 = std::max(shr64, rate(k_shr64, out, iters, blocks));
        alb = std::max(alb, rate(k_alignbit, out, iters, blocks));
    }
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"v_mad_u64_u32_per_s\": %.4e, "
           "\"v_add_u32_per_s\": %.4e, \"v_mul_lo_u32_per_s\": %.4e, \"v_lshl_add_u64_per_s\": %.4e, "
           "\"v_lshrrev_b64_per_s\": %.4e, \"v_alignbit_b32_per_s\": %.4e}\n",
           p.gcnArchName, p.multiProcessorCount, p.clockRate, mad, add, mul, add64, shr64, alb);
    return 0;
}
