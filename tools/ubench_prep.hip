// ubench_prep.hip -- k_msm_points' row form (msm_kernels.hip msm_points_rows_block) launched alone
// on a few encodings, event-timed, against the lane-local form: is the row decompression's time in
// the engine the same as the isolated chain's (tools/ubench_row.hip k_rowdec)?  Prints JSON lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../narwhal_amd/csrc/ed25519_kernels.hip"
#include "../narwhal_amd/csrc/msm_kernels.hip"

using namespace nwv;

// where the waves of a 256-thread workgroup run: HW_ID (wave slot, SIMD, CU, SE, XCC) per wave
__global__ void __launch_bounds__(256) k_hwid(uint32_t* out) {
    uint32_t id, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if ((threadIdx.x & 63) == 0) {
        out[2 * (blockIdx.x * 4 + threadIdx.x / 64)] = id;
        out[2 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = xcc;
    }
    // keep the workgroup resident a while so its waves overlap
    const long long t0 = clock64();
    while (clock64() - t0 < 20000) {
    }
}

int main() {
    {
        uint32_t* d;
        hipMalloc(&d, 4 * 2 * 4 * 8);
        hipLaunchKernelGGL(k_hwid, dim3(8), dim3(256), 0, 0, d);
        uint32_t h[64];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        for (int b = 0; b < 8; b++) {
            printf("{\"block\": %d, \"waves\": [", b);
            for (int w = 0; w < 4; w++) {
                const uint32_t id = h[2 * (4 * b + w)];
                printf("%s{\"wave\": %u, \"simd\": %u, \"cu\": %u, \"sh\": %u, \"se\": %u, \"xcc\": %u}", w ? ", " : "",
                       id & 15, (id >> 4) & 3, (id >> 8) & 15, (id >> 12) & 1, (id >> 13) & 7, h[2 * (4 * b + w) + 1] & 15);
            }
            printf("]}\n");
        }
    }
    const int n = 4096;  // R points (sig + 64 i) and A points (pk + 32 i)
    std::vector<uint8_t> sig(64 * n), pk(32 * n);
    for (int i = 0; i < 64 * n; i++) sig[i] = (uint8_t)(i * 37 + 11);
    for (int i = 0; i < 32 * n; i++) pk[i] = (uint8_t)(i * 53 + 7);
    uint8_t *dsig, *dpk;
    uint32_t *pts, *fail;
    hipMalloc(&dsig, sig.size());
    hipMalloc(&dpk, pk.size());
    hipMalloc(&pts, 4 * MSM_PT_WORDS * (2 * n + 1));
    hipMalloc(&fail, 4);
    hipMemcpy(dsig, sig.data(), sig.size(), hipMemcpyHostToDevice);
    hipMemcpy(dpk, pk.data(), pk.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // the row form: how many waves of it share a CU.  Points p of a call of m = 2 n points: the
    // kernel maps workgroup b, wave w, row r to point (4 b + w) 4 + r, so with 64-thread workgroups
    // (one wave each) `blocks` workgroups cover every 4th group of 4 points -- the same work per wave
    const int cfg[4][2] = {{2, 256}, {8, 64}, {128, 256}, {512, 64}};
    for (auto& c : cfg) {
        // 64-thread workgroups: wave 0 of workgroup b takes points 16 b .. 16 b + 3, so a call of
        // 4 x blocks x 4 points covers them
        const uint64_t nn = (uint64_t)c[0] * 8;  // R and A points: 16 x blocks in all
        MsmPointArgs g{nn, nn, nn, dpk, dsig, pts, fail, 1u};
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_msm_points, dim3(c[0]), dim3(c[1]), 0, 0, g);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float t;
            hipEventElapsedTime(&t, e0, e1);
            if (rep) printf("{\"form\": \"rows\", \"blocks\": %d, \"threads\": %d, \"waves\": %d, \"event_us\": %.2f}\n",
                            c[0], c[1], c[0] * c[1] / 64, t * 1e3);
        }
    }
    return 0;
}
