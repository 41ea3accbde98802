// ubench_bls.hip -- microbenchmark of the BLS12-381 tower (narwhal_amd/csrc/bls381.h) on gfx950:
// per-op latency of one wave (64 lanes, one element per lane) and throughput at a full chip, for
// Fp / Fp2 / Fp6 / Fp12 products, the cyclotomic squaring, one Miller loop and one final
// exponentiation.  Prints one JSON line per op.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "../narwhal_amd/csrc/bls_verify.h"

using namespace bls;

__device__ fp seed_fp(uint32_t t, uint32_t k) {
    fp a = k_one();
    a.l[0] = (a.l[0] + t * 7919u + k) & LM;
    return a;
}
__device__ void sink(uint32_t* out, uint32_t t, const fp& a) {
    uint32_t x = 0;
    for (int j = 0; j < NL; j++) x ^= a.l[j];
    out[t] = x;
}

__global__ __launch_bounds__(64) void k_fp_mul(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp a = seed_fp(t, 1), b = seed_fp(t, 2);
    for (int i = 0; i < reps; i++) a = fp_mul(a, b);
    sink(out, t, a);
}
__global__ __launch_bounds__(64) void k_fp_sqr(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp a = seed_fp(t, 1);
    for (int i = 0; i < reps; i++) a = fp_sqr(a);
    sink(out, t, a);
}
__global__ __launch_bounds__(64) void k_f2_mul(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp2 a = {seed_fp(t, 1), seed_fp(t, 3)}, b = {seed_fp(t, 2), seed_fp(t, 4)};
    for (int i = 0; i < reps; i++) a = f2_mul(a, b);
    sink(out, t, a.c0);
}
__device__ fp12 seed_f12(uint32_t t) {
    fp12 f;
    fp* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
                 &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
    for (int k = 0; k < 12; k++) *c[k] = seed_fp(t, k + 5);
    return f;
}
__global__ __launch_bounds__(64) void k_f6_mul(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp12 f = seed_f12(t);
    fp6 a = f.c0, b = f.c1;
    for (int i = 0; i < reps; i++) a = f6_mul(a, b);
    sink(out, t, a.c0.c0);
}
__global__ __launch_bounds__(64) void k_f12_mul(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp12 a = seed_f12(t), b = seed_f12(t + 1);
    for (int i = 0; i < reps; i++) a = f12_mul(a, b);
    sink(out, t, a.c0.c0.c0);
}
__global__ __launch_bounds__(64) void k_f12_sqr(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp12 a = seed_f12(t);
    for (int i = 0; i < reps; i++) a = f12_sqr(a);
    sink(out, t, a.c0.c0.c0);
}
__global__ __launch_bounds__(64) void k_f12_cyc(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp12 a = seed_f12(t);
    for (int i = 0; i < reps; i++) a = f12_cyc_sqr(a);
    sink(out, t, a.c0.c0.c0);
}
__global__ __launch_bounds__(64) void k_miller(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp px = k_g1x(), py = k_g1y();
    px.l[0] = (px.l[0] + t) & LM;
    fp2 qx = k_g2x(), qy = k_g2y();
    fp12 a = f12_one();
    for (int i = 0; i < reps; i++) a = f12_mul(a, miller_loop2(1, &px, &py, &qx, &qy));
    sink(out, t, a.c0.c0.c0);
}
__global__ __launch_bounds__(64) void k_fexp(int reps, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    fp12 a = seed_f12(t);
    for (int i = 0; i < reps; i++) a = final_exp(a);
    sink(out, t, a.c0.c0.c0);
}

// the 8-lane group forms (bls_group.h): one element per group, 8 groups per wave
#define GK(name, body)                                                                   \
    __global__ __launch_bounds__(64) void name(int reps, uint32_t* out) {               \
        __shared__ uint32_t lds[8 * GX_WORDS];                                           \
        const GCtx g = g_ctx(lds);                                                       \
        const uint32_t t = blockIdx.x * 64 + threadIdx.x;                                \
        G12 a = g_scatter(g, seed_f12(t >> 3)), b = g_scatter(g, seed_f12((t >> 3) + 1)); \
        body;                                                                            \
        sink(out, t, a.v.c0);                                                            \
    }
GK(k_g_mul, for (int i = 0; i < reps; i++) a = g_mul(g, a, b))
GK(k_g_sqr, for (int i = 0; i < reps; i++) a = g_sqr(g, a))
GK(k_g_cyc, for (int i = 0; i < reps; i++) a = g_cyc_sqr(g, a))
GK(k_g_line, for (int i = 0; i < reps; i++) a = g_mul_line(g, a, b.v, a.v, b.v))
GK(k_g_fexp, for (int i = 0; i < reps; i++) a = g_final_exp(g, a))
__device__ G12 miller_reps(const GCtx& g, G12 a, int reps) {
    fp px = k_g1x(), py = k_g1y();
    fp2 qx = k_g2x(), qy = k_g2y();
    for (int i = 0; i < reps; i++) a = g_mul(g, a, g_miller<1>(g, &px, &py, &qx, &qy));
    return a;
}
GK(k_g_miller, a = miller_reps(g, a, reps))
// one Miller-loop doubling step with its line: every lane on its own (ml_dbl) vs over the group
__device__ G12 dbl_reps(const GCtx& g, G12 a, int reps, bool grouped) {
    const fp px = k_g1x(), py = k_g1y();
    jac<fp2> T = jac_from_affine(k_g2x(), k_g2y());
    fp2 l0, l1, l4;
    for (int i = 0; i < reps; i++) {
        if (grouped) {
            g_ml_dbl(g, T, px, py, l0, l1, l4);
        } else {
            ml_dbl(T, l0, l1, l4);
            l1 = f2_mul_fp(l1, px);
            l4 = f2_mul_fp(l4, py);
        }
    }
    a.v = f2_add(f2_add(a.v, l0), f2_add(l1, f2_add(l4, T.x)));
    return a;
}
GK(k_g_dbl_lane, a = dbl_reps(g, a, reps, false))
GK(k_g_dbl_group, a = dbl_reps(g, a, reps, true))
// the same Miller loop with P, Q read from memory (runtime values, as the verification kernels see)
__device__ uint32_t d_pq[2 * NL + 4 * NL];
__device__ G12 miller_reps_mem(const GCtx& g, G12 a, int reps) {
    const fp px = ld_fp(d_pq), py = ld_fp(d_pq + NL);
    const fp2 qx = ld_f2(d_pq + 2 * NL), qy = ld_f2(d_pq + 4 * NL);
    for (int i = 0; i < reps; i++) a = g_mul(g, a, g_miller<1>(g, &px, &py, &qx, &qy));
    return a;
}
GK(k_g_miller_mem, a = miller_reps_mem(g, a, reps))
__global__ void k_init_pq() {
    if (threadIdx.x || blockIdx.x) return;
    st_fp(d_pq, k_g1x());
    st_fp(d_pq + NL, k_g1y());
    st_f2(d_pq + 2 * NL, k_g2x());
    st_f2(d_pq + 4 * NL, k_g2y());
}

typedef void (*kfn)(int, uint32_t*);

int main() {
    struct K {
        const char* name;
        kfn f;
        int reps;
        double fp_mults;  // per op, for the per-Fp-product figure
    } ks[] = {{"fp_mul", k_fp_mul, 2000, 1},       {"fp_sqr", k_fp_sqr, 2000, 1},
              {"f2_mul", k_f2_mul, 1000, 3},       {"f6_mul", k_f6_mul, 200, 18},
              {"f12_mul", k_f12_mul, 50, 54},      {"f12_sqr", k_f12_sqr, 50, 36},
              {"f12_cyc_sqr", k_f12_cyc, 100, 18}, {"miller_loop_1pair", k_miller, 1, 6800},
              {"final_exp", k_fexp, 1, 6000},      {"group8_f12_mul", k_g_mul, 200, 54},
              {"group8_f12_sqr", k_g_sqr, 200, 36}, {"group8_cyc_sqr", k_g_cyc, 200, 18},
              {"group8_line_mul", k_g_line, 200, 13}, {"group8_miller_loop_1pair", k_g_miller, 1, 6800},
              {"group8_final_exp", k_g_fexp, 1, 6000}, {"group8_miller_loop_1pair_mem", k_g_miller_mem, 1, 6800},
              {"group8_ml_dbl_every_lane", k_g_dbl_lane, 200, 29}, {"group8_ml_dbl_over_lanes", k_g_dbl_group, 200, 29}};
    const int blocks_full = 256 * 4 * 2;  // two waves per SIMD
    uint32_t* out;
    if (hipMalloc(&out, 4 * 64 * blocks_full) != hipSuccess) return 2;
    hipLaunchKernelGGL(k_init_pq, dim3(1), dim3(64), 0, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (auto& k : ks) {
        double ms[2];
        const int grids[2] = {1, blocks_full};
        for (int g = 0; g < 2; g++) {
            hipLaunchKernelGGL(k.f, dim3(grids[g]), dim3(64), 0, 0, 1, out);  // warm
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(grids[g]), dim3(64), 0, 0, k.reps, out);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) return 3;
            float m = 0;
            (void)hipEventElapsedTime(&m, e0, e1);
            ms[g] = m;
        }
        const double lat_us = ms[0] * 1e3 / k.reps;
        const bool grp = std::strncmp(k.name, "group8", 6) == 0;  // one element per 8 lanes
        const double thr = (double)blocks_full * (grp ? 8 : 64) * k.reps / (ms[1] * 1e-3);
        printf("{\"op\": \"%s\", \"latency_us_one_wave\": %.3f, \"per_fp_mult_us\": %.4f, \"ops_per_s_full_chip\": %.4g, "
               "\"fp_mults_per_op\": %.0f}\n",
               k.name, lat_us, lat_us / k.fp_mults, thr, k.fp_mults);
        fflush(stdout);
    }
    return 0;
}
