// bls_probe2.hip -- debugging aid: the BLS12-381 point decompression steps as separate kernels
// (so each is selected on its own), compared with the host build of the same code.  Not part of
// the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "../narwhal_amd/csrc/bls_verify.h"

using namespace bls;

NWV_HD void putfp(uint32_t* o, const fp& a) {
    const fp c = fp_canon(a);
    for (int j = 0; j < NL; j++) o[j] = c.l[j];
}

NWV_HD void a_key(const uint8_t* pk, uint32_t* o) { o[0] = key_decode(pk, o + 1); }
NWV_HD void b_g2dec(const uint8_t* pk, uint32_t* o) {
    fp2 x, y;
    bool inf;
    o[0] = g2_decompress(x, y, inf, pk);
    o[1] = inf;
    putfp(o + 2, x.c0); putfp(o + 2 + NL, x.c1); putfp(o + 2 + 2 * NL, y.c0); putfp(o + 2 + 3 * NL, y.c1);
}
NWV_HD void c_frombe(const uint8_t* pk, uint32_t* o) {
    uint8_t b[48];
    for (int i = 0; i < 48; i++) b[i] = pk[i];
    b[0] &= 0x1f;
    fp p1, p0;
    plain_from_be(p1, b);
    plain_from_be(p0, pk + 48);
    for (int j = 0; j < NL; j++) { o[j] = p1.l[j]; o[NL + j] = p0.l[j]; }
    o[2 * NL] = plain_lt_p(p1);
    o[2 * NL + 1] = plain_lt_p(p0);
}
NWV_HD void d_sig(const uint8_t* sg, uint32_t* o) { o[0] = sig_decode(sg, o + 1); }
NWV_HD void e_g1dec(const uint8_t* sg, uint32_t* o) {
    fp x, y;
    bool inf;
    o[0] = g1_decompress(x, y, inf, sg);
    o[1] = inf;
    putfp(o + 2, x); putfp(o + 2 + NL, y);
}
NWV_HD void f_f2sqrt(const uint8_t* pk, uint32_t* o) {
    uint8_t b[48];
    for (int i = 0; i < 48; i++) b[i] = pk[i];
    b[0] &= 0x1f;
    fp p1, p0;
    plain_from_be(p1, b);
    plain_from_be(p0, pk + 48);
    fp2 x;
    x.c0 = fp_to_mont(p0);
    x.c1 = fp_to_mont(p1);
    const fp2 rhs = f2_add(f2_mul(f2_sqr(x), x), k_b2());
    fp2 y;
    o[0] = f2_sqrt(y, rhs);
    putfp(o + 1, y.c0); putfp(o + 1 + NL, y.c1);
    putfp(o + 1 + 2 * NL, rhs.c0); putfp(o + 1 + 3 * NL, rhs.c1);
}
NWV_HD void g_fpsqrt(const uint8_t* sg, uint32_t* o) {
    uint8_t b[48];
    for (int i = 0; i < 48; i++) b[i] = sg[i];
    b[0] &= 0x1f;
    fp px;
    plain_from_be(px, b);
    const fp x = fp_to_mont(px);
    const fp rhs = fp_add(fp_mul(fp_sqr(x), x), k_b1());
    fp y;
    o[0] = fp_sqrt(y, rhs);
    putfp(o + 1, y);
    putfp(o + 1 + NL, rhs);
}

#ifndef PROBE_HOST_ONLY
constexpr int NO = 128;
#define KERN(name, fn) \
    __global__ __launch_bounds__(64) void name(const uint8_t* in, int stride, int n, uint32_t* o) { \
        const int i = blockIdx.x * 64 + threadIdx.x;                                          \
        if (i < n) fn(in + (size_t)stride * i, o + (size_t)NO * i);                          \
    }
KERN(k_a, a_key)
KERN(k_b, b_g2dec)
KERN(k_c, c_frombe)
KERN(k_d, d_sig)
KERN(k_e, e_g1dec)
KERN(k_f, f_f2sqrt)
KERN(k_g, g_fpsqrt)

typedef void (*hostfn)(const uint8_t*, uint32_t*);

static int unhex(const char* h, uint8_t* out, int n) {
    for (int i = 0; i < n; i++) {
        unsigned v;
        if (sscanf(h + 2 * i, "%2x", &v) != 1) return -1;
        out[i] = (uint8_t)v;
    }
    return 0;
}

int main(int argc, char** argv) {
    // inputs: the G2 / G1 generators, then argv's compressed keys (192 hex) and signatures (96 hex)
    const int MAXN = 64;
    static uint8_t k96[MAXN][96], s48[MAXN][48];
    int nk = 0, ns = 0;
    g2_compress(k96[nk++], k_g2x(), k_g2y(), false);
    g1_compress(s48[ns++], k_g1x(), k_g1y(), false);
    for (int a = 1; a < argc; a++) {
        const size_t L = strlen(argv[a]);
        if (L == 192 && nk < MAXN) unhex(argv[a], k96[nk++], 96);
        if (L == 96 && ns < MAXN) unhex(argv[a], s48[ns++], 48);
    }
    const char* names[7] = {"key_decode", "g2_decompress", "plain_from_be(G2)", "sig_decode", "g1_decompress",
                            "f2_sqrt", "fp_sqrt"};
    hostfn hf[7] = {a_key, b_g2dec, c_frombe, d_sig, e_g1dec, f_f2sqrt, g_fpsqrt};
    const void* kf[7] = {(const void*)k_a, (const void*)k_b, (const void*)k_c, (const void*)k_d, (const void*)k_e,
                         (const void*)k_f, (const void*)k_g};
    const bool g2[7] = {true, true, true, false, false, true, false};
    uint8_t* din;
    uint32_t* dout;
    if (hipMalloc(&din, sizeof k96) != hipSuccess || hipMalloc(&dout, 4 * NO * MAXN) != hipSuccess) return 2;
    static uint32_t ho[MAXN][NO], go[MAXN][NO];
    for (int t = 0; t < 7; t++) {
        int n = g2[t] ? nk : ns, stride = g2[t] ? 96 : 48;
        const uint8_t* in = g2[t] ? &k96[0][0] : &s48[0][0];
        memset(ho, 0, sizeof ho);
        memset(go, 0, sizeof go);
        for (int i = 0; i < n; i++) hf[t](in + stride * i, ho[i]);
        (void)hipMemcpy(din, in, (size_t)stride * n, hipMemcpyHostToDevice);
        (void)hipMemset(dout, 0, sizeof go);
        void* args[4] = {&din, &stride, &n, &dout};
        if (hipLaunchKernel(kf[t], dim3(1), dim3(64), args, 0, 0) != hipSuccess) return 3;
        if (hipDeviceSynchronize() != hipSuccess) return 4;
        (void)hipMemcpy(go, dout, sizeof go, hipMemcpyDeviceToHost);
        for (int i = 0; i < n; i++) {
            int nd = 0, first = -1;
            for (int w = 0; w < NO; w++)
                if (ho[i][w] != go[i][w]) {
                    nd++;
                    if (first < 0) first = w;
                }
            printf("%-20s lane %d host[0]=%u gpu[0]=%u  words differing: %d (first %d)\n", names[t], i, ho[i][0],
                   go[i][0], nd, first);
        }
    }
    return 0;
}
#endif
