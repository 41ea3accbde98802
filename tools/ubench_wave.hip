// ubench_wave.hip -- microbenchmark of the one-wave BLS12-381 interpreter (bls_wave.h) on gfx950:
// time per stage program, per Miller loop, per final exponentiation and per pairing check on one
// wave (latency) and with a wave on every SIMD.  Prints one JSON line per case.  Not part of the
// product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "../narwhal_amd/csrc/bls_verify.h"

using namespace bls;
using namespace bls::wave;

// every slot past the constants holds some value below 2p (1 in Montgomery form, perturbed)
__device__ void fill(const Wave& w) {
    init_slots(w);
    for (int s = 1 + NCONSTS_PC + w.lane; s < NSLOTS; s += 64) {
        if (s >= CONST2_SLOT && s < CONST2_SLOT + NCONSTS - NCONSTS_PC) continue;
        fp a = k_one();
        a.l[0] = (a.l[0] + 7919u * s) & LM;
        for (int j = 0; j < NL; j++) w.wm[SW * s + j] = a.l[j];
    }
    w.sync();
}

__host__ __device__ Prog prog_of(int which) {
    switch (which) {
        case 0: return P_CYC_SQR_F;
        case 1: return P_SQR_F;
        case 2: return P_MUL_F_M;
        case 3: return P_ML_DBL_STEP;
        case 4: return P_ML_DBL_FIXED;
        case 5: return P_G1_DBL_U;
        case 7: return P_G1_SUM16;
        default: return P_COPY_F_TO_M;
    }
}

__global__ __launch_bounds__(64) void k_prog(int which, int reps, uint32_t* out, unsigned long long* clk) {
    __shared__ uint32_t wm_lds[WM_WORDS];
    uint32_t* const wm = wm_lds + KP_WORDS;
    const Wave w{wm, (int)threadIdx.x};
    fill(w);
    const Prog p = prog_of(which);
    const unsigned long long t0 = wall_clock64();
#pragma unroll 1
    for (int r = 0; r < reps; r++) w.run(p);
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = wm[SW * REG_F];
        clk[blockIdx.x] = t1 - t0;
    }
}

// the pieces of one pairing check: 0 Miller loop (computed lines), 1 Miller loop (fixed lines),
// 2 final exponentiation, 3 the Fp inversion of lane 0, 4 the whole check, 5 the inversion with
// the update rows on four lanes (fp_inv_wave)
__global__ __launch_bounds__(64) void k_piece(int which, int reps, uint32_t* out, unsigned long long* clk) {
    __shared__ uint32_t wm_lds[WM_WORDS];
    uint32_t* const wm = wm_lds + KP_WORDS;
    const Wave w{wm, (int)threadIdx.x};
    fill(w);
    const unsigned long long t0 = wall_clock64();
    bool ok = false;
#pragma unroll 1
    for (int r = 0; r < reps; r++) {
        if (which == 0 || which == 1) {
            const char* steps = BLS_WAVE_STEPS_STR;
#pragma unroll 1
            for (int k = 0; k < NSTEPS; k++) {
                const bool add = steps[k] == 'a';
                w.run(which ? (add ? P_ML_ADD_FIXED : P_ML_DBL_FIXED) : (add ? P_ML_ADD_STEP : P_ML_DBL_STEP));
            }
        } else if (which == 2) {
            final_exp(w);
        } else if (which == 3) {
            const fp n = w.get(REG_N);
            w.put_fp(REG_N + 1, fp_inv_vt_uniform(n));
            w.sync();
        } else if (which == 5) {
            const fp n = w.get(REG_N);
            w.put_fp(REG_N + 1, fp_inv_wave(n));
            w.sync();
        } else {
            ok ^= pairing_check(w, nullptr);
        }
    }
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = wm[SW * REG_F] ^ ok;
        clk[blockIdx.x] = t1 - t0;
    }
}

// one stage repeated with its record held in registers (no record loads): 0 the copy stage,
// 1 the product stage of cyc_sqr_F, 2 its combination stage; 3 only the record loads (a dependent
// chain: the latency of a lane record fetch)
__global__ __launch_bounds__(64) void k_stage(int which, int reps, uint32_t* out, unsigned long long* clk) {
    __shared__ uint32_t wm_lds[WM_WORDS];
    uint32_t* const wm = wm_lds + KP_WORDS;
    const Wave w{wm, (int)threadIdx.x};
    fill(w);
    const int lane = threadIdx.x;
    const Prog p = which == 0 ? P_COPY_F_TO_M : P_CYC_SQR_F;
    const uint16_t* base = T_DATA + p.off;
    Rec cur = load_rec(base + (uint32_t)min(lane, p.nl0 - 1) * REC);
    if (which == 2) {
        base += (uint32_t)p.nl0 * REC;
        const int nl1 = rec_hdr(cur).nl_next;
        cur = load_rec(base + (uint32_t)min(lane, nl1 - 1) * REC);
    }
    uint32_t acc = 0;
    const unsigned long long c0 = clock64();
    const unsigned long long t0 = wall_clock64();
    if (which == 3) {
#pragma unroll 1
        for (int r = 0; r < reps; r++) {
            cur = load_rec(base + (uint32_t)min(lane, p.nl0 - 1) * REC + (acc & 1));
            acc += cur.w[0] + cur.w[19];
        }
    } else {
        Hdr h = rec_hdr(cur);
        const int nl = __builtin_amdgcn_readfirstlane(h.nl);
#pragma unroll 1
        for (int r = 0; r < reps; r++) {
            if (lane < nl) {
                const uint32_t dst = rec_u16(cur, 0);
                const fp v = lane_value((const wword*)wm, h, cur);
#pragma unroll
                for (int j = 0; j < NL; j++) wm[SW * dst + j] = v.l[j];
            }
            wsync();
        }
    }
    const unsigned long long t1 = wall_clock64();
    const unsigned long long c1 = clock64();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = wm[SW * REG_F] + acc;
        clk[blockIdx.x] = t1 - t0;
        clk[blockIdx.x + 1024] = c1 - c0;
    }
}

// the product stage of cyc_sqr_F split into its parts, repeated: 0 both combinations only (no
// product), 1 the product only (operands read as two plain slots), 2 combination A + product
__global__ __launch_bounds__(64) void k_parts(int which, int reps, uint32_t* out, unsigned long long* clk) {
    __shared__ uint32_t wm_lds[WM_WORDS];
    uint32_t* const wm = wm_lds + KP_WORDS;
    const Wave w{wm, (int)threadIdx.x};
    fill(w);
    const int lane = threadIdx.x;
    const Prog p = P_CYC_SQR_F;
    const Rec cur = load_rec(T_DATA + p.off + (uint32_t)min(lane, p.nl0 - 1) * REC);
    Hdr h = rec_hdr(cur);
    h.nap = __builtin_amdgcn_readfirstlane(h.nap);
    h.nan = __builtin_amdgcn_readfirstlane(h.nan);
    h.nbp = __builtin_amdgcn_readfirstlane(h.nbp);
    h.nbn = __builtin_amdgcn_readfirstlane(h.nbn);
    const int nl = __builtin_amdgcn_readfirstlane(h.nl);
    const uint32_t fl = rec_u16(cur, 1);
    const unsigned long long c0 = clock64();
#pragma unroll 1
    for (int r = 0; r < reps; r++) {
        if (lane < nl) {
            const uint32_t dst = rec_u16(cur, 0);
            fp v;
            if (which == 0) {
                v = lin_comb<4>((const wword*)wm, cur, h.nap, h.nan, rec_u16(cur, 2), (fl & 4) != 0);
                const fp b = lin_comb<4 + 2 * TMAX>((const wword*)wm, cur, h.nbp, h.nbn, rec_u16(cur, 3), (fl & 8) != 0);
                for (int j = 0; j < NL; j++) v.l[j] ^= b.l[j];
            } else if (which == 1) {
                v = fp_mul(w.get(REG_F + (lane & 7)), w.get(REG_G + (lane & 7)));
            } else {
                v = lin_comb<4>((const wword*)wm, cur, h.nap, h.nan, rec_u16(cur, 2), (fl & 4) != 0);
                v = fp_mul(v, w.get(REG_G + (lane & 7)));
            }
#pragma unroll
            for (int j = 0; j < NL; j++) wm[SW * ((dst & 63) + 230) + j] = v.l[j];
        }
        wsync();
    }
    const unsigned long long c1 = clock64();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = wm[SW * REG_F];
        clk[blockIdx.x] = 0;
        clk[blockIdx.x + 1024] = c1 - c0;
    }
}

// the hash to G1 on a wave (no cofactor chain: the key-side form) and its lane-local pieces:
// 0 the whole w_hash_to_g1, 1 expand_message_xmd on lanes 0-1, 2 map_sswu_frac on lanes 0-1,
// 3 one fp_pow (the square-root exponent) on lane 0
__global__ __launch_bounds__(64) void k_h2c(int which, int reps, uint32_t* out, unsigned long long* clk) {
    __shared__ uint32_t wm_lds[WM_WORDS];
    uint32_t* const wm = wm_lds + KP_WORDS;
    const Wave w{wm, (int)threadIdx.x};
    fill(w);
    __shared__ uint8_t msg[64];
    if (threadIdx.x < 64) msg[threadIdx.x] = (uint8_t)(threadIdx.x * 7 + 1);
    const char dst[] = "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_";
    __shared__ uint32_t rec[G1H_REC_WORDS];
    w.sync();
    uint32_t acc = 0;
    const unsigned long long t0 = wall_clock64();
#pragma unroll 1
    for (int r = 0; r < reps; r++) {
        if (which == 0) {
            w_hash_to_g1(w, msg, 32, (const uint8_t*)dst, 43, rec, false);
        } else if (which == 1) {
            w.lanes(2, [&](int j) {
                uint8_t ub[128];
                expand_xmd_128(ub, msg + j, 32, (const uint8_t*)dst, 43);
                acc += ub[5] + ub[77];
            });
        } else if (which == 2) {
            w.lanes(2, [&](int j) {
                fp xn, xd, y, u = k_one();
                u.l[0] += (uint32_t)(r + j);
                map_sswu_frac(xn, xd, y, u);
                acc += xn.l[0] ^ y.l[3];
            });
        } else {
            w.lanes(1, [&](int j) {
                const uint32_t c1[12] = BLS_E_QR;
                fp u = k_one();
                u.l[0] += (uint32_t)(r + j);
                acc += fp_pow(u, c1).l[2];
            });
        }
        w.sync();
    }
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = rec[0] + acc;
        clk[blockIdx.x] = t1 - t0;
    }
}

typedef void (*kfn)(int, int, uint32_t*, unsigned long long*);

int main(int argc, char** argv) {
    struct K {
        const char* name;
        kfn f;
        int which, reps, stages;
    } ks[] = {{"cyc_sqr_F", k_prog, 0, 400, 2},        {"sqr_F", k_prog, 1, 200, 3},
              {"mul_F_M", k_prog, 2, 200, 3},          {"ml_dbl_step", k_prog, 3, 100, 9},
              {"ml_dbl_fixed", k_prog, 4, 100, 9},     {"g1_dbl_u", k_prog, 5, 200, 5},
              {"copy_F_to_M", k_prog, 6, 400, 1},      {"g1_sum16", k_prog, 7, 50, 13},      {"miller_loop", k_piece, 0, 2, 0},
              {"miller_loop_fixed", k_piece, 1, 2, 0}, {"final_exp", k_piece, 2, 2, 0},
              {"fp_inv_vt_lane0", k_piece, 3, 20, 0},  {"fp_inv_wave", k_piece, 5, 20, 0},  {"pairing_check", k_piece, 4, 2, 0},
              {"stage_copy_noload", k_stage, 0, 1000, 0}, {"stage_cyc_products_noload", k_stage, 1, 400, 0},
              {"stage_cyc_combos_noload", k_stage, 2, 1000, 0}, {"record_fetch_latency", k_stage, 3, 1000, 0},
              {"part_combos_only", k_parts, 0, 400, 0}, {"part_product_only", k_parts, 1, 400, 0},
              {"part_comboA_product", k_parts, 2, 400, 0},
              {"h2c_wave_no_cofactor", k_h2c, 0, 5, 0}, {"h2c_expand_xmd", k_h2c, 1, 20, 0},
              {"h2c_map_sswu", k_h2c, 2, 5, 0}, {"fp_pow_sqrt_lane0", k_h2c, 3, 5, 0}};
    const int blocks_full = 256 * 4;  // a wave per SIMD
    uint32_t* out;
    unsigned long long* clk;
    if (hipMalloc(&out, 4 * blocks_full) != hipSuccess || hipMalloc(&clk, 8 * (blocks_full + 1024)) != hipSuccess) return 2;
    int mhz = 100;
    {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, 0) == hipSuccess && v > 0) mhz = v / 1000;
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (auto& k : ks) {
        if (argc > 1 && std::strcmp(argv[1], k.name) != 0) continue;
        double ms[2], us_dev = 0, cyc = 0;
        const int grids[2] = {1, blocks_full};
        for (int g = 0; g < 2; g++) {
            hipLaunchKernelGGL(k.f, dim3(grids[g]), dim3(64), 0, 0, k.which, 1, out, clk);  // warm
            if (hipDeviceSynchronize() != hipSuccess) return 3;
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(grids[g]), dim3(64), 0, 0, k.which, k.reps, out, clk);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) return 3;
            float m = 0;
            (void)hipEventElapsedTime(&m, e0, e1);
            ms[g] = m;
            if (g == 0) {
                unsigned long long c = 0, cc = 0;
                (void)hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
                (void)hipMemcpy(&cc, clk + 1024, 8, hipMemcpyDeviceToHost);
                us_dev = (double)c / mhz / k.reps;
                if (k.f == k_stage || k.f == k_parts) cyc = (double)cc / k.reps;
            }
        }
        const double lat_us = ms[0] * 1e3 / k.reps;
        printf("{\"case\": \"%s\", \"us_one_wave\": %.3f, \"us_one_wave_in_kernel\": %.3f, \"us_per_stage\": %.3f, "
               "\"us_wave_per_simd\": %.3f, \"shader_clocks_per_rep\": %.0f}\n",
               k.name, lat_us, us_dev, k.stages ? us_dev / prog_of(k.which).n : 0.0, ms[1] * 1e3 / k.reps, cyc);
        fflush(stdout);
    }
    return 0;
}
