"""One-off source patch (kept for the record): generalise the MSM point layout to na A-points
(na = n unkeyed, na = m distinct keys when the caller supplies key indices)."""
import re

p = '/root/repo/narwhal_amd/csrc/msm_kernels.hip'
s = open(p).read()

# ---- k_msm_scalars: na, optional key ids (keyed: a_i goes to ascal for k_msm_keysum) ----
s = s.replace('''extern "C" __global__ void __launch_bounds__(256) k_msm_scalars(
    uint64_t n, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, MsmSeed seed, MsmLayout lay, uint32_t* __restrict__ scal,
    int16_t* __restrict__ digits, uint32_t* __restrict__ partial, uint32_t* __restrict__ fail) {''',
'''extern "C" __global__ void __launch_bounds__(256) k_msm_scalars(
    uint64_t n, uint64_t na, int keyed, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, const uint64_t* __restrict__ msg_off,
    const uint32_t* __restrict__ msg_len, MsmSeed seed, MsmLayout lay, uint32_t* __restrict__ ascal,
    int16_t* __restrict__ digits, uint32_t* __restrict__ partial, uint32_t* __restrict__ fail) {''')
s = s.replace('''        // signed digits of A_i's and R_i's scalars straight from registers (window-major rows)
        const uint64_t np = 2 * n + 1;
        msm_recode(a, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + i] = (int16_t)d; });
        msm_recode(z, lay, lay.nw_z, [&](int w, int d) { digits[(uint64_t)w * np + n + 1 + i] = (int16_t)d; });''',
'''        // signed digits straight from registers (window-major rows): R_i always; A_i's scalar
        // z_i k_i here when every signature has its own A point, else summed per key by
        // k_msm_keysum first
        const uint64_t np = na + 1 + n;
        if (keyed) msm_store8(ascal + 8 * i, a);
        else msm_recode(a, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + i] = (int16_t)d; });
        msm_recode(z, lay, lay.nw_z, [&](int w, int d) { digits[(uint64_t)w * np + na + 1 + i] = (int16_t)d; });''')
s = s.replace('''// digits: [window][2n+1] signed digits of every point's scalar (A_i at i, R_i at n+1+i; B's row
// entry n is written by k_msm_bscalar); partial: gridDim.x x 9 words''',
'''// digits: [window][na+1+n] signed digits of every point's scalar (A points at [0, na), B's
// entry na written by k_msm_bscalar, R_i at na+1+i); partial: gridDim.x x 9 words''')

# ---- k_msm_keysum: per-key sum of z_i k_i (CSR of signatures by key) ----
keysum = '''
// Keyed batches (ed25519_consensus groups batch entries by verification key): one workgroup per
// distinct key sums z_i k_i over its signatures (CSR: key_off[m+1], key_sig[n]), reduces mod l
// and writes the key point's digits (row entry = key index).
extern "C" __global__ void __launch_bounds__(256) k_msm_keysum(
    uint64_t n, uint64_t na, MsmLayout lay, const uint32_t* __restrict__ key_off,
    const uint32_t* __restrict__ key_sig, const uint32_t* __restrict__ ascal, int16_t* __restrict__ digits) {
    __shared__ unsigned long long col[256 * 9];
    const uint32_t key = blockIdx.x;
    unsigned long long s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t t = key_off[key] + threadIdx.x; t < key_off[key + 1]; t += 256) {
        const uint32_t* a = ascal + 8 * (size_t)key_sig[t];
#pragma unroll
        for (int k = 0; k < 8; k++) s[k] += a[k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) col[threadIdx.x * 9 + k] = s[k];
    __syncthreads();
    if (threadIdx.x < 8) {
        unsigned long long t = 0;
        for (int r = 0; r < 256; r++) t += col[r * 9 + threadIdx.x];  // < 2^(32+32)
        col[threadIdx.x] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x[16];
        unsigned long long c = 0;
        for (int k = 0; k < 16; k++) {
            if (k < 8) {
                const unsigned long long v = col[k];
                const unsigned long long lo = (c & 0xffffffffull) + (v & 0xffffffffull);
                x[k] = (uint32_t)lo;
                c = (c >> 32) + (v >> 32) + (lo >> 32);
            } else {
                x[k] = (uint32_t)c;
                c >>= 32;
            }
        }
        uint32_t r[8];
        sc_reduce512(x, r);
        const uint64_t np = na + 1 + n;
        msm_recode(r, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + key] = (int16_t)d; });
    }
}
'''
s = s.replace('''// One workgroup of 256: b = -(sum of the partials) mod l''', keysum.lstrip('\n') + '''
// One workgroup of 256: b = -(sum of the partials) mod l''')

# ---- k_msm_bscalar: B at index na ----
s = s.replace('''extern "C" __global__ void __launch_bounds__(256) k_msm_bscalar(
    uint64_t n, uint32_t nparts, MsmLayout lay, const uint32_t* __restrict__ partial,''',
'''extern "C" __global__ void __launch_bounds__(256) k_msm_bscalar(
    uint64_t n, uint64_t na, uint32_t nparts, MsmLayout lay, const uint32_t* __restrict__ partial,''')
s = s.replace('''        for (int k = 0; k < 8; k++) scal[8 * n + k] = b[k];
        const uint64_t np = 2 * n + 1;
        msm_recode(b, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + n] = (int16_t)d; });''',
'''        for (int k = 0; k < 8; k++) scal[k] = b[k];
        const uint64_t np = na + 1 + n;
        msm_recode(b, lay, lay.nw, [&](int w, int d) { digits[(uint64_t)w * np + na] = (int16_t)d; });''')
s = s.replace('''        pts[(size_t)MSM_PT_WORDS * n + threadIdx.x] =''', '''        pts[(size_t)MSM_PT_WORDS * na + threadIdx.x] =''')
s = s.replace('''// One workgroup of 256: b = -(sum of the partials) mod l -> scal[n]; B's affine entry -> pts[n]''',
              '''// One workgroup of 256: b = -(sum of the partials) mod l -> scal[0..8), digits of point na;
// B's record -> pts[na]''')

# ---- k_msm_points: R waves then A waves ----
old = s[s.index('// Two lanes per signature in different waves (as k_ed_points)'):s.index('// points of window w:')]
new = '''// Decompression, wave-uniform roles: waves [0, ceil(n/64)) decompress R_i into point na+1+i,
// the following ceil(na/64) waves decompress the A points (apk: per-signature keys, or the
// distinct keys of a keyed batch) into points [0, na).
extern "C" __global__ void __launch_bounds__(256) k_msm_points(
    uint64_t n, uint64_t na, const uint8_t* __restrict__ apk, const uint8_t* __restrict__ sig,
    uint32_t* __restrict__ pts, uint32_t* __restrict__ fail) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t rwaves = (n + 63) / 64;
    const bool is_r = (t >> 6) < rwaves;
    const uint64_t i = is_r ? t : t - 64 * rwaves;
    if (i >= (is_r ? n : na)) return;
    uint32_t w[8];
    msm_load8(is_r ? sig + 64 * i : apk + 32 * i, w);
    ge_p3 P;
    const bool ok = ge_decompress(w, P);
    msm_store_point(pts + (size_t)MSM_PT_WORDS * (is_r ? na + 1 + i : i), P);
    if (!ok) atomicOr(fail, 2u);
}

'''
s = s.replace(old, new)
s = s.replace('''// points of window w: all 2n+1 below nw_z, else the prefix [0, n]
__device__ __forceinline__ uint64_t msm_window_points(uint64_t n, int w, int nw_z) {
    return w < nw_z ? 2 * n + 1 : n + 1;
}''', '''// points of window w: all na+1+n below nw_z, else the prefix [0, na] (A points and B)
__device__ __forceinline__ uint64_t msm_window_points(uint64_t n, uint64_t na, int w, int nw_z) {
    return w < nw_z ? na + 1 + n : na + 1;
}''')
for kern in ('k_msm_hist', 'k_msm_scatter'):
    pass
s = s.replace('''extern "C" __global__ void __launch_bounds__(256) k_msm_hist(
    uint64_t n, MsmLayout lay,''', '''extern "C" __global__ void __launch_bounds__(256) k_msm_hist(
    uint64_t n, uint64_t na, MsmLayout lay,''')
s = s.replace('''extern "C" __global__ void __launch_bounds__(256) k_msm_scatter(
    uint64_t n, MsmLayout lay,''', '''extern "C" __global__ void __launch_bounds__(256) k_msm_scatter(
    uint64_t n, uint64_t na, MsmLayout lay,''')
s = s.replace('''    const uint64_t np = 2 * n + 1, cnt_w = msm_window_points(n, w, nw_z);''',
              '''    const uint64_t np = na + 1 + n, cnt_w = msm_window_points(n, na, w, nw_z);''')
assert '2 * n + 1' not in s, [m.start() for m in re.finditer(r'2 \* n \+ 1', s)]
open(p, 'w').write(s)
print('kernels patched')
