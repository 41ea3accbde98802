// nwv_bls.hip -- BLS12-381 min_sig verification engine on gfx950: the
// kernels over bls_verify.h and the C ABI of include/nwv_bls.h.
//
// A call stages its inputs in one pinned arena and one H2D copy, then runs
//   k_bls_keys   one lane per distinct public key: decode + G2 membership (psi(Q) = [x] Q)
//   k_bls_sigs   one lane per item: decode + G1 membership (phi(P) = [-x^2] P)
//   k_bls_h2c    one lane per item: H(msg) (RFC 9380 hash_to_curve G1)
//   k_bls_apk    one lane per item: the sum of the item's validated keys, affine
//   the pairing check, by default as ONE batch check over the call (bls_verify.h):
//     k_bls_rlc    one lane per item: [r_i] H_i, [r_i] sig_i, the Miller loop of ([r_i] H_i, apk_i)
//     k_bls_fold   ceil(log2 n) levels of a product tree (Fp12 products, G1 sums)
//     k_bls_final  one lane: times the Miller loop of (-sum r_i sig_i, g2), final exponentiation
//   and only when that rejects (or under NWV_FLAG_BLS_PER_ITEM)
//     k_bls_pair   one lane per item: e(-sig, g2) e(H, apk) == 1 (two-pair Miller loop + final exp)
// and copies the per-item statuses back.  The Miller loops are the hot part: Fp products on VALU
// v_mad_u64_u32 (bls381.h), no MFMA (no dense contraction).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/nwv.h"
#include "../../include/nwv_bls.h"
#include "bls_verify.h"

using namespace bls;

__attribute__((visibility("hidden"))) int nwv_internal_set_err(int code, const char* msg);
extern "C" {  // defined in nwv_host.hip's extern "C" section
__attribute__((visibility("hidden"))) uint32_t nwv_internal_ctx_flags(const nwv_ctx* ctx);
__attribute__((visibility("hidden"))) void nwv_internal_fill_seed(const uint8_t* seed32, uint8_t out[32]);
}

// ------------------------------------------------------------------------------ kernels
#define BLS_LANES 64
#define BLS_IDX() const uint32_t i = blockIdx.x * BLS_LANES + threadIdx.x; \
    if (i >= n) return

__global__ __launch_bounds__(BLS_LANES) void k_bls_keys(uint32_t n, const uint8_t* pk, uint32_t* rec, int32_t* st) {
    BLS_IDX();
    st[i] = key_decode(pk + 96 * (size_t)i, rec + (size_t)G2_REC_WORDS * i);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_sigs(uint32_t n, const uint8_t* sig, uint32_t* rec, int32_t* st) {
    BLS_IDX();
    st[i] = sig_decode(sig + 48 * (size_t)i, rec + (size_t)G1_REC_WORDS * i);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_h2c(uint32_t n, const uint8_t* msg, const uint64_t* off,
                                                       const uint32_t* len, const uint8_t* dst, uint32_t dl,
                                                       const int32_t* st, uint32_t* rec) {
    BLS_IDX();
    if (st && st[i] != ST_OK) return;
    h2c_record(msg + off[i], len[i], dst, dl, rec + (size_t)G1_REC_WORDS * i);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_apk(uint32_t n, const uint32_t* key_rec, const int32_t* key_st,
                                                       const uint32_t* pk_off, const uint32_t* pk_cnt,
                                                       const uint32_t* pk_idx, uint32_t* rec, int32_t* st) {
    BLS_IDX();
    if (st[i] != ST_OK) return;
    st[i] = apk_record(key_rec, key_st, pk_idx + pk_off[i], pk_cnt[i], rec + (size_t)G2_REC_WORDS * i);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_pair(uint32_t n, const uint32_t* sig_rec, const uint32_t* h_rec,
                                                        const uint32_t* apk_rec, int32_t* st) {
    BLS_IDX();
    if (st[i] != ST_OK) return;
    st[i] = pairing_check(sig_rec + (size_t)G1_REC_WORDS * i, h_rec + (size_t)G1_REC_WORDS * i,
                          apk_rec + (size_t)G2_REC_WORDS * i)
                ? ST_OK
                : ST_VERIFY_FAIL;
}
// the batch check (bls_verify.h): every item's share, then a product tree, then one lane's final
__global__ __launch_bounds__(BLS_LANES) void k_bls_rlc(uint32_t n, const uint32_t* sig_rec, const uint32_t* h_rec,
                                                       const uint32_t* apk_rec, const int32_t* st,
                                                       const uint8_t* seed, uint32_t* frec, uint32_t* srec) {
    BLS_IDX();
    uint32_t* f = frec + (size_t)F12_REC_WORDS * i;
    uint32_t* s = srec + (size_t)G1J_REC_WORDS * i;
    if (st[i] != ST_OK) {
        rlc_neutral(f, s);
        return;
    }
    rlc_item(sig_rec + (size_t)G1_REC_WORDS * i, h_rec + (size_t)G1_REC_WORDS * i, apk_rec + (size_t)G2_REC_WORDS * i,
             rlc_scalar(seed, i), f, s);
}
// one level of the tree over m shares: share j <- share j (+) share j + h, h = ceil(m / 2), j < m - h
__global__ __launch_bounds__(BLS_LANES) void k_bls_fold(uint32_t m, uint32_t* frec, uint32_t* srec) {
    const uint32_t h = (m + 1) / 2;
    const uint32_t n = m - h;
    BLS_IDX();
    rlc_fold(frec + (size_t)F12_REC_WORDS * i, srec + (size_t)G1J_REC_WORDS * i,
             frec + (size_t)F12_REC_WORDS * (i + h), srec + (size_t)G1J_REC_WORDS * (i + h));
}
__global__ void k_bls_final(const uint32_t* frec, const uint32_t* srec, int32_t* ok) {
    if (blockIdx.x || threadIdx.x) return;
    *ok = rlc_final(frec, srec) ? 1 : 0;
}
// sum of n decoded signatures (AggregateAuthenticator::aggregate), one lane
__global__ void k_bls_g1_sum(uint32_t n, const uint32_t* rec, const int32_t* st, uint8_t* out48, int32_t* out_st) {
    if (blockIdx.x || threadIdx.x) return;
    jac<fp> acc;
    acc.inf = true;
    acc.x = acc.y = acc.z = fp_zero();
    for (uint32_t k = 0; k < n; k++) {
        if (st[k] != ST_OK) {
            *out_st = st[k];
            return;
        }
        const uint32_t* r = rec + (size_t)G1_REC_WORDS * k;
        if (!r[2 * NL]) acc = jac_add(acc, jac_from_affine(ld_fp(r), ld_fp(r + NL)));
    }
    fp x = fp_zero(), y = fp_zero();
    if (!acc.inf) g1_to_affine(x, y, acc);
    g1_compress(out48, x, y, acc.inf);
    *out_st = ST_OK;
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_keygen(uint32_t n, const uint8_t* sk, uint8_t* pk) {
    BLS_IDX();
    const jac<fp2> q = jac_mul_be(jac_from_affine(k_g2x(), k_g2y()), sk + 32 * (size_t)i, 32);
    fp2 x = f2_zero(), y = f2_zero();
    if (!q.inf) g2_to_affine(x, y, q);
    g2_compress(pk + 96 * (size_t)i, x, y, q.inf);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_sign(uint32_t n, const uint8_t* sk, const uint8_t* msg,
                                                        const uint64_t* off, const uint32_t* len, const uint8_t* dst,
                                                        uint32_t dl, uint8_t* sig) {
    BLS_IDX();
    const jac<fp> s = jac_mul_be(hash_to_g1(msg + off[i], len[i], dst, dl), sk + 32 * (size_t)i, 32);
    fp x = fp_zero(), y = fp_zero();
    if (!s.inf) g1_to_affine(x, y, s);
    g1_compress(sig + 48 * (size_t)i, x, y, s.inf);
}
__device__ void be_to_mont(fp& r, const uint8_t* b) {
    fp t;
    plain_from_be(t, b);
    r = fp_to_mont(t);
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_h2c_out(uint32_t n, const uint8_t* msg, const uint64_t* off,
                                                           const uint32_t* len, const uint8_t* dst, uint32_t dl,
                                                           uint8_t* out) {
    BLS_IDX();
    uint32_t rec[G1_REC_WORDS];
    h2c_record(msg + off[i], len[i], dst, dl, rec);
    uint8_t* o = out + 96 * (size_t)i;
    if (rec[2 * NL]) {
        for (int k = 0; k < 96; k++) o[k] = 0;
        return;
    }
    plain_to_be(o, fp_from_mont(ld_fp(rec)));
    plain_to_be(o + 48, fp_from_mont(ld_fp(rec + NL)));
}
__global__ __launch_bounds__(BLS_LANES) void k_bls_pairing_raw(uint32_t n, const uint8_t* P, const uint8_t* Q,
                                                               uint8_t* out) {
    BLS_IDX();
    const uint8_t* p = P + 96 * (size_t)i;
    const uint8_t* q = Q + 192 * (size_t)i;
    uint32_t zp = 0, zq = 0;
    for (int k = 0; k < 96; k++) zp |= p[k];
    for (int k = 0; k < 192; k++) zq |= q[k];
    fp12 e = f12_one();
    if (zp && zq) {
        fp px, py;
        fp2 qx, qy;
        be_to_mont(px, p);
        be_to_mont(py, p + 48);
        be_to_mont(qx.c1, q);
        be_to_mont(qx.c0, q + 48);
        be_to_mont(qy.c1, q + 96);
        be_to_mont(qy.c0, q + 144);
        e = final_exp(miller_loop2(1, &px, &py, &qx, &qy));
    }
    const fp* c[12] = {&e.c0.c0.c0, &e.c0.c0.c1, &e.c0.c1.c0, &e.c0.c1.c1, &e.c0.c2.c0, &e.c0.c2.c1,
                       &e.c1.c0.c0, &e.c1.c0.c1, &e.c1.c1.c0, &e.c1.c1.c1, &e.c1.c2.c0, &e.c1.c2.c1};
    uint8_t* o = out + 576 * (size_t)i;
    for (int k = 0; k < 12; k++) plain_to_be(o + 48 * k, fp_from_mont(*c[k]));
}

// ------------------------------------------------------------------------------- host side
namespace {

#define BLS_HIP(x)                                                                  \
    do {                                                                            \
        const hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) return nwv_internal_set_err(NWV_ERR_HIP, hipGetErrorString(e_)); \
    } while (0)

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return NWV_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, n) != hipSuccess) return nwv_internal_set_err(NWV_ERR_OOM, "hipMalloc (bls)");
        cap = n;
        return NWV_OK;
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return NWV_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess)
            return nwv_internal_set_err(NWV_ERR_OOM, "hipHostMalloc (bls)");
        cap = n;
        return NWV_OK;
    }
    ~HBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// one device of a context: a stream and reusable staging / scratch buffers (one call at a time)
struct BlsDev {
    int ordinal = -1;
    uint32_t flags = 0;  // the context's nwv_init flags
    hipStream_t stream = nullptr;
    std::mutex mu;
    HBuf stage;
    DBuf in, work;
    hipEvent_t ev[6] = {};       // around the five stages of the last verify_many call
    double last_ms[5] = {0, 0, 0, 0, 0};
    int last_path = 0;           // nwv_bls_last_path
    ~BlsDev() {
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
};
std::mutex g_mu;
std::unordered_map<nwv_ctx*, BlsDev*> g_devs;

int dev_of(nwv_ctx* ctx, BlsDev** out) {
    if (!ctx) return nwv_internal_set_err(NWV_ERR_ARG, "null context");
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_devs.find(ctx);
    if (it != g_devs.end()) {
        *out = it->second;
        return NWV_OK;
    }
    const int ord = nwv_device_ordinal(ctx, 0);
    if (ord < 0) return nwv_internal_set_err(NWV_ERR_NODEV, "context has no device");
    auto* d = new BlsDev;
    d->ordinal = ord;
    d->flags = nwv_internal_ctx_flags(ctx);
    if (hipSetDevice(ord) != hipSuccess || hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
        delete d;
        return nwv_internal_set_err(NWV_ERR_HIP, "bls stream");
    }
    g_devs[ctx] = d;
    *out = d;
    return NWV_OK;
}

// an arena of sections placed 256-byte aligned, filled on the host, copied with one H2D
struct Arena {
    std::vector<std::pair<const void*, size_t>> parts;
    std::vector<size_t> offs;
    size_t total = 0;
    size_t add(const void* p, size_t n) {
        const size_t o = total;
        parts.push_back({p, n});
        offs.push_back(o);
        total += (n + 255) & ~(size_t)255;
        return o;
    }
};

constexpr int kBlocks(size_t n) { return (int)((n + BLS_LANES - 1) / BLS_LANES); }

// the whole verify_many pipeline on one device
int verify_on(BlsDev& d, size_t n_keys, const uint8_t* keys, size_t n, const uint8_t* sigs, const uint32_t* pk_off,
              const uint32_t* pk_cnt, const uint32_t* pk_idx, size_t n_idx, const uint8_t* msg_base,
              const uint64_t* msg_off, const uint32_t* msg_len, size_t msg_bytes, const uint8_t* dst, size_t dl,
              int32_t* status) {
    std::lock_guard<std::mutex> g(d.mu);
    BLS_HIP(hipSetDevice(d.ordinal));
    static const uint8_t zero[8] = {0};
    const bool batch = !(d.flags & NWV_FLAG_BLS_PER_ITEM);
    uint8_t seed[32];
    nwv_internal_fill_seed(nullptr, seed);  // the batch coefficients' key: OS entropy per call
    Arena a;
    const size_t o_keys = a.add(keys, 96 * n_keys), o_sigs = a.add(sigs, 48 * n), o_off = a.add(pk_off, 4 * n),
                 o_cnt = a.add(pk_cnt, 4 * n), o_idx = a.add(n_idx ? (const void*)pk_idx : zero, 4 * n_idx + 4),
                 o_msg = a.add(msg_bytes ? (const void*)msg_base : zero, msg_bytes + 1),
                 o_moff = a.add(msg_off, 8 * n), o_mlen = a.add(msg_len, 4 * n), o_dst = a.add(dst, dl),
                 o_seed = a.add(seed, 32);
    int rc;
    if ((rc = d.stage.ensure(((a.total + 255) & ~(size_t)255) + 64)) || (rc = d.in.ensure(a.total))) return rc;
    uint8_t* h = static_cast<uint8_t*>(d.stage.p);
    for (size_t k = 0; k < a.parts.size(); k++)
        if (a.parts[k].second) std::memcpy(h + a.offs[k], a.parts[k].first, a.parts[k].second);
    // scratch: key records + statuses, item sig / H / apk records, item statuses, the batch
    // check's shares (Fp12 + Jacobian G1 per item) and its verdict word
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t w_krec = 0, w_kst = w_krec + 4 * G2_REC_WORDS * n_keys, w_srec = al(w_kst + 4 * n_keys),
                 w_hrec = w_srec + 4 * G1_REC_WORDS * n, w_arec = w_hrec + 4 * G1_REC_WORDS * n,
                 w_st = w_arec + 4 * G2_REC_WORDS * n, w_ok = al(w_st + 4 * n), w_frec = al(w_ok + 4),
                 w_jrec = al(w_frec + 4 * F12_REC_WORDS * (batch ? n : 0)),
                 w_end = w_jrec + 4 * G1J_REC_WORDS * (batch ? n : 0) + 4;
    if ((rc = d.work.ensure(w_end))) return rc;
    uint8_t* in = static_cast<uint8_t*>(d.in.p);
    uint8_t* w = static_cast<uint8_t*>(d.work.p);
    BLS_HIP(hipMemcpyAsync(in, h, a.total, hipMemcpyHostToDevice, d.stream));
    auto* krec = reinterpret_cast<uint32_t*>(w + w_krec);
    auto* kst = reinterpret_cast<int32_t*>(w + w_kst);
    auto* srec = reinterpret_cast<uint32_t*>(w + w_srec);
    auto* hrec = reinterpret_cast<uint32_t*>(w + w_hrec);
    auto* arec = reinterpret_cast<uint32_t*>(w + w_arec);
    auto* st = reinterpret_cast<int32_t*>(w + w_st);
    auto* okw = reinterpret_cast<int32_t*>(w + w_ok);
    auto* frec = reinterpret_cast<uint32_t*>(w + w_frec);
    auto* jrec = reinterpret_cast<uint32_t*>(w + w_jrec);
    if (!d.ev[0])
        for (auto& e : d.ev) BLS_HIP(hipEventCreate(&e));
    BLS_HIP(hipEventRecord(d.ev[0], d.stream));
    if (n_keys)
        hipLaunchKernelGGL(k_bls_keys, dim3(kBlocks(n_keys)), dim3(BLS_LANES), 0, d.stream, (uint32_t)n_keys,
                           in + o_keys, krec, kst);
    BLS_HIP(hipEventRecord(d.ev[1], d.stream));
    hipLaunchKernelGGL(k_bls_sigs, dim3(kBlocks(n)), dim3(BLS_LANES), 0, d.stream, (uint32_t)n, in + o_sigs, srec, st);
    BLS_HIP(hipEventRecord(d.ev[2], d.stream));
    hipLaunchKernelGGL(k_bls_h2c, dim3(kBlocks(n)), dim3(BLS_LANES), 0, d.stream, (uint32_t)n, in + o_msg,
                       reinterpret_cast<const uint64_t*>(in + o_moff), reinterpret_cast<const uint32_t*>(in + o_mlen),
                       in + o_dst, (uint32_t)dl, (const int32_t*)st, hrec);
    BLS_HIP(hipEventRecord(d.ev[3], d.stream));
    hipLaunchKernelGGL(k_bls_apk, dim3(kBlocks(n)), dim3(BLS_LANES), 0, d.stream, (uint32_t)n, (const uint32_t*)krec,
                       (const int32_t*)kst, reinterpret_cast<const uint32_t*>(in + o_off),
                       reinterpret_cast<const uint32_t*>(in + o_cnt), reinterpret_cast<const uint32_t*>(in + o_idx),
                       arec, st);
    BLS_HIP(hipEventRecord(d.ev[4], d.stream));
    auto per_item = [&]() {
        hipLaunchKernelGGL(k_bls_pair, dim3(kBlocks(n)), dim3(BLS_LANES), 0, d.stream, (uint32_t)n,
                           (const uint32_t*)srec, (const uint32_t*)hrec, (const uint32_t*)arec, st);
    };
    int32_t* hst = reinterpret_cast<int32_t*>(h + al(a.total));  // pinned: the batch verdict word
    if (batch) {
        hipLaunchKernelGGL(k_bls_rlc, dim3(kBlocks(n)), dim3(BLS_LANES), 0, d.stream, (uint32_t)n,
                           (const uint32_t*)srec, (const uint32_t*)hrec, (const uint32_t*)arec, (const int32_t*)st,
                           (const uint8_t*)(in + o_seed), frec, jrec);
        for (uint32_t m = (uint32_t)n; m > 1; m = (m + 1) / 2)
            hipLaunchKernelGGL(k_bls_fold, dim3(kBlocks(m / 2)), dim3(BLS_LANES), 0, d.stream, m, frec, jrec);
        hipLaunchKernelGGL(k_bls_final, dim3(1), dim3(BLS_LANES), 0, d.stream, (const uint32_t*)frec,
                           (const uint32_t*)jrec, okw);
        BLS_HIP(hipMemcpyAsync(hst, okw, 4, hipMemcpyDeviceToHost, d.stream));
        BLS_HIP(hipStreamSynchronize(d.stream));
        BLS_HIP(hipGetLastError());
        d.last_path = *hst == 1 ? 1 : 2;
        if (*hst != 1) per_item();  // the batch check rejected: name the failing items exactly
    } else {
        per_item();
        d.last_path = 0;
    }
    BLS_HIP(hipEventRecord(d.ev[5], d.stream));
    BLS_HIP(hipGetLastError());
    BLS_HIP(hipMemcpyAsync(status, st, 4 * n, hipMemcpyDeviceToHost, d.stream));
    BLS_HIP(hipStreamSynchronize(d.stream));
    for (int k = 0; k < 5; k++) {
        float ms = 0;
        BLS_HIP(hipEventElapsedTime(&ms, d.ev[k], d.ev[k + 1]));
        d.last_ms[k] = ms;
    }
    return NWV_OK;
}

const uint8_t* dst_or_default(const uint8_t* dst, size_t* dl) {
    if (dst) return dst;
    *dl = sizeof(NWV_BLS_DST) - 1;
    return reinterpret_cast<const uint8_t*>(NWV_BLS_DST);
}

}  // namespace

__attribute__((visibility("hidden"))) void nwv_bls_ctx_release(nwv_ctx* ctx) {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_devs.find(ctx);
    if (it == g_devs.end()) return;
    (void)hipSetDevice(it->second->ordinal);
    delete it->second;
    g_devs.erase(it);
}

extern "C" {

int nwv_bls_verify_many(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys, size_t n, const uint8_t* sigs,
                        const uint32_t* pk_off, const uint32_t* pk_cnt, const uint32_t* pk_idx,
                        const uint8_t* msg_base, const uint64_t* msg_off, const uint32_t* msg_len,
                        const uint8_t* dst, size_t dst_len, int32_t* status) {
    if (n == 0) return NWV_OK;
    if (!sigs || !pk_off || !pk_cnt || !msg_off || !msg_len || !status || (n_keys && !keys))
        return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    if (n > (1u << 26) || n_keys > (1u << 26)) return nwv_internal_set_err(NWV_ERR_ARG, "batch too large");
    dst = dst_or_default(dst, &dst_len);
    if (dst_len > 255) return nwv_internal_set_err(NWV_ERR_ARG, "DST longer than 255 bytes");
    // host-side shape checks: every key index and message range in bounds
    size_t n_idx = 0, msg_bytes = 0;
    for (size_t i = 0; i < n; i++) {
        n_idx = std::max<size_t>(n_idx, (size_t)pk_off[i] + pk_cnt[i]);
        if (msg_len[i] && !msg_base) return nwv_internal_set_err(NWV_ERR_ARG, "null msg_base");
        msg_bytes = std::max<size_t>(msg_bytes, msg_off[i] + msg_len[i]);
    }
    if (n_idx && !pk_idx) return nwv_internal_set_err(NWV_ERR_ARG, "null pk_idx");
    for (size_t k = 0; k < n_idx; k++)
        if (pk_idx[k] >= n_keys) return nwv_internal_set_err(NWV_ERR_ARG, "key index out of range");
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    return verify_on(*d, n_keys, keys, n, sigs, pk_off, pk_cnt, pk_idx, n_idx, msg_base, msg_off, msg_len, msg_bytes,
                     dst, dst_len, status);
}

int nwv_bls_last_kernel_ms(nwv_ctx* ctx, double out_ms[5]) {
    if (!out_ms) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    for (int k = 0; k < 5; k++) out_ms[k] = d->last_ms[k];
    return NWV_OK;
}

int nwv_bls_last_path(nwv_ctx* ctx) {
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    return d->last_path;
}

int nwv_bls_aggregate_verify(nwv_ctx* ctx, const uint8_t* sig48, const uint8_t* pks, size_t n_pks, const uint8_t* msg,
                             size_t msg_len) {
    if (!sig48) return NWV_ERR_SIGNATURE;  // sig: None
    if ((n_pks && !pks) || (msg_len && !msg)) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    std::vector<uint32_t> idx(n_pks);
    for (size_t k = 0; k < n_pks; k++) idx[k] = (uint32_t)k;
    const uint32_t off = 0, cnt = (uint32_t)n_pks, len = (uint32_t)msg_len;
    const uint64_t moff = 0;
    int32_t st = 0;
    static const uint8_t empty[1] = {0};
    const int rc = nwv_bls_verify_many(ctx, n_pks, pks, 1, sig48, &off, &cnt, idx.data(), msg_len ? msg : empty, &moff,
                                       &len, nullptr, 0, &st);
    if (rc) return rc;
    return st == NWV_BLS_OK ? NWV_OK : NWV_ERR_SIGNATURE;
}

int nwv_bls_verify(nwv_ctx* ctx, const uint8_t pk[96], const uint8_t* msg, size_t msg_len, const uint8_t sig[48]) {
    if (!pk || !sig) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    return nwv_bls_aggregate_verify(ctx, sig, pk, 1, msg, msg_len);
}

int nwv_bls_aggregate(nwv_ctx* ctx, size_t n, const uint8_t* sigs48, uint8_t out48[48], int32_t* status_or_null) {
    if (status_or_null) *status_or_null = NWV_BLS_AGGR_MISMATCH;
    if (n == 0) return NWV_ERR_SIGNATURE;
    if (!sigs48 || !out48) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    BLS_HIP(hipSetDevice(d->ordinal));
    const size_t w_rec = 0, w_st = 4 * G1_REC_WORDS * n, w_out = w_st + 4 * n, w_ost = w_out + 64, w_end = w_ost + 8;
    if ((rc = d->in.ensure(48 * n)) || (rc = d->work.ensure(w_end)) || (rc = d->stage.ensure(128))) return rc;
    uint8_t* w = static_cast<uint8_t*>(d->work.p);
    BLS_HIP(hipMemcpyAsync(d->in.p, sigs48, 48 * n, hipMemcpyHostToDevice, d->stream));
    hipLaunchKernelGGL(k_bls_sigs, dim3(kBlocks(n)), dim3(BLS_LANES), 0, d->stream, (uint32_t)n,
                       (const uint8_t*)d->in.p, reinterpret_cast<uint32_t*>(w + w_rec), reinterpret_cast<int32_t*>(w + w_st));
    hipLaunchKernelGGL(k_bls_g1_sum, dim3(1), dim3(1), 0, d->stream, (uint32_t)n,
                       reinterpret_cast<const uint32_t*>(w + w_rec), reinterpret_cast<const int32_t*>(w + w_st),
                       w + w_out, reinterpret_cast<int32_t*>(w + w_ost));
    BLS_HIP(hipGetLastError());
    uint8_t* hs = static_cast<uint8_t*>(d->stage.p);
    BLS_HIP(hipMemcpyAsync(hs, w + w_out, 64 + 8, hipMemcpyDeviceToHost, d->stream));
    BLS_HIP(hipStreamSynchronize(d->stream));
    int32_t st;
    std::memcpy(&st, hs + 64, 4);
    if (status_or_null) *status_or_null = st;
    if (st != NWV_BLS_OK) return NWV_ERR_SIGNATURE;
    std::memcpy(out48, hs, 48);
    return NWV_OK;
}

int nwv_bls_verify_batch_empty_fail(nwv_ctx* ctx, const uint8_t* msg, size_t msg_len, const uint8_t* pks,
                                    size_t n_pks, const uint8_t* sigs, size_t n_sigs) {
    if (n_sigs == 0)
        return nwv_internal_set_err(NWV_ERR_EMPTY,
                                    "Critical Error! This behavious can signal something dangerous, and that "
                                    "someone may be trying to bypass signature verification through providing "
                                    "empty batches.");
    if (n_pks != n_sigs)
        return nwv_internal_set_err(NWV_ERR_LENGTH, "Mismatch between number of signatures and public keys provided");
    uint8_t agg[48];
    int rc = nwv_bls_aggregate(ctx, n_sigs, sigs, agg, nullptr);
    if (rc) return rc;
    return nwv_bls_aggregate_verify(ctx, agg, pks, n_pks, msg, msg_len);
}

int nwv_bls_aggregate_batch_verify(nwv_ctx* ctx, size_t n_aggs, const uint8_t* const* sigs48,
                                   const uint8_t* const* pks, const size_t* n_pks, const uint8_t* const* msgs,
                                   const size_t* msg_lens, size_t n_msgs) {
    if (n_aggs != n_msgs) return nwv_internal_set_err(NWV_ERR_LENGTH, "signatures / messages count mismatch");
    if (n_aggs == 0) return NWV_OK;
    if (!sigs48 || !pks || !n_pks || !msgs || !msg_lens) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    std::vector<uint8_t> keys, sg(48 * n_aggs), mb;
    std::vector<uint32_t> off(n_aggs), cnt(n_aggs), idx, len(n_aggs);
    std::vector<uint64_t> moff(n_aggs);
    for (size_t i = 0; i < n_aggs; i++) {
        if (!sigs48[i]) return NWV_ERR_SIGNATURE;  // an aggregate holding no signature
        std::memcpy(sg.data() + 48 * i, sigs48[i], 48);
        off[i] = (uint32_t)idx.size();
        cnt[i] = (uint32_t)n_pks[i];
        for (size_t k = 0; k < n_pks[i]; k++) {
            idx.push_back((uint32_t)(keys.size() / 96));
            keys.insert(keys.end(), pks[i] + 96 * k, pks[i] + 96 * (k + 1));
        }
        moff[i] = mb.size();
        len[i] = (uint32_t)msg_lens[i];
        if (msg_lens[i]) mb.insert(mb.end(), msgs[i], msgs[i] + msg_lens[i]);
    }
    mb.push_back(0);
    std::vector<int32_t> st(n_aggs);
    const int rc = nwv_bls_verify_many(ctx, keys.size() / 96, keys.data(), n_aggs, sg.data(), off.data(), cnt.data(),
                                       idx.data(), mb.data(), moff.data(), len.data(), nullptr, 0, st.data());
    if (rc) return rc;
    for (int32_t s : st)
        if (s != NWV_BLS_OK) return NWV_ERR_SIGNATURE;
    return NWV_OK;
}

static int simple_launch(nwv_ctx* ctx, size_t in_bytes, const void* in_host, size_t in2_bytes, const void* in2_host,
                         size_t out_bytes, void* out_host,
                         const std::function<void(hipStream_t, uint8_t*, uint8_t*, uint8_t*)>& launch) {
    BlsDev* d;
    int rc = dev_of(ctx, &d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    BLS_HIP(hipSetDevice(d->ordinal));
    const size_t o2 = (in_bytes + 255) & ~(size_t)255;
    if ((rc = d->in.ensure(o2 + in2_bytes + 16)) || (rc = d->work.ensure(out_bytes + 16))) return rc;
    uint8_t* in = static_cast<uint8_t*>(d->in.p);
    if (in_bytes) BLS_HIP(hipMemcpyAsync(in, in_host, in_bytes, hipMemcpyHostToDevice, d->stream));
    if (in2_bytes) BLS_HIP(hipMemcpyAsync(in + o2, in2_host, in2_bytes, hipMemcpyHostToDevice, d->stream));
    launch(d->stream, in, in + o2, static_cast<uint8_t*>(d->work.p));
    BLS_HIP(hipGetLastError());
    BLS_HIP(hipMemcpyAsync(out_host, d->work.p, out_bytes, hipMemcpyDeviceToHost, d->stream));
    BLS_HIP(hipStreamSynchronize(d->stream));
    return NWV_OK;
}

// messages + offsets + lengths + dst packed into one host block (the second input)
static std::vector<uint8_t> pack_msgs(size_t n, const uint8_t* msg_base, const uint64_t* msg_off,
                                      const uint32_t* msg_len, const uint8_t* dst, size_t dl, size_t* o_off,
                                      size_t* o_len, size_t* o_dst) {
    size_t bytes = 0;
    for (size_t i = 0; i < n; i++) bytes = std::max<size_t>(bytes, msg_off[i] + msg_len[i]);
    *o_off = (bytes + 1 + 7) & ~(size_t)7;
    *o_len = *o_off + 8 * n;
    *o_dst = *o_len + 4 * n;
    std::vector<uint8_t> v(*o_dst + dl + 1, 0);
    if (bytes) std::memcpy(v.data(), msg_base, bytes);
    std::memcpy(v.data() + *o_off, msg_off, 8 * n);
    std::memcpy(v.data() + *o_len, msg_len, 4 * n);
    std::memcpy(v.data() + *o_dst, dst, dl);
    return v;
}

int nwv_bls_keygen_many(nwv_ctx* ctx, size_t n, const uint8_t* sks, uint8_t* pks) {
    if (n == 0) return NWV_OK;
    if (!sks || !pks) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    return simple_launch(ctx, 32 * n, sks, 0, nullptr, 96 * n, pks, [&](hipStream_t s, uint8_t* in, uint8_t*, uint8_t* out) {
        hipLaunchKernelGGL(k_bls_keygen, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n, in, out);
    });
}

int nwv_bls_sign_many(nwv_ctx* ctx, size_t n, const uint8_t* sks, const uint8_t* msg_base, const uint64_t* msg_off,
                      const uint32_t* msg_len, const uint8_t* dst, size_t dst_len, uint8_t* sigs) {
    if (n == 0) return NWV_OK;
    if (!sks || !msg_off || !msg_len || !sigs) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    dst = dst_or_default(dst, &dst_len);
    size_t o_off, o_len, o_dst;
    const std::vector<uint8_t> m = pack_msgs(n, msg_base, msg_off, msg_len, dst, dst_len, &o_off, &o_len, &o_dst);
    return simple_launch(ctx, 32 * n, sks, m.size(), m.data(), 48 * n, sigs,
                         [&](hipStream_t s, uint8_t* in, uint8_t* mm, uint8_t* out) {
                             hipLaunchKernelGGL(k_bls_sign, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n, in, mm,
                                                reinterpret_cast<const uint64_t*>(mm + o_off),
                                                reinterpret_cast<const uint32_t*>(mm + o_len), mm + o_dst,
                                                (uint32_t)dst_len, out);
                         });
}

int nwv_bls_hash_to_g1_many(nwv_ctx* ctx, size_t n, const uint8_t* msg_base, const uint64_t* msg_off,
                            const uint32_t* msg_len, const uint8_t* dst, size_t dst_len, uint8_t* out96) {
    if (n == 0) return NWV_OK;
    if (!msg_off || !msg_len || !out96) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    dst = dst_or_default(dst, &dst_len);
    size_t o_off, o_len, o_dst;
    const std::vector<uint8_t> m = pack_msgs(n, msg_base, msg_off, msg_len, dst, dst_len, &o_off, &o_len, &o_dst);
    return simple_launch(ctx, 0, nullptr, m.size(), m.data(), 96 * n, out96,
                         [&](hipStream_t s, uint8_t*, uint8_t* mm, uint8_t* out) {
                             hipLaunchKernelGGL(k_bls_h2c_out, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n, mm,
                                                reinterpret_cast<const uint64_t*>(mm + o_off),
                                                reinterpret_cast<const uint32_t*>(mm + o_len), mm + o_dst,
                                                (uint32_t)dst_len, out);
                         });
}

int nwv_bls_pairing_many(nwv_ctx* ctx, size_t n, const uint8_t* P96, const uint8_t* Q192, uint8_t* out576) {
    if (n == 0) return NWV_OK;
    if (!P96 || !Q192 || !out576) return nwv_internal_set_err(NWV_ERR_ARG, "null argument");
    return simple_launch(ctx, 96 * n, P96, 192 * n, Q192, 576 * n, out576,
                         [&](hipStream_t s, uint8_t* in, uint8_t* in2, uint8_t* out) {
                             hipLaunchKernelGGL(k_bls_pairing_raw, dim3(kBlocks(n)), dim3(BLS_LANES), 0, s, (uint32_t)n,
                                                in, in2, out);
                         });
}

}  // extern "C"
