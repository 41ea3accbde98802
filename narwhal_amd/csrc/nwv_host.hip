// nwv_host.hip -- host side of the C ABI in include/nwv.h: device contexts, SoA staging,
// sharding by signature index over devices, kernel pipelines, fastcrypto trait semantics.
//
// One translation unit with the kernels (non-RDC build of a single code object).  Every
// verification runs on the GPU; there is no CPU fallback in this library: if no gfx950 device
// can be opened, nwv_init fails with NWV_ERR_NODEV.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/nwv.h"
#include "blake2b_kernels.hip"
#include "ed25519_kernels.hip"
#include "msm_kernels.hip"
#include "tiny_kernels.hip"
#include "shard.h"
#include "stage_args.h"

#include <random>

#include <sys/random.h>
#include <cerrno>

namespace {

thread_local std::string g_last_error = "";

// NWV_HOST_TRACE=1: host-side phase timestamps on stderr (diagnostics only)
void htrace(const char* what) {
    static const bool on = std::getenv("NWV_HOST_TRACE") != nullptr;
    if (!on) return;
    const double us = std::chrono::duration<double, std::micro>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "nwv-trace %.1f %s\n", us, what);
}

}  // namespace
// shared with the BLS12-381 translation unit (nwv_bls.hip); not part of the public ABI
__attribute__((visibility("hidden"))) void nwv_bls_ctx_release(nwv_ctx* ctx);
__attribute__((visibility("hidden"))) int nwv_internal_set_err(int code, const char* msg) {
    g_last_error = msg;
    return code;
}
namespace {
int set_err(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define NWV_HIP(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return set_err(e_ == hipErrorOutOfMemory ? NWV_ERR_OOM : NWV_ERR_HIP,       \
                           std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

constexpr size_t MSG_PAD = 64;  // over-read slack after every message arena

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool view = false;  // p points into another buffer (the staging arena): never freed here
    int ensure(size_t bytes) {
        if (bytes <= cap) return NWV_OK;
        if (p && !view) (void)hipFree(p);
        view = false;
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return set_err(NWV_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
        cap = want;
        return NWV_OK;
    }
    void release() {
        if (p && !view) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        view = false;
    }
    void set_view(void* base, size_t bytes) {
        release();
        p = base;
        cap = bytes;
        view = true;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

// Pinned host staging buffer: inputs are packed here and cross PCIe in one DMA
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes, unsigned flags = hipHostMallocDefault) {
        if (bytes <= cap) return NWV_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
        if (hipHostMalloc(&p, want, flags) != hipSuccess) {
            p = nullptr;
            return set_err(NWV_ERR_OOM, "hipHostMalloc");
        }
        cap = want;
        return NWV_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Device-resident inputs + intermediates of one Ed25519 batch: the per-signature pipeline
// (kbuf, flags, tables, verdict) and the batch MSM (m_*)
struct EdBuffers {
    DevBuf pk, sig, msg, off, len, kbuf, flags, tables, verdict;
    DevBuf m_scal, m_partial, m_state, m_pts, m_digits, m_cnt, m_tiles, m_entries, m_kstart, m_hpart,
        m_bsum, m_wsum, m_tpart, m_ctr, m_stamps, m_mid, m_kst2, m_segkey;
    // keyed batches: distinct keys (m x 32), CSR of signatures by key, per-signature z_i k_i
    DevBuf keys, koff, ksig, m_ascal;
    DevBuf kslot;  // keyed batches over the key cache: each distinct key's cache slot
    DevBuf in;  // staging arena: pk, sig, off, len, m_state and msg are views into it
    size_t nkeys_distinct = 0;  // 0: every signature is its own A point
    bool kc_split = false;      // keyed batch whose keys are all in the device's key cache
    // the last batch MSM already built the per-signature fallback's tables (early form, msm_launch)
    bool tables_ready = false;
    // a keyed batch of at most TINY_MAX signatures by registered keys (ed_stage_keyed): the
    // one-launch path (k_ed_tiny) with each signature's key cache slot and comb table
    bool tiny = false;
    uint32_t tiny_slot[TINY_MAX], tiny_cidx[TINY_MAX];
    void release() {
        for (DevBuf* b : {&pk, &sig, &msg, &off, &len, &kbuf, &flags, &tables, &verdict, &m_scal,
                          &m_partial, &m_state, &m_pts, &m_digits, &m_cnt, &m_tiles, &m_entries,
                          &m_kstart, &m_hpart, &m_bsum, &m_wsum, &m_tpart, &m_ctr, &m_stamps, &m_mid, &m_kst2, &m_segkey, &keys, &koff, &ksig, &m_ascal,
                          &kslot, &in})
            b->release();
        nkeys_distinct = 0;
        kc_split = false;
        tables_ready = false;
        tiny = false;
    }
};

struct Gpu;

// One in-flight call on a device: its own stream, pinned staging buffers and device buffers.  A
// device keeps a small pool of lanes, so calls from several host threads overlap (one call's H2D
// copy with another's kernels) instead of queueing behind one device lock.
struct Lane {
    Gpu* gpu = nullptr;
    int ordinal = -1;
    uint32_t flags = 0;  // nwv_init flags (NWV_FLAG_*)
    const DevBuf* btabp = nullptr;  // the device's basepoint table (read-only)
    hipStream_t stream = nullptr;
    const DevBuf& btab() const { return *btabp; }
    EdBuffers ed;
    PinnedBuf hstage;              // host side of ed_stage's single H2D copy
    hipEvent_t hstage_ev = nullptr;  // recorded after that copy; hstage is reusable once it fires
    DevBuf b2_base, b2_off, b2_len, b2_out, b2_packed, b2_plen, b2_err;
    DevBuf b2_in;                  // small digest batches: off, len and bytes in one arena
    PinnedBuf b2stage;             // host side of that arena's single H2D copy
    PinnedBuf b2dig;               // digests of a digest-then-verify call, copied back early
    hipEvent_t b2stage_ev = nullptr;
    // large stagings (ed_stage's piped form): pksig_ev fires once pk, sig, the offsets and the MSM
    // state words are on the device, while the messages are still crossing PCIe; the batch MSM's
    // decompressions then start on `aux` (msm_launch's early form), aux_ev joins them back
    hipStream_t aux = nullptr;
    hipEvent_t pksig_ev = nullptr, aux_ev = nullptr;
    bool pksig_pending = false;
    // one word of coherent pinned host memory: the batch MSM's tail stores its verdict there and
    // batch_on_device polls it (no verdict copy, no wait for the stream's completion signal)
    uint32_t* hword = nullptr;  // 64 bytes: [0] the verdict code, [2, 4) k_ed_tiny's verdict bits
    uint32_t hseq = 0;  // sequence number of the lane's last polled call (30 bits, never 0)
    // staged runs with prep chaining (NWV_STAGE_CHAIN): k_msm_prep waits for chain_wait (an earlier
    // staged run's prep on this device) and chain_rec is recorded after it; null otherwise
    hipEvent_t chain_wait = nullptr, chain_rec = nullptr;
    DevBuf tiny_ws;  // k_ed_tiny's workspace (zeroed once; the kernel leaves it zeroed)
};

// Committee key cache of a device.  fastcrypto decompresses a public key once, when it is
// deserialized; keyed calls (the types layer, nwv_ed25519_verify_batch_keyed) name their keys,
// so each key's point record and that of 2^128 A are computed once (k_keycache_fill) and kept
// in HBM.  A keyed batch whose keys are all cached then carries every MSM scalar in 128 bits
// (K = lo + 2^128 hi on A and 2^128 A, the same for B): half the windows and half the final
// doubling chain, and no key decompression in k_msm_prep.  Slots are append-only (a slot in
// use by an in-flight or captured batch is never rewritten); when the cache is full a call
// uses the uncached form.  Slot 0 holds B.
struct Key32 {
    uint8_t b[32];
    bool operator==(const Key32& o) const { return std::memcmp(b, o.b, 32) == 0; }
};
// All 32 key bytes, mixed with a per-process random seed: keys chosen to collide in the map
// would otherwise make every lookup under the cache lock linear.
struct Key32Hash {
    size_t operator()(const Key32& k) const {
        static const uint64_t seed = [] {
            std::random_device rd;
            return ((uint64_t)rd() << 32) ^ rd() ^ 0x9E3779B97F4A7C15ull;
        }();
        uint64_t h = seed;
        for (int i = 0; i < 4; i++) {
            uint64_t w;
            std::memcpy(&w, k.b + 8 * i, 8);
            h = (h ^ w) * 0xFF51AFD7ED558CCDull;
            h ^= h >> 32;
        }
        return (size_t)h;
    }
};
struct KeyCache {
    std::mutex mu;
    std::unordered_map<Key32, uint32_t, Key32Hash> slot;
    DevBuf recs;  // cap x KC_SLOT_WORDS words
    uint32_t used = 0, cap = 0;
    bool broken = false;  // allocation or fill failed once: stay uncached
    bool b_ready = false;  // slot 0 (B) filled
    // registered keys' fixed-base comb tables (k_key_comb_fill, COMB_WORDS words each; allocated
    // once at full size, NWV_COMB_KEYS tables, default 1,024 = 64 MiB); comb_of[slot] = table
    DevBuf combs;
    uint32_t comb_cap = 0, comb_used = 0;
    std::vector<uint32_t> comb_of;
    uint64_t reg_fp = 0;  // fingerprint of the last key list registered with every key combed
};

// One device of a context: the basepoint table, the key cache and the pool of lanes (created on
// demand, up to max_lanes; env NWV_LANES, default 4).
struct Gpu {
    int ordinal = -1;
    uint32_t flags = 0;
    DevBuf btab;
    DevBuf comb;  // fixed-base comb table of the MSM's basepoint term (msm.h)
    KeyCache kc;
    std::mutex mu;  // guards the pool
    std::condition_variable cv;
    std::vector<Lane*> lanes, idle;
    size_t max_lanes = 4;
    // staged-run prep chain (NWV_STAGE_CHAIN = k): a ring of k events; run r's prep waits for run
    // r - k's and records into slot r mod k
    std::mutex chain_mu;
    std::vector<hipEvent_t> chain_ev;
    uint64_t chain_runs = 0;
    // diagnostics (nwv_diag_counters): one-launch tiny batches, batch MSMs, per-signature passes
    std::atomic<uint64_t> n_tiny{0}, n_msm{0}, n_each{0};
};

int with_device(Lane& d) {
    NWV_HIP(hipSetDevice(d.ordinal));
    return NWV_OK;
}

void lane_close(Lane& d) {
    if (d.ordinal < 0) return;
    (void)hipSetDevice(d.ordinal);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    d.ed.release();
    d.hstage.release();
    if (d.hstage_ev) (void)hipEventDestroy(d.hstage_ev);
    d.hstage_ev = nullptr;
    if (d.b2stage_ev) (void)hipEventDestroy(d.b2stage_ev);
    d.b2stage_ev = nullptr;
    if (d.aux) (void)hipStreamSynchronize(d.aux);
    for (hipEvent_t* e : {&d.pksig_ev, &d.aux_ev}) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
    }
    if (d.aux) (void)hipStreamDestroy(d.aux);
    d.aux = nullptr;
    if (d.hword) (void)hipHostFree(d.hword);
    d.hword = nullptr;
    d.b2stage.release();
    d.b2dig.release();
    d.tiny_ws.release();
    for (DevBuf* b : {&d.b2_base, &d.b2_off, &d.b2_len, &d.b2_out, &d.b2_packed, &d.b2_plen, &d.b2_err, &d.b2_in})
        b->release();
    if (d.stream) (void)hipStreamDestroy(d.stream);
    d.stream = nullptr;
}

// new lane of g (the calling thread has selected g's device)
int lane_open(Gpu& g, Lane** out) {
    *out = nullptr;
    auto* d = new (std::nothrow) Lane;
    if (!d) return set_err(NWV_ERR_OOM, "lane allocation");
    d->gpu = &g;
    d->ordinal = g.ordinal;
    d->flags = g.flags;
    d->btabp = &g.btab;
    hipError_t e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->hstage_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->b2stage_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&d->aux, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->pksig_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&d->aux_ev, hipEventDisableTiming);
    if (e == hipSuccess &&
        hipHostMalloc(reinterpret_cast<void**>(&d->hword), 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        d->hword = nullptr;  // (optional: the verdict is then copied back)
    // both events start out complete, so the first wait on them returns at once
    if (e == hipSuccess) e = hipEventRecord(d->hstage_ev, d->stream);
    if (e == hipSuccess) e = hipEventRecord(d->b2stage_ev, d->stream);
    if (e != hipSuccess) {
        lane_close(*d);
        delete d;
        return set_err(NWV_ERR_HIP, std::string("lane: ") + hipGetErrorString(e));
    }
    *out = d;
    return NWV_OK;
}

// Exclusive use of one lane of g for the scope of a call: an idle lane, a new one while the pool
// is below max_lanes, else wait for a lane to be returned.
class LaneRef {
  public:
    explicit LaneRef(Gpu& g) : g_(g) {
        std::unique_lock<std::mutex> lk(g.mu);
        for (;;) {
            if (!g.idle.empty()) {
                lane_ = g.idle.back();
                g.idle.pop_back();
                break;
            }
            if (g.lanes.size() < g.max_lanes) {
                Lane* l = nullptr;
                if (hipSetDevice(g.ordinal) != hipSuccess) {
                    rc_ = set_err(NWV_ERR_HIP, "hipSetDevice");
                    return;
                }
                if ((rc_ = lane_open(g, &l))) return;
                g.lanes.push_back(l);
                lane_ = l;
                break;
            }
            g.cv.wait(lk);
        }
        lk.unlock();
        rc_ = with_device(*lane_);
    }
    ~LaneRef() {
        if (!lane_) return;
        {
            std::lock_guard<std::mutex> lk(g_.mu);
            g_.idle.push_back(lane_);
        }
        g_.cv.notify_one();
    }
    LaneRef(const LaneRef&) = delete;
    LaneRef& operator=(const LaneRef&) = delete;
    int rc() const { return rc_; }
    Lane& operator*() const { return *lane_; }

  private:
    Gpu& g_;
    Lane* lane_ = nullptr;
    int rc_ = NWV_OK;
};

int gpu_open(Gpu& g, int ordinal, uint32_t flags) {
    g.ordinal = ordinal;
    g.flags = flags;
    if (const char* e = std::getenv("NWV_LANES")) g.max_lanes = (size_t)std::max(1L, std::strtol(e, nullptr, 10));
    hipDeviceProp_t prop;
    NWV_HIP(hipGetDeviceProperties(&prop, ordinal));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(NWV_ERR_NODEV, std::string("device is ") + prop.gcnArchName + ", need gfx950");
    NWV_HIP(hipSetDevice(ordinal));
    int rc = g.btab.ensure(BTAB_WORDS * sizeof(uint32_t));
    if (rc) return rc;
    Lane* l = nullptr;
    if ((rc = lane_open(g, &l))) return rc;
    g.lanes.push_back(l);
    g.idle.push_back(l);
    hipLaunchKernelGGL(k_base_table, dim3((BASE_TABLE_ENTRIES + 63) / 64), dim3(64), 0, l->stream,
                       g.btab.as<uint32_t>());
    if ((rc = g.comb.ensure((size_t)4 * MSM_PT_WORDS * COMB_TABLES * COMB_ENTRIES))) return rc;
    hipLaunchKernelGGL(k_comb_table, dim3((COMB_TABLES * COMB_ENTRIES + 63) / 64), dim3(64), 0, l->stream,
                       g.comb.as<uint32_t>());
    NWV_HIP(hipGetLastError());
    NWV_HIP(hipStreamSynchronize(l->stream));
    return NWV_OK;
}

void gpu_close(Gpu& g) {
    if (g.ordinal < 0) return;
    (void)hipSetDevice(g.ordinal);
    for (Lane* l : g.lanes) {
        lane_close(*l);
        delete l;
    }
    g.lanes.clear();
    g.idle.clear();
    g.btab.release();
    g.comb.release();
    g.kc.recs.release();
    g.kc.combs.release();
    for (hipEvent_t e : g.chain_ev) (void)hipEventDestroy(e);
    g.chain_ev.clear();
}

// --------------------------------------------------------------- Ed25519 pipeline ------
struct KernelTimes {
    double ms[3] = {0, 0, 0};  // hash, points, straus
    long runs = 0;
};

// Launch the three-phase per-signature pipeline on buffers already resident on `d`.
// Events bracket each kernel on d.stream when `ev` is non-null (ev[0..5]).
// Per-signature scratch (k 32 B, flags 4 B, the 0..8 A and 0..8 R tables = LANE_SCRATCH_WORDS
// = 2 x 9 x 50 words = 3,600 B, verdict bits): about 3.6 KiB per signature, allocated on the
// first per-signature run of a buffer set, so batches that the MSM accepts never hold it.  The
// largest shard the engine stages (a 2,097,152-signature firehose sub-shard, exercised by the
// exact-bad-set GPU tests) takes 7.6 GB of it; the 288 GB HBM holds that many times over.
int ed_scratch(EdBuffers& b, size_t n) {
    int rc;
    if ((rc = b.kbuf.ensure(32 * n + 16)) || (rc = b.flags.ensure(4 * n + 4)) ||
        (rc = b.tables.ensure((size_t)LANE_SCRATCH_WORDS * 4 * n + 16)) ||
        (rc = b.verdict.ensure(8 * ((n + 63) / 64) + 8)))
        return rc;
    return NWV_OK;
}

// msm_pts: the point records of a batch MSM that just ran on these buffers over per-signature
// keys (na = n A points): k_ed_points_msm reuses its decompressions.
// tables_ready: the batch MSM's early form already built the tables (and k, the flags): only the
// Straus pass runs, returning at once when the MSM's state words (gate) say it accepted.
int ed_launch(Lane& d, EdBuffers& b, size_t n, hipStream_t stream, hipEvent_t* ev,
              const uint32_t* msm_pts = nullptr, bool tables_ready = false, const uint32_t* gate = nullptr) {
    if (n == 0) return NWV_OK;
    int rc = ed_scratch(b, n);
    if (rc) return rc;
    const size_t waves = (n + 63) / 64;
    const dim3 blk(256), grid((unsigned)((n + 255) / 256)), grid2((unsigned)((2 * 64 * waves + 255) / 256));
    if (ev) NWV_HIP(hipEventRecord(ev[0], stream));
    if (!msm_pts && !tables_ready)  // (after a batch MSM over per-signature keys, k_msm_prep left k and the flags)
        hipLaunchKernelGGL(k_ed_hash, grid, blk, 0, stream, (uint64_t)n, b.pk.as<uint8_t>(),
                           b.sig.as<uint8_t>(), b.msg.as<uint8_t>(), b.off.as<uint64_t>(),
                           b.len.as<uint32_t>(), b.kbuf.as<uint8_t>(), b.flags.as<uint32_t>());
    if (ev) NWV_HIP(hipEventRecord(ev[1], stream));
    if (tables_ready) {
    } else if (msm_pts)
        hipLaunchKernelGGL(k_ed_points_msm, grid2, blk, 0, stream, (uint64_t)n, (uint64_t)n, msm_pts,
                           b.tables.as<uint32_t>(), b.flags.as<uint32_t>());
    else
        hipLaunchKernelGGL(k_ed_points, grid2, blk, 0, stream, (uint64_t)n, b.pk.as<uint8_t>(),
                           b.sig.as<uint8_t>(), b.tables.as<uint32_t>(), b.flags.as<uint32_t>());
    if (ev) NWV_HIP(hipEventRecord(ev[2], stream));
    static const bool straus_pf = [] {
        const char* e = std::getenv("NWV_STRAUS_PF");  // the prefetching form unless NWV_STRAUS_PF=0
        return !(e && e[0] == '0');
    }();
    hipLaunchKernelGGL(straus_pf ? k_ed_straus_pf : k_ed_straus, grid, blk, 0, stream, (uint64_t)n, b.sig.as<uint8_t>(),
                       b.kbuf.as<uint8_t>(), b.tables.as<uint32_t>(), b.flags.as<uint32_t>(),
                       d.btab().as<uint32_t>(), b.verdict.as<uint64_t>(), gate);
    if (ev) NWV_HIP(hipEventRecord(ev[3], stream));
    NWV_HIP(hipGetLastError());
    return NWV_OK;
}

// ------------------------------------------------------------------ batch MSM (K5) ------
// Window layout and work decomposition of one batch MSM over np = na + 1 + n points (na A
// points: n, or the m distinct keys of a keyed batch).
struct MsmPlan {
    MsmLayout lay{};
    MsmXcdMap xm{};  // k_msm_scatter's windows per XCD group
    uint32_t chunk_pts = 0, chunks = 0, nkeys = 0;
    uint32_t seg = 0;  // entries per k_msm_bucket lane
    uint32_t tail_S = 1;  // k_msm_tail: bucket chunks per window
    uint64_t np = 0, na = 0, cnt_len = 0, max_entries = 0, nseg = 0;
    // two-level counting sort (msm.h): coarse layout lay2 (widths reduced by shift)
    int shift = 0;
    MsmLayout lay2{};
};

// Base width c minimises  7 Fmul x entries + 18 Fmul x buckets  (SURVEY.md §8d K5 cost model:
// one mixed addition per nonzero digit, two full additions per bucket in the running-sum
// reduction).
// split: a keyed batch over the key cache (na = 2m + 1 points before B, every scalar < 2^128):
// only the z range, nw == nw_z.
// sort2: 1 forces the two-level counting sort whenever the sort has more than one chunk (tests),
// 0 lets the size decide (windows of at least NWV_MSM_SORT2_MIN_PTS points, default 2^20)
// batches of at most this many signatures run the tail's butterflies on lane quads throughout
// (latency-bound); larger ones keep lane-local additions (fewer instructions while other batches
// fill the chip) except in the top windows.  NWV_TAIL_QUAD_MAX_N
uint64_t tail_quad_max_n() {
    static const uint64_t v = [] {
        const char* e = std::getenv("NWV_TAIL_QUAD_MAX_N");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)16384;
    }();
    return v;
}

MsmPlan msm_plan(size_t n, size_t na, bool split = false, int sort2 = 0) {
    MsmPlan p;
    p.na = na;
    p.np = (uint64_t)na + 1 + n;
    double best = 1e300;
    const bool narrow_top = n > tail_quad_max_n();  // (msm_split)
    // window widths: ~7 field multiplies per bucket entry against ~18 per bucket (running sums),
    // chosen separately for the z range (all na + 1 + n points) and the range above it (na + 1)
    for (int c_lo = 6; c_lo <= 15; c_lo++)
        for (int c_hi = 3; c_hi <= 15; c_hi++) {
            if (split && c_hi > 3) break;
            MsmLayout L;
            if (!(split ? msm_make_layout_z(c_lo, L) : msm_make_layout2(c_lo, c_hi, L, narrow_top))) continue;
            const double entries = (double)(na + 1) * L.nw + (double)n * L.nw_z;
            const double cost = 7.0 * entries + 18.0 * L.kbase[L.nw];
            if (cost < best) {
                best = cost;
                p.lay = L;
            }
        }
    p.chunk_pts = (uint32_t)std::max<uint64_t>(8192, (p.np + 63) / 64);
    p.chunks = (uint32_t)((p.np + p.chunk_pts - 1) / p.chunk_pts);
    msm_xcd_map(p.lay, n, na, p.chunk_pts, p.xm);
    p.nkeys = p.lay.kbase[p.lay.nw];
    p.cnt_len = (uint64_t)p.nkeys * p.chunks;
    // two-level sort: at most 128 coarse bins per window (bins of 2^shift buckets).  A scatter
    // workgroup keeps one partly written line open per bin; with 128 bins the open lines of all
    // the workgroups on an XCD stay well inside its 4 MB L2, so each line is written back whole
    // (1,024 bins measured 6.3x the entry bytes written at 2M, from L2 evictions)
    static const uint64_t sort2_min = [] {
        const char* e = std::getenv("NWV_MSM_SORT2_MIN_PTS");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)1 << 20;
    }();
    if (p.chunks > 1 && (sort2 == 1 || p.np >= sort2_min)) {
        int lgc = 0;
        while (lgc < 7 && ((uint64_t)1 << (lgc + 1)) <= p.chunk_pts / 64) lgc++;
        int cmin = 99;
        for (int w = 0; w < p.lay.nw; w++) cmin = std::min(cmin, (int)p.lay.width[w]);
        int sh = std::min(MSM_SORT2_MAX_SHIFT, std::max(0, (p.lay.cmax - 1) - lgc));
        if (sort2 == 1) sh = std::max(sh, 2);
        sh = std::min(sh, cmin - 1);
        if (sh >= 2 && p.np < ((uint64_t)1 << (31 - sh))) {
            p.shift = sh;
            p.lay2 = p.lay;
            uint32_t kb = 0;
            int cm = 0;
            for (int w = 0; w < p.lay.nw; w++) {
                p.lay2.width[w] = (uint8_t)(p.lay.width[w] - sh);
                p.lay2.kbase[w] = kb;
                kb += 1u << (p.lay2.width[w] - 1);
                cm = std::max(cm, (int)p.lay2.width[w]);
            }
            p.lay2.kbase[p.lay.nw] = kb;
            p.lay2.cmax = cm;
            p.cnt_len = (uint64_t)kb * p.chunks;
        }
    }
    p.max_entries = (uint64_t)(na + 1) * p.lay.nw + (uint64_t)n * p.lay.nw_z;
    // ~2 waves per SIMD of bucket lanes (256 CUs x 4 SIMDs x 2 x 64), 8..64 entries each
    p.seg = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(8, p.max_entries / (256 * 4 * 2 * 64)));
    // tiny batches (a certificate's few signatures): nearly every bucket is empty, and each lane's
    // segment close walks to the next non-empty bucket by dependent loads; two entries a lane
    // (C1 Certificate::verify n = 4: p50 0.191 -> 0.184 ms; a 1K batch is slower below 8)
    if (p.max_entries <= 2048) p.seg = 2;
    if (const char* e = std::getenv("NWV_MSM_SEG")) p.seg = (uint32_t)std::max(1L, std::strtol(e, nullptr, 10));
    p.nseg = (p.max_entries + p.seg - 1) / p.seg;
    // tail: chunks of at most 256 buckets (one per lane of a k_msm_tail workgroup)
    p.tail_S = 1;
    while (((1u << (p.lay.cmax - 1)) / p.tail_S) > 256) p.tail_S <<= 1;
    if (const char* e = std::getenv("NWV_MSM_TAIL_S")) {
        const long v = std::strtol(e, nullptr, 10);  // only larger (smaller chunks) than the minimum
        while (p.tail_S < 64 && (long)(p.tail_S << 1) <= v) p.tail_S <<= 1;
    }
    return p;
}

// points before B: the A points (n, or the m distinct keys), or A and 2^128 A per cached key
// and 2^128 B (split form)
size_t msm_na(const EdBuffers& b, size_t n) {
    if (!b.nkeys_distinct) return n;
    return b.kc_split ? 2 * b.nkeys_distinct + 1 : b.nkeys_distinct;
}

constexpr size_t MSM_CTR_BYTES = 512;  // k_msm_tail arrival counters (128 words)

int msm_alloc(EdBuffers& b, const MsmPlan& p, size_t n) {
    const size_t nblk = (n + 63) / 64;  // k_msm_prep's hash workgroups (64 or 256 threads)
    int rc;
    if ((b.nkeys_distinct && (rc = b.m_ascal.ensure(32 * n + 32))) || (rc = b.m_partial.ensure(36 * nblk + 36)) ||
        (rc = b.m_state.ensure(128)) ||
        (rc = b.m_pts.ensure((size_t)4 * MSM_PT_WORDS * p.np + 64)) ||
        (rc = b.m_digits.ensure((size_t)2 * p.lay.nw * p.np + 64)) ||
        (p.chunks > 1 && (rc = b.m_cnt.ensure((size_t)4 * (p.cnt_len + (size_t)p.lay.nw * p.chunks) + 64))) ||
        (rc = b.m_tiles.ensure((size_t)4 * (MSM_MAX_WINDOWS + 1) + 64)) ||
        (rc = b.m_entries.ensure((size_t)4 * p.max_entries + 64)) ||
        (p.shift && (rc = b.m_mid.ensure((size_t)4 * p.max_entries + 64))) ||
        (p.shift && (rc = b.m_kst2.ensure((size_t)4 * p.lay2.kbase[p.lay2.nw] + 64))) ||
        (rc = b.m_kstart.ensure((size_t)4 * p.nkeys + 64)) ||
        (rc = b.m_hpart.ensure((size_t)4 * P3_WORDS * p.nseg + 64)) ||
        (p.chunks == 1 && (rc = b.m_segkey.ensure((size_t)4 * p.nseg + 64))) ||
        (rc = b.m_bsum.ensure((size_t)4 * P3_WORDS * p.nkeys + 64)) ||
        (rc = b.m_wsum.ensure((size_t)4 * 64 * (2 * p.lay.nw + 1) + 64)) ||
        (rc = b.m_tpart.ensure((size_t)4 * P3_WORDS * TAIL_PART_SLOTS * p.lay.nw * p.tail_S + 64)) ||
        (rc = b.m_ctr.ensure(MSM_CTR_BYTES)))
        return rc;
    return NWV_OK;
}

static const char* const ED_KERNEL_NAMES[] = {"k_ed_hash", "k_ed_points", "k_ed_straus"};
// event slots of one batch MSM; nullptr = no kernel in that slot (k_msm_prep runs the hash and
// the decompression as one grid unless NWV_FLAG_MSM_SPLIT_PREP)
static const char* const MSM_KERNEL_NAMES[] = {
    "k_msm_prep", nullptr, nullptr, "k_msm_hist", "k_msm_wscan",
    "k_msm_scatter", "k_msm_bucket", "k_msm_tail", nullptr};
static const char* const MSM_KERNEL_NAMES_SPLIT[] = {
    "k_msm_scalars", nullptr, "k_msm_points", "k_msm_hist", "k_msm_wscan",
    "k_msm_scatter", "k_msm_bucket", "k_msm_tail", nullptr};
constexpr int MSM_NKERNELS = 9;
constexpr int MSM_NEVENTS = MSM_NKERNELS + 1;  // one event before each kernel, one after the last

// Launch the batch MSM on resident buffers; the verdict word (1 = batch accepted) is
// m_state[1] (m_state[0] = failure flags).  ev: MSM_NEVENTS events or null.
// Early form (a piped staging left pksig_pending: pk and sig landed before the messages): the
// decompressions (k_msm_points) start on the lane's aux stream as soon as pk and sig are on the
// device, under the messages' PCIe transfer, and -- spec_tables, the caller wants verdict bits --
// so does the per-signature fallback's table build from their records (k_ed_points_msm, ~0.13 ms
// at 65,536 that a rejected batch no longer waits for); the hash role (k_msm_scalars) runs when
// the messages are in, and the sort waits for both.
int msm_launch(Lane& d, EdBuffers& b, size_t n, const uint8_t seed32[32], hipStream_t stream,
               hipEvent_t* ev, bool state_ready, bool spec_tables = false, uint32_t* hverdict = nullptr,
               uint32_t hseq = 0) {
    const bool pksig = d.pksig_pending;
    d.pksig_pending = false;
    b.tables_ready = false;
    if (n == 0) return NWV_OK;
    const size_t na = msm_na(b, n);
    const MsmPlan p = msm_plan(n, na, b.kc_split, (d.flags & NWV_FLAG_MSM_SORT2) ? 1 : 0);
    int rc = msm_alloc(b, p, n);
    if (rc) return rc;
    // [0] fail flags, [1] verdict, [2..4) accepted / rejected run tally, [8..16) seed
    uint32_t* state = b.m_state.as<uint32_t>();
    if (seed32 && !state_ready) NWV_HIP(hipMemcpyAsync(state + 8, seed32, 32, hipMemcpyHostToDevice, stream));
    auto mark = [&](int k) -> int {
        if (ev) NWV_HIP(hipEventRecord(ev[k], stream));
        return NWV_OK;
    };
    if (!state_ready) NWV_HIP(hipMemsetAsync(state, 0, 8, stream));
    if ((rc = mark(0))) return rc;
    int16_t* digits = b.m_digits.as<int16_t>();
    const int keyed = b.nkeys_distinct ? 1 : 0;
    // per-signature keys: the hash role also leaves k_i and the s < l flag for the fallback
    const bool reuse = !keyed && !(d.flags & NWV_FLAG_NO_MSM_REUSE);
    if (reuse && ((rc = b.kbuf.ensure(32 * n + 16)) || (rc = b.flags.ensure(4 * n + 4)))) return rc;
    const bool early = pksig && reuse && !b.kc_split && stream == d.stream && !ev && state_ready &&
                       !(d.flags & NWV_FLAG_NO_EARLY_PREP);
    if (early && spec_tables && (rc = ed_scratch(b, n))) return rc;
    MsmScalarArgs gs{(uint64_t)n, (uint64_t)na, keyed, b.pk.as<uint8_t>(), b.sig.as<uint8_t>(),
                           b.msg.as<uint8_t>(), b.off.as<uint64_t>(), b.len.as<uint32_t>(), state + 8,
                           b.m_ascal.as<uint32_t>(), digits, b.m_partial.as<uint32_t>(), state,
                           b.kc_split ? 1u : 0u, b.m_ctr.as<uint32_t>(), reuse ? b.kbuf.as<uint32_t>() : nullptr,
                           reuse ? b.flags.as<uint32_t>() : nullptr, early ? 1u : 0u};
    // decompression on 16-lane rows when the batch is small enough to be latency-bound
    static const uint64_t row_prep_max = [] {
        const char* e = std::getenv("NWV_MSM_ROW_PREP_MAX");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)8192;
    }();
    const uint64_t ndec = b.kc_split ? 0 : (uint64_t)na;
    const bool rows = !(d.flags & NWV_FLAG_NO_ROW_PREP) && n + ndec <= row_prep_max;
    const MsmPointArgs gp{(uint64_t)n, (uint64_t)na, ndec, keyed ? b.keys.as<uint8_t>() : b.pk.as<uint8_t>(),
                          b.sig.as<uint8_t>(), b.m_pts.as<uint32_t>(), state, rows ? 1u : 0u};
    // row form: single-wave workgroups (a wave alone on its CU decompresses faster than four
    // waves of one workgroup sharing a CU), so the fused grid's hash role uses 64 threads too
    const unsigned pthr = rows ? 64u : 256u;
    const size_t waves = (n + 63) / 64 + (na + 63) / 64;
    const unsigned sblk = (unsigned)((n + pthr - 1) / pthr);  // hash workgroups (k_msm_tail's partials)
    const unsigned pblk = rows ? (unsigned)((n + ndec + 3) / 4) : (unsigned)((64 * waves + 255) / 256);
    const bool fused = !(d.flags & NWV_FLAG_MSM_SPLIT_PREP) && !early;
    const uint32_t* kc = b.kc_split ? d.gpu->kc.recs.as<uint32_t>() : nullptr;
    // a keyed batch whose hashes fit one workgroup: its key sums run in that workgroup
    // (MsmScalarArgs::fuse_keysum) instead of a k_msm_keysum launch
    if (keyed && fused && sblk == 1 && b.nkeys_distinct <= pthr && !(d.flags & NWV_FLAG_NO_FUSED_KEYSUM)) {
        gs.fuse_keysum = 1u;
        gs.nkeys = (uint32_t)b.nkeys_distinct;
        gs.key_off = b.koff.as<uint32_t>();
        gs.key_sig = b.ksig.as<uint32_t>();
        gs.kslot = b.kslot.as<uint32_t>();
        gs.kc = kc;
        gs.pts = b.m_pts.as<uint32_t>();
    }
    if (early) {
        NWV_HIP(hipStreamWaitEvent(d.aux, d.pksig_ev, 0));
        hipLaunchKernelGGL(k_msm_points, dim3(pblk), dim3(pthr), 0, d.aux, gp);
        if (spec_tables) {
            const size_t waves2 = 2 * 64 * ((n + 63) / 64);
            hipLaunchKernelGGL(k_ed_points_msm, dim3((unsigned)((waves2 + 255) / 256)), dim3(256), 0, d.aux, (uint64_t)n,
                               (uint64_t)n, b.m_pts.as<uint32_t>(), b.tables.as<uint32_t>(), b.flags.as<uint32_t>());
            b.tables_ready = true;
        }
        NWV_HIP(hipEventRecord(d.aux_ev, d.aux));
        hipLaunchKernelGGL(k_msm_scalars, dim3(sblk), dim3(pthr), 0, stream, gs, p.lay);
        NWV_HIP(hipStreamWaitEvent(stream, d.aux_ev, 0));
    } else if (fused) {
        if (d.chain_wait) NWV_HIP(hipStreamWaitEvent(stream, d.chain_wait, 0));
        hipLaunchKernelGGL(k_msm_prep, dim3(sblk + pblk), dim3(pthr), 0, stream, gs, p.lay, gp, sblk);
        if (d.chain_rec) NWV_HIP(hipEventRecord(d.chain_rec, stream));
    } else {
        hipLaunchKernelGGL(k_msm_scalars, dim3(sblk), dim3(pthr), 0, stream, gs, p.lay);
    }
    if (keyed && !gs.fuse_keysum)
        hipLaunchKernelGGL(k_msm_keysum, dim3((unsigned)b.nkeys_distinct), dim3(256), 0, stream, (uint64_t)n,
                           (uint64_t)na, p.lay, b.koff.as<uint32_t>(), b.ksig.as<uint32_t>(), b.m_ascal.as<uint32_t>(),
                           digits, (uint32_t)b.nkeys_distinct, b.kslot.as<uint32_t>(), kc, b.m_pts.as<uint32_t>(),
                           state);
    if ((rc = mark(1))) return rc;
    if ((rc = mark(2))) return rc;
    if (!fused && !early) hipLaunchKernelGGL(k_msm_points, dim3(pblk), dim3(pthr), 0, stream, gp);
    if ((rc = mark(3))) return rc;
    const size_t lds_nb = (size_t)4 << (p.lay.cmax - 1);
    uint32_t* kst = b.m_kstart.as<uint32_t>();
    uint32_t* tot = b.m_tiles.as<uint32_t>();  // [nw] entries per window, [MSM_MAX_WINDOWS] all
    uint32_t* ent = b.m_entries.as<uint32_t>();
    if (p.chunks == 1) {
        // one chunk per window: the whole counting sort of a window in one workgroup (timed in
        // the k_msm_hist slot)
        hipLaunchKernelGGL(k_msm_sort1, dim3((unsigned)p.lay.nw), dim3(1024), lds_nb, stream, (uint64_t)n,
                           (uint64_t)na, p.lay, digits, kst, tot, ent, p.seg, b.m_segkey.as<uint32_t>(), state);
        if ((rc = mark(4))) return rc;
        if ((rc = mark(5))) return rc;
    } else {
        uint32_t* cnt = b.m_cnt.as<uint32_t>();
        uint32_t* nzc = cnt + p.cnt_len;  // [nw][chunks] nonzero digits per histogram workgroup
        // two-level form: the first level sorts coarse bins (lay2) into mid, k_msm_lsort the rest
        const MsmLayout& l1 = p.shift ? p.lay2 : p.lay;
        const size_t lds1 = (size_t)4 << (l1.cmax - 1);
        uint32_t* kst1 = p.shift ? b.m_kst2.as<uint32_t>() : kst;
        uint32_t* ent1 = p.shift ? b.m_mid.as<uint32_t>() : ent;
        hipLaunchKernelGGL(k_msm_hist, dim3(p.chunks, (unsigned)p.lay.nw), dim3(256), lds1, stream, (uint64_t)n,
                           (uint64_t)na, l1, p.chunk_pts, digits, cnt, nzc, p.shift, state);
        if ((rc = mark(4))) return rc;
        // per window: entry base, bucket totals -> scan -> absolute (bucket, chunk) slice offsets
        hipLaunchKernelGGL(k_msm_wscan, dim3((unsigned)p.lay.nw), dim3(1024), 0, stream, l1, p.chunks, cnt, nzc,
                           kst1, tot, state);
        if ((rc = mark(5))) return rc;
        hipLaunchKernelGGL(k_msm_scatter, dim3(MSM_XCD_GROUPS * p.xm.slots), dim3(256), lds1, stream, (uint64_t)n,
                           (uint64_t)na, l1, p.xm, p.chunks, p.chunk_pts, digits, cnt, ent1, p.shift, state);
        if (p.shift)  // timed with k_msm_scatter
            hipLaunchKernelGGL(k_msm_lsort, dim3(1u << (p.lay2.cmax - 1), (unsigned)p.lay.nw), dim3(256), 0, stream,
                               p.lay, p.lay2, p.shift, ent1, kst1, tot, ent, kst, state);
    }
    if ((rc = mark(6))) return rc;
    const uint32_t* E = tot + MSM_MAX_WINDOWS;
    const uint32_t* seg_key = p.chunks == 1 ? b.m_segkey.as<uint32_t>() : nullptr;
    // bucket sums on quads where they are latency-bound (small batches), else one lane per chunk
    static const uint64_t bucket_quad_max_n = [] {
        const char* e = std::getenv("NWV_BUCKET_QUAD_MAX_N");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)4096;
    }();
    if (n <= bucket_quad_max_n)  // single-wave workgroups: spread over the CUs (see k_msm_prep's row form)
        hipLaunchKernelGGL(k_msm_bucket_q, dim3((unsigned)((p.nseg + 15) / 16)), dim3(64), 0, stream, p.seg,
                           p.nkeys, E, ent, kst, b.m_pts.as<uint32_t>(), b.m_bsum.as<uint32_t>(),
                           b.m_hpart.as<uint32_t>(), seg_key, state);
    else
        hipLaunchKernelGGL(k_msm_bucket, dim3((unsigned)((p.nseg + 255) / 256)), dim3(256), 0, stream, p.seg,
                           p.nkeys, E, ent, kst, b.m_pts.as<uint32_t>(), b.m_bsum.as<uint32_t>(),
                           b.m_hpart.as<uint32_t>(), seg_key, state);
    if ((rc = mark(7))) return rc;
    // window sums, their scaling, the basepoint term and the verdict: one launch (its arrival
    // counters were zeroed by k_msm_prep's first workgroup, graph replays included)
    static const bool stamps = std::getenv("NWV_TAIL_STAMPS") != nullptr;  // diagnostics only
    unsigned long long* st_buf = nullptr;
    if (stamps && (rc = b.m_stamps.ensure(8 * 8 * (size_t)MSM_MAX_WINDOWS))) return rc;
    if (stamps) {
        st_buf = b.m_stamps.as<unsigned long long>();
        NWV_HIP(hipMemsetAsync(st_buf, 0, 8 * 8 * (size_t)MSM_MAX_WINDOWS, stream));
    }
    // quad-lane butterflies where the tail is latency-bound (small batches, tail_quad_max_n)
    const uint32_t quad_max_c = n <= tail_quad_max_n() ? 256u : 0u;
    // the top windows' butterflies precede the longest chains: on quads at any size where they
    // take one quad pass a level (NWV_TAIL_QUAD_TOP_C, 0 = never)
    static const uint32_t quad_top_c = [] {
        const char* e = std::getenv("NWV_TAIL_QUAD_TOP_C");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 128u;
    }();
    // NWV_TAIL_SPIN_LIMIT (test hook): the _spin1 kernels, whose final-sum wave gives up on a window
    // at its first poll -- the undetermined outcome
    static const bool spin1 = std::getenv("NWV_TAIL_SPIN_LIMIT") != nullptr;
    const MsmTailArgs ta{b.m_bsum.as<uint32_t>(), b.m_hpart.as<uint32_t>(), kst, E, p.nkeys, p.seg,
                         b.m_tpart.as<uint32_t>(), b.m_wsum.as<uint32_t>(),
                         b.m_ctr.as<uint32_t>(), state, b.m_partial.as<uint32_t>(),
                         d.gpu->comb.as<uint32_t>(), sblk, quad_max_c, state + 1, state + 2, p.tail_S, st_buf,
                         hverdict, quad_top_c, hseq & 0x3FFFFFFFu};
    // combine items per thread: (lg C + 1) x S_w over the windows (C = nb / S_w buckets per chunk)
    int items = 0;
    for (int w = 0; w < p.lay.nw; w++) {
        const int nb = 1 << (p.lay.width[w] - 1), Sw = (int)p.tail_S < nb ? (int)p.tail_S : nb;
        int lgC = 0;
        while ((1 << lgC) < nb / Sw) lgC++;
        items = std::max(items, (lgC + 1) * Sw);
    }
    if (items <= 256)
        hipLaunchKernelGGL(spin1 ? k_msm_tail_spin1 : k_msm_tail, dim3(p.tail_S, (unsigned)p.lay.nw + 1), dim3(256),
                           (size_t)4 * (256 * P3_WORDS + 4), stream, p.lay, ta);
    else
        hipLaunchKernelGGL(spin1 ? k_msm_tail_wide_spin1 : k_msm_tail_wide, dim3(p.tail_S, (unsigned)p.lay.nw + 1),
                           dim3(256), (size_t)4 * (256 * P3_WORDS + 4), stream, p.lay, ta);
    if ((rc = mark(8))) return rc;
    if ((rc = mark(9))) return rc;
    NWV_HIP(hipGetLastError());
    return NWV_OK;
}

// Persistent helper threads for the host-side staging copies (created once per process, on first
// use): a call hands its piece loop to the pool and works on it too, instead of creating threads
// per call (thread start-up was a visible share of a 40 MB staging).  One call uses the pool at a
// time; a concurrent call finds it busy and copies alone.
class StagePool {
  public:
    static StagePool& get() {
        static StagePool* p = new StagePool();  // never destroyed: helpers may outlive static teardown
        return *p;
    }
    // fn(helper) on the caller and on up to kHelpers pool threads; returns once every started
    // helper has finished.  Returns false (fn not run) when the pool is busy.
    template <class F>
    bool run(F&& fn) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (!started_) start();
            job_ = std::function<void(bool)>(fn);
            open_ = true;
            taken_ = finished_ = 0;
            gen_++;
        }
        cv_.notify_all();
        fn(false);
        std::unique_lock<std::mutex> g(mu_);
        open_ = false;  // no helper starts on this job from now on
        done_.wait(g, [&] { return finished_ == taken_; });
        job_ = nullptr;
        return true;
    }

  private:
    static constexpr int kHelpers = 15;
    void start() {
        started_ = true;
        for (int t = 0; t < kHelpers; t++) {
            try {
                std::thread(&StagePool::loop, this).detach();
            } catch (...) {  // fewer helpers (never throw across the C ABI)
                break;
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            if (!open_ || !job_) continue;
            taken_++;
            std::function<void(bool)> fn = job_;
            g.unlock();
            fn(true);
            g.lock();
            ++finished_;
            done_.notify_all();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    std::function<void(bool)> job_;
    uint64_t gen_ = 0;
    int taken_ = 0, finished_ = 0;
    bool open_ = false, started_ = false;
};

// fn(helper) over the staging pool, or -- the pool busy with another call's staging (batches in
// flight on several lanes or devices) -- over a few helper threads of this call's own, so that
// concurrent large stagings do not drop to one copying thread each
template <class F>
static void stage_run(F&& work) {
    if (StagePool::get().run(work)) return;
    constexpr int kOwn = 3;
    std::vector<std::thread> th;
    for (int t = 0; t < kOwn; t++) {
        try {
            th.emplace_back([&work] { work(true); });
        } catch (...) {
            break;  // no thread: the others (and the caller) take the pieces
        }
    }
    work(false);
    for (auto& t : th) t.join();
}

// Host-side packing copy into the pinned staging buffer: a 65,536 x 512 B batch is ~40 MB, which
// one thread copies at a few GB/s (longer than the PCIe transfer and the batch MSM together), so
// copies above 4 MiB are split into 2 MiB pieces over the staging pool.
static void pack_copy(uint8_t* dst, const uint8_t* src, size_t bytes) {
    constexpr size_t kMin = (size_t)4 << 20, kPiece = (size_t)2 << 20;
    if (bytes < kMin) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const size_t np = (bytes + kPiece - 1) / kPiece;
    std::atomic<size_t> next{0};
    auto work = [&](bool) {
        for (size_t k; (k = next.fetch_add(1)) < np;)
            std::memcpy(dst + k * kPiece, src + k * kPiece, std::min(kPiece, bytes - k * kPiece));
    };
    stage_run(work);
}

// Large message regions: packing into pinned memory and the H2D DMA overlap.  The caller and the
// staging pool's threads take 2 MiB pieces in order, copy each into the pinned buffer and queue its
// DMA on `stream` at once, so the copy engine starts on the first pieces while the rest are packed
// (C4, 33.5 MB of messages: pack ~0.74 ms then DMA ~0.72 ms back to back before).
struct PackSeg {
    size_t off;          // offset in the arena (host and device alike)
    const uint8_t* src;  // caller's bytes
    size_t len;
};
static int pack_copy_h2d(int ordinal, uint8_t* dev_base, uint8_t* host_base, const std::vector<PackSeg>& segs,
                         hipStream_t stream) {
    constexpr size_t kPiece = (size_t)2 << 20;
    std::vector<PackSeg> pieces;
    for (const PackSeg& g : segs)
        for (size_t o = 0; o < g.len; o += kPiece)
            pieces.push_back(PackSeg{g.off + o, g.src + o, std::min(kPiece, g.len - o)});
    std::atomic<size_t> next{0}, done{0};
    std::atomic<int> err{0};
    auto work = [&](bool helper) {
        // a helper that cannot select the device takes no piece (the others copy them all)
        if (helper && hipSetDevice(ordinal) != hipSuccess) return;
        for (size_t k; (k = next.fetch_add(1)) < pieces.size(); done.fetch_add(1)) {
            const PackSeg& q = pieces[k];
            std::memcpy(host_base + q.off, q.src, q.len);
            if (hipMemcpyAsync(dev_base + q.off, host_base + q.off, q.len, hipMemcpyHostToDevice, stream) !=
                hipSuccess)
                err.store(1);
        }
    };
    if (pieces.size() < 2) work(false);
    else stage_run(work);
    return (err.load() || done.load() != pieces.size()) ? set_err(NWV_ERR_HIP, "pipelined staging copy") : NWV_OK;
}

// Stage host inputs [lo, hi) onto buffers b of device d (message region rebased).  pk/sig
// may be null (signing stages seeds separately).  Everything is packed into the pinned host
// buffer and crosses PCIe as ONE async copy into b.in on d.stream (pk, sig, off, len, msg and,
// with seed32, the MSM state words are views into it); no synchronisation here: work on other
// streams must wait for d.stream.  seed32 (optional): m_state = {0 flags, 0 verdict, .., seed}
// so that msm_launch(state_ready) needs neither a memset nor a seed copy.
// Keyed batches' per-call tables (distinct keys, CSR of signatures per key), packed into the
// same arena so that a keyed batch still crosses PCIe as one copy with no host synchronisation
struct KeyedTail {
    const uint8_t* keys;   // m x 32
    size_t m;
    const uint32_t* koff;  // m + 1
    const uint32_t* ksig;  // n
    const uint32_t* kslot;  // m key cache slots, or null (uncached)
};

int ed_stage(Lane& d, EdBuffers& b, size_t lo, size_t hi, const uint8_t* pk, const uint8_t* sig,
             const uint8_t* msg_base, const uint64_t* msg_off, const uint32_t* msg_len,
             const uint8_t* seed32, const KeyedTail* kt = nullptr, const DevBuf* dev_msg = nullptr) {
    const size_t n = hi - lo;
    uint64_t mlo = UINT64_MAX, mhi = 0;
    for (size_t i = lo; i < hi; i++) {
        mlo = std::min<uint64_t>(mlo, msg_off[i]);
        mhi = std::max<uint64_t>(mhi, msg_off[i] + msg_len[i]);
    }
    if (n == 0 || mhi < mlo) { mlo = 0; mhi = 0; }
    // dev_msg: the messages are already on the device (offsets index it as they are)
    if (dev_msg) {
        if (mhi + MSG_PAD > dev_msg->cap) return set_err(NWV_ERR_ARG, "device message offset out of range");
        mlo = 0;
        mhi = 0;
    }
    const size_t mbytes = (size_t)(mhi - mlo);
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const bool inputs = pk && sig;
    const size_t o_pk = 0, o_sig = o_pk + (inputs ? up(32 * n + 16) : 0);
    const size_t o_off = o_sig + (inputs ? up(64 * n + 16) : 0), o_len = o_off + up(8 * n + 8);
    const size_t o_state = o_len + up(4 * n + 4), o_msg = o_state + 256, o_keys = up(o_msg + mbytes + MSG_PAD);
    const size_t m = kt ? kt->m : 0;
    const size_t o_koff = o_keys + (kt ? up(32 * m + 32) : 0), o_ksig = o_koff + (kt ? up(4 * m + 8) : 0);
    const size_t o_kslot = o_ksig + (kt ? up(4 * n + 8) : 0);
    const size_t total = o_kslot + (kt && kt->kslot ? up(4 * m + 8) : 0);
    int rc;
    if ((rc = b.in.ensure(total))) return rc;
    // views into the arena are stale once it may have moved: drop the ones not re-pointed below
    if (!inputs && b.pk.view) b.pk.release();
    if (!inputs && b.sig.view) b.sig.release();
    if (!seed32 && b.m_state.view) b.m_state.release();
    if (!kt)
        for (DevBuf* v : {&b.keys, &b.koff, &b.ksig})
            if (v->view) v->release();
    if ((!kt || !kt->kslot) && b.kslot.view) b.kslot.release();
    if (!inputs && ((rc = b.pk.ensure(32 * n + 16)) || (rc = b.sig.ensure(64 * n + 16)))) return rc;
    // the previous call's copy must have left the pinned buffer before it is rewritten
    htrace("stage:ensure");
    NWV_HIP(hipEventSynchronize(d.hstage_ev));
    if ((rc = d.hstage.ensure(total))) return rc;
    uint8_t* h = static_cast<uint8_t*>(d.hstage.p);
    d.pksig_pending = false;
    b.tables_ready = false;
    b.tiny = false;
    // large stagings: the caller's pk / sig / message bytes are packed piece by piece with each
    // piece's DMA queued at once (pack_copy_h2d); the small computed regions go first
    const bool piped = 96 * (inputs ? n : 0) + mbytes >= ((size_t)16 << 20);
    if (inputs && !piped) {
        pack_copy(h + o_pk, pk + 32 * lo, 32 * n);
        pack_copy(h + o_sig, sig + 64 * lo, 64 * n);
    }
    uint64_t* hoff = reinterpret_cast<uint64_t*>(h + o_off);
    for (size_t i = 0; i < n; i++) hoff[i] = msg_off[lo + i] - mlo;
    std::memcpy(h + o_len, msg_len + lo, 4 * n);
    std::memset(h + o_state, 0, 256);
    if (seed32) std::memcpy(h + o_state + 32, seed32, 32);
    if (mbytes && !piped) pack_copy(h + o_msg, msg_base + mlo, mbytes);
    std::memset(h + o_msg + mbytes, 0, MSG_PAD);
    if (kt) {
        if (m) std::memcpy(h + o_keys, kt->keys, 32 * m);
        std::memcpy(h + o_koff, kt->koff, 4 * (m + 1));
        if (n) std::memcpy(h + o_ksig, kt->ksig, 4 * n);
        if (kt->kslot) std::memcpy(h + o_kslot, kt->kslot, 4 * m);
    }
    htrace("stage:packed");
    if (piped) {
        // offsets, lengths and MSM state, then pk / sig / messages piece by piece as they are
        // packed, then the padding and keyed tables behind them (the early form's flag words are
        // allocated before the first copy: an error return must not leave a copy reading `h`)
        if (inputs && !kt && (rc = b.flags.ensure(4 * n + 4))) return rc;
        uint8_t* gdev = b.in.as<uint8_t>();
        NWV_HIP(hipMemcpyAsync(gdev + o_off, h + o_off, o_msg - o_off, hipMemcpyHostToDevice, d.stream));
        // pk and sig (and the fallback's zeroed flag words) ahead of the messages: pksig_ev lets the
        // batch MSM decompress while the messages are still in flight
        int prc = NWV_OK;
        if (inputs && !kt) {
            NWV_HIP(hipMemsetAsync(b.flags.p, 0, 4 * n + 4, d.stream));
            prc = pack_copy_h2d(d.ordinal, gdev, h, {PackSeg{o_pk, pk + 32 * lo, 32 * n}, PackSeg{o_sig, sig + 64 * lo, 64 * n}},
                                d.stream);
            if (!prc && hipEventRecord(d.pksig_ev, d.stream) == hipSuccess) d.pksig_pending = true;
        } else if (inputs) {
            prc = pack_copy_h2d(d.ordinal, gdev, h, {PackSeg{o_pk, pk + 32 * lo, 32 * n}, PackSeg{o_sig, sig + 64 * lo, 64 * n}},
                                d.stream);
        }
        if (!prc && mbytes) prc = pack_copy_h2d(d.ordinal, gdev, h, {PackSeg{o_msg, msg_base + mlo, mbytes}}, d.stream);
        if (prc) {
            // copies already queued may still read the pinned buffer: the next staging waits
            (void)hipEventRecord(d.hstage_ev, d.stream);
            return prc;
        }
        NWV_HIP(hipMemcpyAsync(gdev + o_msg + mbytes, h + o_msg + mbytes, total - o_msg - mbytes,
                               hipMemcpyHostToDevice, d.stream));
    } else {
        NWV_HIP(nwv_stage::stage_h2d(b.in.p, h, total, d.stream));  // small calls: through kernel arguments
    }
    NWV_HIP(hipEventRecord(d.hstage_ev, d.stream));
    htrace("stage:copy-issued");
    uint8_t* g = b.in.as<uint8_t>();
    if (inputs) {
        b.pk.set_view(g + o_pk, 32 * n + 16);
        b.sig.set_view(g + o_sig, 64 * n + 16);
    }
    b.off.set_view(g + o_off, 8 * n + 8);
    b.len.set_view(g + o_len, 4 * n + 4);
    if (dev_msg) b.msg.set_view(dev_msg->p, dev_msg->cap);
    else b.msg.set_view(g + o_msg, mbytes + MSG_PAD);
    if (seed32) b.m_state.set_view(g + o_state, 256);
    if (kt) {
        b.keys.set_view(g + o_keys, 32 * m + 32);
        b.koff.set_view(g + o_koff, 4 * m + 8);
        b.ksig.set_view(g + o_ksig, 4 * n + 8);
        if (kt->kslot) b.kslot.set_view(g + o_kslot, 4 * m + 8);
    }
    b.nkeys_distinct = m;
    b.kc_split = kt && kt->kslot && m;
    return NWV_OK;
}

// Cache slots of m distinct keys on d's device (misses are filled first, on d.stream, under the
// cache lock); out is left empty when the call should go uncached (cache disabled or full, or
// more keys than NWV_KEYCACHE_MAX_KEYS: a batch of mostly fresh keys would pay 128 doublings
// per key for nothing).  lookup_only: use the cache only if every key is already in it (single
// verifies: a one-off or undecodable key must neither take a slot for good nor make the call
// wait for a fill under the device-wide lock).
int keycache_slots(Lane& d, const uint8_t* keys, size_t m, std::vector<uint32_t>& out, bool lookup_only = false) {
    out.clear();
    static const long max_keys = [] {
        const char* e = std::getenv("NWV_KEYCACHE_MAX_KEYS");
        return e ? std::strtol(e, nullptr, 10) : 4096L;
    }();
    if (m == 0 || (d.flags & NWV_FLAG_NO_KEYCACHE) || (long)m > max_keys) return NWV_OK;
    KeyCache& kc = d.gpu->kc;
    std::lock_guard<std::mutex> g(kc.mu);
    if (kc.broken) return NWV_OK;
    if (lookup_only) {
        if (!kc.cap || !kc.b_ready) return NWV_OK;
        out.resize(m);
        for (size_t j = 0; j < m; j++) {
            Key32 k;
            std::memcpy(k.b, keys + 32 * j, 32);
            auto it = kc.slot.find(k);
            if (it == kc.slot.end()) {
                out.clear();
                return NWV_OK;
            }
            out[j] = it->second;
        }
        return NWV_OK;
    }
    constexpr uint32_t kCap = 1u << 16;  // 16 MiB of records
    if (!kc.cap) {
        // allocated once at full size: captured graphs and in-flight batches hold its address
        if (kc.recs.ensure((size_t)4 * KC_SLOT_WORDS * kCap)) {
            kc.broken = true;
            return NWV_OK;
        }
        kc.cap = kCap;
        kc.used = 1;  // slot 0: B (filled with the first misses below)
    }
    out.resize(m);
    thread_local std::vector<uint8_t> miss_keys;
    thread_local std::vector<uint32_t> miss_slots;
    miss_keys.clear();
    miss_slots.clear();
    if (!kc.b_ready) {  // first fill: B into slot 0
        uint32_t bw[8];
        ge_basepoint_words(bw);
        miss_keys.insert(miss_keys.end(), (const uint8_t*)bw, (const uint8_t*)bw + 32);
        miss_slots.push_back(0);
    }
    std::vector<Key32> fresh;
    uint32_t next = kc.used;
    for (size_t j = 0; j < m; j++) {
        Key32 k;
        std::memcpy(k.b, keys + 32 * j, 32);
        auto it = kc.slot.find(k);
        if (it != kc.slot.end()) {
            out[j] = it->second;
            continue;
        }
        // a key repeated inside one call gets one slot (keys are distinct per call, but be safe)
        bool dup = false;
        for (size_t f = 0; f < fresh.size() && !dup; f++)
            if (fresh[f] == k) {
                out[j] = miss_slots[miss_slots.size() - fresh.size() + f];
                dup = true;
            }
        if (dup) continue;
        if (next >= kc.cap) {  // full: this call goes uncached, nothing is published
            out.clear();
            return NWV_OK;
        }
        fresh.push_back(k);
        miss_keys.insert(miss_keys.end(), keys + 32 * j, keys + 32 * j + 32);
        miss_slots.push_back(next);
        out[j] = next++;
    }
    if (!miss_slots.empty()) {
        const size_t cnt = miss_slots.size();
        DevBuf tmp;
        auto fail = [&](int rc) {
            tmp.release();
            kc.broken = true;
            out.clear();
            return rc;
        };
        if (tmp.ensure(36 * cnt + 64)) return fail(NWV_OK);
        uint8_t* tk = tmp.as<uint8_t>();
        uint32_t* ts = reinterpret_cast<uint32_t*>(tk + 32 * cnt);
        if (hipMemcpyAsync(tk, miss_keys.data(), 32 * cnt, hipMemcpyHostToDevice, d.stream) != hipSuccess ||
            hipMemcpyAsync(ts, miss_slots.data(), 4 * cnt, hipMemcpyHostToDevice, d.stream) != hipSuccess)
            return fail(set_err(NWV_ERR_HIP, "key cache upload"));
        hipLaunchKernelGGL(k_keycache_fill, dim3((unsigned)((cnt + 63) / 64)), dim3(64), 0, d.stream, (uint32_t)cnt,
                           tk, ts, kc.recs.as<uint32_t>());
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(d.stream) != hipSuccess)
            return fail(set_err(NWV_ERR_HIP, "key cache fill"));
        tmp.release();
        for (size_t f = 0; f < fresh.size(); f++) kc.slot.emplace(fresh[f], miss_slots[miss_slots.size() - fresh.size() + f]);
        kc.b_ready = true;
        kc.used = next;
    }
    return NWV_OK;
}

// Keyed staging: signature i of [lo, hi) is by keys[key_idx[i]].  The distinct keys that occur
// in the range are renumbered densely, uploaded with the CSR of signatures per key, and pk is
// expanded per signature (the per-signature fallback reads it).
int ed_stage_keyed(Lane& d, EdBuffers& b, size_t lo, size_t hi, size_t n_keys, const uint8_t* keys,
                   const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                   const uint64_t* msg_off, const uint32_t* msg_len, const uint8_t* seed32,
                   const DevBuf* dev_msg = nullptr, bool kc_lookup_only = false) {
    const size_t n = hi - lo;
    // per-thread scratch reused across calls (fresh large vectors are page-faulted in every call)
    thread_local std::vector<uint32_t> local, cnt, kid, koff, ksig, cur;
    thread_local std::vector<uint8_t> klist, pk;
    local.assign(n_keys, UINT32_MAX);
    cnt.clear();
    kid.resize(n);
    klist.clear();
    pk.resize(32 * n + 16);
    for (size_t i = 0; i < n; i++) {
        const uint32_t g = key_idx[lo + i];
        if (g >= n_keys) return set_err(NWV_ERR_ARG, "key index out of range");
        if (local[g] == UINT32_MAX) {
            local[g] = (uint32_t)cnt.size();
            cnt.push_back(0);
            klist.insert(klist.end(), keys + 32 * (size_t)g, keys + 32 * (size_t)g + 32);
        }
        kid[i] = local[g];
        cnt[kid[i]]++;
        std::memcpy(pk.data() + 32 * i, keys + 32 * (size_t)g, 32);
    }
    const size_t m = cnt.size();
    koff.assign(m + 1, 0);
    ksig.resize(n);
    for (size_t k = 0; k < m; k++) koff[k + 1] = koff[k] + cnt[k];
    cur.assign(koff.begin(), koff.end() - 1);
    for (size_t i = 0; i < n; i++) ksig[cur[kid[i]]++] = (uint32_t)i;
    thread_local std::vector<uint32_t> kslot;
    int rc = keycache_slots(d, klist.data(), m, kslot, kc_lookup_only);
    if (rc) return rc;
    const KeyedTail kt{klist.data(), m, koff.data(), ksig.data(), kslot.empty() ? nullptr : kslot.data()};
    rc = ed_stage(d, b, 0, n, pk.data(), sig + 64 * lo, msg_base, msg_off + lo, msg_len + lo, seed32, &kt, dev_msg);
    if (rc) return rc;
    // the one-launch path: few signatures, every key registered (comb table present)
    if (n && n <= (size_t)TINY_MAX && !kslot.empty() && !(d.flags & (NWV_FLAG_NO_TINY | NWV_FLAG_MSM_NEVER))) {
        KeyCache& kc = d.gpu->kc;
        std::lock_guard<std::mutex> g(kc.mu);
        bool all = !kc.comb_of.empty();
        for (size_t i = 0; i < n && all; i++) {
            const uint32_t sl = kslot[kid[i]];
            const uint32_t c = sl < kc.comb_of.size() ? kc.comb_of[sl] : UINT32_MAX;
            all = c != UINT32_MAX;
            b.tiny_slot[i] = sl;
            b.tiny_cidx[i] = c;
        }
        b.tiny = all;
    }
    return NWV_OK;
}

bool verdicts_all_valid(const uint64_t* bits, size_t n) {
    for (size_t w = 0; w < n / 64; w++)
        if (bits[w] != ~0ULL) return false;
    if (n % 64) {
        const uint64_t m = (1ULL << (n % 64)) - 1;
        if ((bits[n / 64] & m) != m) return false;
    }
    return true;
}

}  // namespace

struct nwv_ctx {
    std::vector<Gpu*> devs;
    // a call splits over the devices only into ranges of at least this many signatures
    // (shard.h; env NWV_SHARD_MIN, read at nwv_init)
    size_t shard_min = 16384;
    size_t b2_shard_min = 4096;  // the same for BLAKE2b digest calls (messages; NWV_B2_SHARD_MIN)
};

// Per-kernel device time of the staged pipelines (HIP events on the batch's own stream).
struct KernelLog {
    std::vector<const char*> names;  // static strings
    std::vector<double> ms;
    long runs = 0;
    void add(const char* const* nm, const float* t, int k) {  // nm[i] == nullptr: empty slot
        if (names.empty())
            for (int i = 0; i < k; i++)
                if (nm[i]) {
                    names.push_back(nm[i]);
                    ms.push_back(0.0);
                }
        for (int i = 0, j = 0; i < k; i++)
            if (nm[i]) ms[j++] += t[i];
        runs++;
    }
};

struct nwv_staged {
    nwv_ctx* ctx = nullptr;
    Gpu* gpu = nullptr;
    Lane own;                      // the batch's launch context: its own stream, the device's table
    std::mutex mu;                 // one call at a time on a staged batch
    EdBuffers buf;
    size_t n = 0;
    hipStream_t stream = nullptr;  // each resident batch runs on its own stream, so several
    hipEvent_t ev[MSM_NEVENTS] = {};  // staged batches on one device overlap
    KernelLog log[2];              // [0] per-signature pipeline, [1] batch MSM
    int last_mode = -1;
    bool pending_timing = false;
    hipGraphExec_t graph = nullptr;  // captured batch MSM (mode 1, unchained replays)
    bool graph_failed = false;
    bool chain_ready = false;  // first run done: chained replays launch directly
    bool tally_ready = false;  // m_state[2..4) zeroed before the first mode-1 run
    // per-run coefficient seeds go to the device from a ring of pinned slots, so a graph replay is
    // two truly asynchronous calls (a pageable copy may wait for the stream)
    static constexpr int SEED_SLOTS = 64;
    PinnedBuf seeds;
    hipEvent_t seed_ev[SEED_SLOTS] = {};
    uint64_t seed_runs = 0;
    std::vector<hipEvent_t> marks;  // nwv_staged_mark: step-completion timestamps on this stream
};

// Shard [0, n) into contiguous, 64-aligned ranges of at least ctx->shard_min signatures over the
// context's devices (shard.h) and run fn(lane, lo, hi) for each: range 0 on the calling thread, the
// others on one host thread each.  A call below 2 shard_min runs on device 0 alone.
template <class Fn>
static int for_shards(nwv_ctx* ctx, size_t n, Fn fn) {
    const auto ranges = nwv::ed_shard_ranges(n, ctx->devs.size(), ctx->shard_min);
    return nwv::for_ranges(ranges, [&](size_t k, size_t lo, size_t hi) -> int {
        LaneRef lane(*ctx->devs[k]);
        const int rc = lane.rc();
        return rc ? rc : fn(*lane, lo, hi);
    });
}

extern "C" {

int nwv_abi_version(void) { return NWV_ABI_VERSION; }
const char* nwv_last_error(void) { return g_last_error.c_str(); }

static size_t env_size(const char* name, size_t dflt, size_t lo, size_t hi) {
    const char* e = std::getenv(name);
    if (!e || !*e) return dflt;
    const unsigned long long v = std::strtoull(e, nullptr, 10);
    return (size_t)std::min<unsigned long long>(hi, std::max<unsigned long long>(lo, v));
}

// Test hook: env NWV_DEVICE_REPLICAS=r (read at nwv_init, 1..8) opens r independent device
// objects (own lanes, key cache, basepoint tables) per ordinal, so the multi-device split of
// for_shards -- ranges, per-range seeds, verdict words at lo / 64, the rc merge -- runs on a
// one-GPU box exactly as it does over r real devices.
static int init_devices(nwv_ctx** out, std::vector<int> ordinals, uint32_t flags) {
    if (!out) return set_err(NWV_ERR_ARG, "null out");
    *out = nullptr;
    auto* ctx = new (std::nothrow) nwv_ctx;
    if (!ctx) return set_err(NWV_ERR_OOM, "context allocation");
    ctx->shard_min = env_size("NWV_SHARD_MIN", ctx->shard_min, 1, SIZE_MAX);
    ctx->b2_shard_min = env_size("NWV_B2_SHARD_MIN", ctx->b2_shard_min, 1, SIZE_MAX);
    const size_t replicas = env_size("NWV_DEVICE_REPLICAS", 1, 1, 8);
    for (int o : ordinals)
        for (size_t r = 0; r < replicas; r++) {
            auto* d = new Gpu;
            int rc = gpu_open(*d, o, flags);
            if (rc) {
                gpu_close(*d);
                delete d;
                nwv_free(ctx);
                return rc;
            }
            ctx->devs.push_back(d);
        }
    *out = ctx;
    return NWV_OK;
}

int nwv_init(nwv_ctx** out, int n_devices, uint32_t flags) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) return set_err(NWV_ERR_NODEV, "no HIP device visible");
    if (n_devices < 0) return set_err(NWV_ERR_ARG, "n_devices < 0");
    if (n_devices == 0 || n_devices > count) n_devices = count;
    std::vector<int> ords;
    for (int i = 0; i < n_devices; i++) ords.push_back(i);
    return init_devices(out, ords, flags);
}

int nwv_init_device(nwv_ctx** out, int device_ordinal, uint32_t flags) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) return set_err(NWV_ERR_NODEV, "no HIP device visible");
    if (device_ordinal < 0 || device_ordinal >= count) return set_err(NWV_ERR_ARG, "bad ordinal");
    return init_devices(out, {device_ordinal}, flags);
}

void nwv_free(nwv_ctx* ctx) {
    if (!ctx) return;
    nwv_bls_ctx_release(ctx);  // the BLS12-381 engine's per-context state (nwv_bls.hip)
    for (Gpu* d : ctx->devs) {
        gpu_close(*d);
        delete d;
    }
    delete ctx;
}

int nwv_device_count(const nwv_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }
int nwv_diag_counters(const nwv_ctx* ctx, uint64_t out[3]) {
    if (!ctx || !out) return set_err(NWV_ERR_ARG, "null argument");
    out[0] = out[1] = out[2] = 0;
    for (const Gpu* g : ctx->devs) {
        out[0] += g->n_tiny.load();
        out[1] += g->n_msm.load();
        out[2] += g->n_each.load();
    }
    return NWV_OK;
}
int nwv_device_ordinal(const nwv_ctx* ctx, int i) {
    return (ctx && i >= 0 && i < (int)ctx->devs.size()) ? ctx->devs[i]->ordinal : -1;
}

int nwv_ed25519_verify_each(nwv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig,
                            const uint8_t* msg_base, const uint64_t* msg_off,
                            const uint32_t* msg_len, uint64_t* verdict_bits) {
    if (!ctx || (n && (!pk || !sig || !msg_off || !msg_len || !verdict_bits)))
        return set_err(NWV_ERR_ARG, "null argument");
    if (n == 0) return NWV_OK;
    for (size_t i = 0; i < n; i++)
        if (msg_len[i] && !msg_base) return set_err(NWV_ERR_ARG, "null msg_base");
    return for_shards(ctx, n, [&](Lane& d, size_t lo, size_t hi) -> int {
        int rc = ed_stage(d, d.ed, lo, hi, pk, sig, msg_base, msg_off, msg_len, nullptr);
        if (rc) return rc;
        if ((rc = ed_launch(d, d.ed, hi - lo, d.stream, nullptr))) return rc;
        const size_t words = (hi - lo + 63) / 64;
        NWV_HIP(hipMemcpyAsync(verdict_bits + lo / 64, d.ed.verdict.p, 8 * words,
                               hipMemcpyDeviceToHost, d.stream));
        NWV_HIP(hipStreamSynchronize(d.stream));
        return NWV_OK;
    });
}

// Batches of at least this many signatures go through the MSM (K5); smaller ones through the
// per-signature pipeline (tools/latency_sweep.py measures the crossover: the MSM's quad-lane
// window Horner is shorter than the per-signature Straus chain already at small n).
#ifndef NWV_MSM_MIN_N_DEFAULT
#define NWV_MSM_MIN_N_DEFAULT 1
#endif
static size_t msm_min_n() {
    static const size_t v = [] {
        const char* e = std::getenv("NWV_MSM_MIN_N");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)NWV_MSM_MIN_N_DEFAULT;
    }();
    return v;
}

// OS entropy for the batch coefficients, as the reference's OsRng / thread_rng: a per-thread
// ChaCha20 generator keyed by getrandom(2) (rekeyed every 2^20 seeds) -- a getrandom call per
// batch cost ~20 us of host time per launch here, std::random_device more
static void os_entropy(uint8_t* out, size_t len) {
    size_t got = 0;
    while (got < len) {
        const ssize_t r = getrandom(out + got, len - got, 0);
        if (r > 0) {
            got += (size_t)r;
        } else if (r < 0 && errno != EINTR) {
            std::random_device rd;  // fallback only if the syscall is unavailable
            for (size_t i = got; i < len; i++) out[i] = (uint8_t)rd();
            got = len;
        }
    }
}

static void fill_seed(const uint8_t* seed32, uint8_t out[32]) {
    if (seed32) {
        std::memcpy(out, seed32, 32);
        return;
    }
    thread_local uint32_t key[8];
    thread_local uint64_t ctr = 0;
    if ((ctr & ((1u << 20) - 1)) == 0) os_entropy(reinterpret_cast<uint8_t*>(key), sizeof(key));
    const uint32_t nonce[3] = {(uint32_t)(ctr >> 32), 0x2d76776eu /* "nwv-" */, 0x64656573u /* "seed" */};
    uint32_t blk[16];
    nwv::chacha20_block(key, (uint32_t)ctr, nonce, blk);
    ctr++;
    std::memcpy(out, blk, 32);
}
// shared with nwv_bls.hip (hidden): the context's nwv_init flags, and a batch-coefficient seed
__attribute__((visibility("hidden"))) uint32_t nwv_internal_ctx_flags(const nwv_ctx* ctx) {
    return (ctx && !ctx->devs.empty()) ? ctx->devs[0]->flags : 0u;
}
__attribute__((visibility("hidden"))) void nwv_internal_fill_seed(const uint8_t* seed32, uint8_t out[32]) {
    fill_seed(seed32, out);
}

// point records of the batch MSM that ran last on b, when the per-signature fallback can reuse
// them: per-signature keys (every A_i decompressed at point i, R_i at n + 1 + i)
static const uint32_t* msm_reusable(const Lane& d, const EdBuffers& b, bool msm_ran) {
    if (!msm_ran || b.nkeys_distinct || (d.flags & NWV_FLAG_NO_MSM_REUSE)) return nullptr;
    return b.m_pts.as<uint32_t>();
}

static void set_ones(uint64_t* bits, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) bits[i >> 6] |= 1ULL << (i & 63);
}

// k_ed_tiny over a staged tiny keyed batch (b.tiny): every signature's verdict in one launch,
// read back through the lane's polled host word (or the workspace when the lane has none)
static int tiny_on_device(Lane& d, EdBuffers& b, size_t n, hipStream_t stream, int* ok, uint64_t* bits) {
    int rc;
    if (!d.tiny_ws.p) {
        if ((rc = d.tiny_ws.ensure(64))) return rc;
        NWV_HIP(hipMemsetAsync(d.tiny_ws.p, 0, 64, stream));
    }
    static const bool no_poll = std::getenv("NWV_NO_HOST_POLL") != nullptr;
    uint32_t* hv = (!no_poll && stream == d.stream) ? d.hword : nullptr;
    TinyArgs a{};
    a.pk = b.pk.as<uint8_t>();
    a.sig = b.sig.as<uint8_t>();
    a.msg = b.msg.as<uint8_t>();
    a.off = b.off.as<uint64_t>();
    a.len = b.len.as<uint32_t>();
    a.kc = d.gpu->kc.recs.as<uint32_t>();
    a.combs = d.gpu->kc.combs.as<uint32_t>();
    a.bcomb = d.gpu->comb.as<uint32_t>();
    a.ws = d.tiny_ws.as<uint32_t>();
    a.hword = hv;
    a.n = (uint32_t)n;
    if (hv) {
        d.hseq = (d.hseq + 1) & 0x3FFFFFFFu;
        if (d.hseq == 0) d.hseq = 1;
        a.hseq = d.hseq;
        __atomic_store_n(hv, 0u, __ATOMIC_RELEASE);
    }
    std::memcpy(a.kslot, b.tiny_slot, 4 * n);
    std::memcpy(a.cidx, b.tiny_cidx, 4 * n);
    static const bool stamps = std::getenv("NWV_TINY_STAMPS") != nullptr;  // diagnostics only
    if (stamps) {
        if ((rc = b.m_stamps.ensure(8 * 8))) return rc;
        NWV_HIP(hipMemsetAsync(b.m_stamps.p, 0, 64, stream));
        a.stamps = b.m_stamps.as<unsigned long long>();
    }
    hipLaunchKernelGGL(k_ed_tiny, dim3((unsigned)n), dim3(64 * TINY_WAVES), 0, stream, a);
    if (hipGetLastError() != hipSuccess) {
        (void)hipStreamSynchronize(stream);
        return set_err(NWV_ERR_HIP, "k_ed_tiny launch");
    }
    uint64_t vb = 0;
    uint32_t all = 0;
    bool got = false;
    if (hv) {
        uint32_t v = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t k = 0; ((v = __atomic_load_n(hv, __ATOMIC_ACQUIRE)) >> 2) != a.hseq; k++) {
            if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
            __builtin_ia32_pause();
        }
        NWV_HIP(hipStreamSynchronize(stream));
        if ((v >> 2) == a.hseq) {
            vb = (uint64_t)hv[2] | ((uint64_t)hv[3] << 32);
            all = (v & 3u) == 1u;
            got = true;
        }
    }
    if (!got) {
        uint32_t r[4] = {0, 0, 0, 0};
        NWV_HIP(hipMemcpyAsync(r, a.ws + 4, 16, hipMemcpyDeviceToHost, stream));
        NWV_HIP(hipStreamSynchronize(stream));
        vb = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
        all = r[2];
    }
    htrace("batch:tiny-done");
    if (stamps) {  // phase times of workgroup 0 in us from its start (s_memrealtime: 100 MHz)
        unsigned long long t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpy(t, b.m_stamps.p, 64, hipMemcpyDeviceToHost) == hipSuccess)
            std::fprintf(stderr, "tiny n=%zu: R %.1f 8R %.1f hash %.1f 8P %.1f barrier %.1f final %.1f us\n", n,
                         (t[1] - t[0]) / 100.0, (t[3] - t[0]) / 100.0, (t[2] - t[0]) / 100.0, (t[4] - t[0]) / 100.0,
                         (t[5] - t[0]) / 100.0, (t[6] - t[0]) / 100.0);
    }
    *ok = all ? 1 : 0;
    if (bits) bits[0] = vb;
    return NWV_OK;
}

// Batch verdict of resident buffers: MSM, then (only if it rejects) the per-signature fallback
// for the exact bad set.  bits: the shard's verdict words (may be null).  A tiny keyed batch by
// registered keys takes the one-launch per-signature path instead (exact bits, no fallback).
static int batch_on_device(Lane& d, EdBuffers& b, size_t n, const uint8_t seed[32], hipStream_t stream,
                           int* ok, uint64_t* bits, bool state_ready = false) {
    int rc;
    if (b.tiny && n <= (size_t)TINY_MAX) {
        d.gpu->n_tiny++;
        return tiny_on_device(d, b, n, stream, ok, bits);
    }
    const bool use_msm = (d.flags & NWV_FLAG_MSM_ALWAYS) ||
                         (!(d.flags & NWV_FLAG_MSM_NEVER) && n >= msm_min_n());
    if (use_msm) {
        d.gpu->n_msm++;
        htrace("batch:msm-launch");
        // batch-verdict calls of up to 65,536 signatures (latency-bound: a spinning host thread
        // costs little) poll the tail's word in pinned host memory instead of copying the verdict
        // back and waiting for the stream: 1K p50 0.233 -> 0.227 ms (NWV_NO_HOST_POLL: the copy)
        static const bool no_poll = std::getenv("NWV_NO_HOST_POLL") != nullptr;
        uint32_t* hv = (!bits && !no_poll && stream == d.stream && n <= 65536) ? d.hword : nullptr;
        uint32_t seq = 0;
        if (hv) {
            d.hseq = (d.hseq + 1) & 0x3FFFFFFFu;
            if (d.hseq == 0) d.hseq = 1;
            seq = d.hseq;
            __atomic_store_n(hv, 0u, __ATOMIC_RELEASE);
        }
        if ((rc = msm_launch(d, b, n, seed, stream, nullptr, state_ready, bits != nullptr, hv, seq))) {
            // a launch that failed part-way may have queued work that still stores into the word:
            // drain the stream so the lane's next call starts clean
            (void)hipStreamSynchronize(stream);
            return rc;
        }
        htrace("batch:msm-launched");
        if (hv) {
            // spin on the word until it carries this call's sequence number (a few hundred us at
            // most for the batches that come this way), then the stream's own completion; a word
            // that never flips (bounded at ~2 s) falls back to the copy below
            uint32_t v = 0;
            const auto t0 = std::chrono::steady_clock::now();
            for (uint64_t k = 0; ((v = __atomic_load_n(hv, __ATOMIC_ACQUIRE)) >> 2) != seq; k++) {
                if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
                __builtin_ia32_pause();
            }
            // the stream's own completion too (by now the tail has stored its last word: this
            // returns at once; without it p99 rose by ~10 us while p50 gained ~2 us)
            NWV_HIP(hipStreamSynchronize(stream));
            const uint32_t code = (v >> 2) == seq ? (v & 3u) : 0u;
            if (code == 1u || code == 2u) {
                htrace("batch:verdict-polled");
                *ok = code == 1u ? 1 : 0;
                return NWV_OK;
            }
            // code 3 (the tail could not determine the verdict) or no word: the state copy below
        }
        if (bits && b.tables_ready) {
            // the early form built the fallback's tables: its Straus pass queues behind the MSM now
            // (gated on the MSM's verdict word) and one read-back brings both
            if ((rc = ed_launch(d, b, n, stream, nullptr, nullptr, true, b.m_state.as<uint32_t>()))) return rc;
            uint32_t st[2] = {0, 0};
            NWV_HIP(hipMemcpyAsync(st, b.m_state.p, 8, hipMemcpyDeviceToHost, stream));
            NWV_HIP(hipMemcpyAsync(bits, b.verdict.p, 8 * ((n + 63) / 64), hipMemcpyDeviceToHost, stream));
            NWV_HIP(hipStreamSynchronize(stream));
            htrace("batch:gated-done");
            if (st[1] == 1) {
                std::memset(bits, 0, 8 * ((n + 63) / 64));
                set_ones(bits, 0, n);
                *ok = 1;
            } else {
                *ok = verdicts_all_valid(bits, n) ? 1 : 0;
            }
            return NWV_OK;
        }
        uint32_t st[2] = {0, 0};
        NWV_HIP(hipMemcpyAsync(st, b.m_state.p, 8, hipMemcpyDeviceToHost, stream));
        NWV_HIP(hipStreamSynchronize(stream));
        if (st[1] == 1) {
            *ok = 1;
            if (bits) {
                std::memset(bits, 0, 8 * ((n + 63) / 64));
                set_ones(bits, 0, n);
            }
            return NWV_OK;
        }
        // a batch of valid signatures always passes (the cofactored equation holds for each term
        // whatever z_i), so a rejection means some signature is invalid: callers that only want
        // the batch verdict (fastcrypto's verify_batch / aggregate verify) get it without the
        // per-signature pass, which only runs to name the bad signatures.  An undetermined MSM
        // (st[1] == 2: the tail gave up waiting for a window) is never reported as a rejection:
        // the per-signature pass decides.
        if (!bits && st[1] == 0) {
            *ok = 0;
            return NWV_OK;
        }
    }
    htrace("batch:fallback");
    d.gpu->n_each++;
    if ((rc = ed_launch(d, b, n, stream, nullptr, msm_reusable(d, b, use_msm)))) return rc;
    std::vector<uint64_t> tmp;
    uint64_t* out = bits;
    if (!out) {
        tmp.assign((n + 63) / 64, 0);
        out = tmp.data();
    }
    NWV_HIP(hipMemcpyAsync(out, b.verdict.p, 8 * ((n + 63) / 64), hipMemcpyDeviceToHost, stream));
    NWV_HIP(hipStreamSynchronize(stream));
    htrace("batch:fallback-done");
    *ok = verdicts_all_valid(out, n) ? 1 : 0;
    return NWV_OK;
}

int nwv_ed25519_verify_batch(nwv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig,
                             const uint8_t* msg_base, const uint64_t* msg_off,
                             const uint32_t* msg_len, const uint8_t seed32[32], int* all_valid,
                             uint64_t* verdict_bits_or_null) {
    if (!ctx || !all_valid || (n && (!pk || !sig || !msg_off || !msg_len)))
        return set_err(NWV_ERR_ARG, "null argument");
    *all_valid = 1;
    if (n == 0) return NWV_OK;
    for (size_t i = 0; i < n; i++)
        if (msg_len[i] && !msg_base) return set_err(NWV_ERR_ARG, "null msg_base");
    uint8_t seed[32];
    fill_seed(seed32, seed);
    std::mutex omu;
    int rc = for_shards(ctx, n, [&](Lane& d, size_t lo, size_t hi) -> int {
        // each shard gets its own coefficient stream: seed' = seed with the shard start mixed in
        uint8_t s2[32];
        std::memcpy(s2, seed, 32);
        for (int k = 0; k < 8; k++) s2[24 + k] ^= (uint8_t)((uint64_t)lo >> (8 * k));
        int r = ed_stage(d, d.ed, lo, hi, pk, sig, msg_base, msg_off, msg_len, s2);
        if (r) return r;
        int ok = 1;
        r = batch_on_device(d, d.ed, hi - lo, s2, d.stream, &ok,
                            verdict_bits_or_null ? verdict_bits_or_null + lo / 64 : nullptr, true);
        if (r) return r;
        std::lock_guard<std::mutex> g(omu);
        if (!ok) *all_valid = 0;
        return NWV_OK;
    });
    return rc;
}

static int verify_batch_keyed_impl(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys, size_t n,
                                   const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                                   const uint64_t* msg_off, const uint32_t* msg_len,
                                   const uint8_t seed32[32], int* all_valid, uint64_t* verdict_bits_or_null,
                                   bool kc_lookup_only) {
    if (!ctx || !all_valid || (n && (!keys || !key_idx || !sig || !msg_off || !msg_len)))
        return set_err(NWV_ERR_ARG, "null argument");
    *all_valid = 1;
    if (n == 0) return NWV_OK;
    for (size_t i = 0; i < n; i++)
        if (msg_len[i] && !msg_base) return set_err(NWV_ERR_ARG, "null msg_base");
    uint8_t seed[32];
    fill_seed(seed32, seed);
    std::mutex omu;
    return for_shards(ctx, n, [&](Lane& d, size_t lo, size_t hi) -> int {
        uint8_t s2[32];
        std::memcpy(s2, seed, 32);
        for (int k = 0; k < 8; k++) s2[24 + k] ^= (uint8_t)((uint64_t)lo >> (8 * k));
        int r = ed_stage_keyed(d, d.ed, lo, hi, n_keys, keys, key_idx, sig, msg_base, msg_off, msg_len, s2,
                               nullptr, kc_lookup_only);
        if (r) return r;
        int ok = 1;
        r = batch_on_device(d, d.ed, hi - lo, s2, d.stream, &ok,
                            verdict_bits_or_null ? verdict_bits_or_null + lo / 64 : nullptr, true);
        if (r) return r;
        std::lock_guard<std::mutex> g(omu);
        if (!ok) *all_valid = 0;
        return NWV_OK;
    });
}

int nwv_ed25519_verify_batch_keyed(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys, size_t n,
                                   const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                                   const uint64_t* msg_off, const uint32_t* msg_len,
                                   const uint8_t seed32[32], int* all_valid, uint64_t* verdict_bits_or_null) {
    return verify_batch_keyed_impl(ctx, n_keys, keys, n, key_idx, sig, msg_base, msg_off, msg_len, seed32, all_valid,
                                   verdict_bits_or_null, false);
}

// Committee registration (epoch start, Core::change_epoch primary/src/core.rs:592-611): fill the
// key cache of every device with the committee's keys, so single verifies by them
// (nwv_ed25519_pubkey_verify, which only looks keys up) take the 128-bit-scalar form.
int nwv_keycache_register(nwv_ctx* ctx, size_t n_keys, const uint8_t* keys) {
    if (!ctx || (n_keys && !keys)) return set_err(NWV_ERR_ARG, "null argument");
    // the same key list as the last registration (the types layer registers its committee on
    // every call): nothing to do
    uint64_t fp = 0x9E3779B97F4A7C15ull ^ (uint64_t)n_keys;
    for (size_t i = 0; i < 4 * n_keys; i++) {
        uint64_t w;
        std::memcpy(&w, keys + 8 * i, 8);
        fp = (fp ^ w) * 0xFF51AFD7ED558CCDull;
        fp ^= fp >> 29;
    }
    if (fp == 0) fp = 1;
    static const uint32_t comb_keys = (uint32_t)env_size("NWV_COMB_KEYS", 1024, 0, 1u << 16);
    for (Gpu* g : ctx->devs) {
        {
            std::lock_guard<std::mutex> lk(g->kc.mu);
            if (g->kc.reg_fp == fp) continue;
        }
        LaneRef lane(*g);
        int rc = lane.rc();
        std::vector<uint32_t> slots, all;
        for (size_t a = 0; a < n_keys && !rc; a += 4096) {
            rc = keycache_slots(*lane, keys + 32 * a, std::min<size_t>(4096, n_keys - a), slots);
            all.insert(all.end(), slots.begin(), slots.end());
        }
        if (rc) return rc;
        if (all.size() != n_keys || comb_keys == 0 || (g->flags & NWV_FLAG_NO_KEYCACHE)) continue;  // uncached
        // fixed-base comb tables for the keys that have none yet (the one-launch path, k_ed_tiny)
        KeyCache& kc = g->kc;
        std::lock_guard<std::mutex> lk(kc.mu);
        if (!kc.comb_cap) {
            if (kc.combs.ensure((size_t)4 * COMB_WORDS * comb_keys)) continue;  // no room: batches use the MSM
            kc.comb_cap = comb_keys;
            kc.comb_of.assign(kc.cap ? kc.cap : (1u << 16), UINT32_MAX);
        }
        std::vector<uint8_t> nk;
        std::vector<uint32_t> ni, nslot;
        for (size_t j = 0; j < n_keys; j++) {
            const uint32_t sl = all[j];
            if (sl >= kc.comb_of.size() || kc.comb_of[sl] != UINT32_MAX) continue;
            bool dup = false;
            for (uint32_t q : nslot) dup = dup || q == sl;
            if (dup) continue;
            if (kc.comb_used + ni.size() >= kc.comb_cap) break;  // full: later keys take the MSM path
            nk.insert(nk.end(), keys + 32 * j, keys + 32 * j + 32);
            ni.push_back(kc.comb_used + (uint32_t)ni.size());
            nslot.push_back(sl);
        }
        if (!ni.empty()) {
            Lane& d = *lane;
            DevBuf tmp;
            if ((rc = tmp.ensure(36 * ni.size() + 64))) return rc;
            uint8_t* tk = tmp.as<uint8_t>();
            uint32_t* ti = reinterpret_cast<uint32_t*>(tk + 32 * ni.size());
            NWV_HIP(hipMemcpyAsync(tk, nk.data(), nk.size(), hipMemcpyHostToDevice, d.stream));
            NWV_HIP(hipMemcpyAsync(ti, ni.data(), 4 * ni.size(), hipMemcpyHostToDevice, d.stream));
            const size_t lanes = ni.size() * COMB_TABLES * COMB_ENTRIES;
            hipLaunchKernelGGL(k_key_comb_fill, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, d.stream,
                               (uint32_t)ni.size(), tk, ti, kc.combs.as<uint32_t>());
            NWV_HIP(hipGetLastError());
            NWV_HIP(hipStreamSynchronize(d.stream));  // published only once the tables are written
            for (size_t q = 0; q < ni.size(); q++) kc.comb_of[nslot[q]] = ni[q];
            kc.comb_used += (uint32_t)ni.size();
        }
        bool every = true;
        for (size_t j = 0; j < n_keys && every; j++) every = all[j] < kc.comb_of.size() && kc.comb_of[all[j]] != UINT32_MAX;
        if (every) kc.reg_fp = fp;
    }
    return NWV_OK;
}

// ---- fastcrypto trait surface ---------------------------------------------------------
// Verifier::verify: a one-signature keyed batch.  With z != 0 its MSM verdict is exactly the
// signature's ZIP-215 verdict, the key goes through the committee key cache (128-bit scalars:
// Narwhal verifies committee members' keys), and no per-signature pass is needed either way.
// Contexts opened with NWV_FLAG_MSM_NEVER use the per-signature pipeline.
int nwv_ed25519_pubkey_verify(nwv_ctx* ctx, const uint8_t pk[32], const uint8_t* msg,
                              size_t msg_len, const uint8_t sig[64]) {
    if (!ctx || !pk || !sig || (msg_len && !msg)) return set_err(NWV_ERR_ARG, "null argument");
    if (msg_len > UINT32_MAX) return set_err(NWV_ERR_ARG, "message too long");
    const uint64_t off = 0;
    const uint32_t len = (uint32_t)msg_len;
    static const uint8_t empty[1] = {0};
    if (ctx->devs.empty() || (ctx->devs[0]->flags & NWV_FLAG_MSM_NEVER)) {
        uint64_t bits = 0;
        int rc = nwv_ed25519_verify_each(ctx, 1, pk, sig, msg_len ? msg : empty, &off, &len, &bits);
        if (rc) return rc;
        return (bits & 1) ? NWV_OK : NWV_ERR_SIGNATURE;
    }
    const uint32_t kidx = 0;
    int all = 0;
    int rc = verify_batch_keyed_impl(ctx, 1, pk, 1, &kidx, sig, msg_len ? msg : empty, &off, &len, nullptr, &all,
                                     nullptr, true);
    if (rc) return rc;
    return all ? NWV_OK : NWV_ERR_SIGNATURE;
}

static int shared_msg_batch(nwv_ctx* ctx, size_t n, const uint8_t* pks, const uint8_t* sigs,
                            const uint8_t* msg, size_t msg_len, const uint8_t* seed32) {
    if (msg_len > UINT32_MAX) return set_err(NWV_ERR_ARG, "message too long");
    std::vector<uint64_t> off(n, 0);
    std::vector<uint32_t> len(n, (uint32_t)msg_len);
    static const uint8_t empty[1] = {0};
    int all = 0;
    int rc = nwv_ed25519_verify_batch(ctx, n, pks, sigs, msg_len ? msg : empty, off.data(),
                                      len.data(), seed32, &all, nullptr);
    if (rc) return rc;
    return all ? NWV_OK : NWV_ERR_SIGNATURE;
}

int nwv_ed25519_verify_batch_empty_fail(nwv_ctx* ctx, const uint8_t* msg, size_t msg_len,
                                        const uint8_t* pks, size_t n_pks, const uint8_t* sigs,
                                        size_t n_sigs, const uint8_t seed32[32]) {
    if (n_sigs == 0)
        return set_err(NWV_ERR_EMPTY,
                       "Critical Error! This behavious can signal something dangerous, and that "
                       "someone may be trying to bypass signature verification through providing "
                       "empty batches.");
    if (n_sigs != n_pks)
        return set_err(NWV_ERR_LENGTH, "Mismatch between number of signatures and public keys provided");
    if (!pks || !sigs || (msg_len && !msg)) return set_err(NWV_ERR_ARG, "null argument");
    return shared_msg_batch(ctx, n_sigs, pks, sigs, msg, msg_len, seed32);
}

int nwv_ed25519_aggregate_verify(nwv_ctx* ctx, const uint8_t* sigs, size_t n_sigs,
                                 const uint8_t* pks, size_t n_pks, const uint8_t* msg,
                                 size_t msg_len, const uint8_t seed32[32]) {
    if (n_pks != n_sigs) return set_err(NWV_ERR_LENGTH, "pks/sigs length mismatch");
    if (n_sigs == 0) return NWV_OK;  // an empty ed25519_consensus batch verifies
    if (!pks || !sigs || (msg_len && !msg)) return set_err(NWV_ERR_ARG, "null argument");
    return shared_msg_batch(ctx, n_sigs, pks, sigs, msg, msg_len, seed32);
}

int nwv_ed25519_aggregate_batch_verify(nwv_ctx* ctx, size_t n_aggs, const uint8_t* const* sigs,
                                       const size_t* n_sigs, const uint8_t* const* pks,
                                       const size_t* n_pks, const uint8_t* const* msgs,
                                       const size_t* msg_lens, size_t n_msgs,
                                       const uint8_t seed32[32]) {
    if (n_msgs != n_aggs) return set_err(NWV_ERR_LENGTH, "messages/aggregates length mismatch");
    size_t total = 0, mtotal = 0;
    for (size_t a = 0; a < n_aggs; a++) {
        if (n_pks[a] != n_sigs[a]) return set_err(NWV_ERR_LENGTH, "pks/sigs length mismatch");
        total += n_sigs[a];
        mtotal += msg_lens[a];
    }
    if (total == 0) return NWV_OK;
    std::vector<uint8_t> P(32 * total), S(64 * total), M(mtotal + 1);
    std::vector<uint64_t> off(total);
    std::vector<uint32_t> len(total);
    size_t k = 0, mo = 0;
    for (size_t a = 0; a < n_aggs; a++) {
        if (msg_lens[a]) std::memcpy(M.data() + mo, msgs[a], msg_lens[a]);
        for (size_t j = 0; j < n_sigs[a]; j++, k++) {
            std::memcpy(P.data() + 32 * k, pks[a] + 32 * j, 32);
            std::memcpy(S.data() + 64 * k, sigs[a] + 64 * j, 64);
            off[k] = mo;
            len[k] = (uint32_t)msg_lens[a];
        }
        mo += msg_lens[a];
    }
    int all = 0;
    int rc = nwv_ed25519_verify_batch(ctx, total, P.data(), S.data(), M.data(), off.data(),
                                      len.data(), seed32, &all, nullptr);
    if (rc) return rc;
    return all ? NWV_OK : NWV_ERR_SIGNATURE;
}

// ---- staged (device-resident) batches ---------------------------------------------------
}  // extern "C"

template <class StageFn>
static int staged_create(nwv_ctx* ctx, int device_index, size_t n, nwv_staged** out, StageFn stage) {
    if (!ctx || !out || device_index < 0 || device_index >= (int)ctx->devs.size())
        return set_err(NWV_ERR_ARG, "bad context/device");
    *out = nullptr;
    auto* st = new (std::nothrow) nwv_staged;
    if (!st) return set_err(NWV_ERR_OOM, "staged allocation");
    st->ctx = ctx;
    st->gpu = ctx->devs[device_index];
    st->n = n;
    int rc;
    {
        // the inputs cross PCIe through a lane's pinned staging buffer, then stay resident
        LaneRef lane(*st->gpu);
        rc = lane.rc();
        if (!rc) rc = stage(*lane, st->buf);
        if (!rc && hipStreamSynchronize((*lane).stream) != hipSuccess) rc = set_err(NWV_ERR_HIP, "stage sync");
    }
    Lane& o = st->own;
    o.gpu = st->gpu;
    o.ordinal = st->gpu->ordinal;
    o.flags = st->gpu->flags;
    o.btabp = &st->gpu->btab;
    if (!rc && hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess)
        rc = set_err(NWV_ERR_HIP, "hipStreamCreate");
    o.stream = st->stream;
    for (auto& e : st->ev)
        if (!rc && hipEventCreate(&e) != hipSuccess) rc = set_err(NWV_ERR_HIP, "hipEventCreate");
    if (rc) {
        o.stream = nullptr;  // owned by st (destroyed below), not by the lane view
        for (auto& e : st->ev)
            if (e) (void)hipEventDestroy(e);
        if (st->stream) (void)hipStreamDestroy(st->stream);
        st->buf.release();
        delete st;
        return rc;
    }
    *out = st;
    return NWV_OK;
}

extern "C" {

int nwv_stage_ed25519(nwv_ctx* ctx, int device_index, size_t n, const uint8_t* pk,
                      const uint8_t* sig, const uint8_t* msg_base, const uint64_t* msg_off,
                      const uint32_t* msg_len, nwv_staged** out) {
    return staged_create(ctx, device_index, n, out, [&](Lane& d, EdBuffers& b) {
        return ed_stage(d, b, 0, n, pk, sig, msg_base, msg_off, msg_len, nullptr);
    });
}

int nwv_stage_ed25519_keyed(nwv_ctx* ctx, int device_index, size_t n_keys, const uint8_t* keys, size_t n,
                            const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                            const uint64_t* msg_off, const uint32_t* msg_len, nwv_staged** out) {
    if (n && (!keys || !key_idx || !sig || !msg_off || !msg_len)) return set_err(NWV_ERR_ARG, "null argument");
    return staged_create(ctx, device_index, n, out, [&](Lane& d, EdBuffers& b) {
        return ed_stage_keyed(d, b, 0, n, n_keys, keys, key_idx, sig, msg_base, msg_off, msg_len, nullptr);
    });
}

static int staged_collect_times(nwv_staged* st) {
    if (!st->pending_timing) return NWV_OK;
    float t[MSM_NKERNELS];
    if (st->last_mode == 1) {
        NWV_HIP(hipEventSynchronize(st->ev[MSM_NKERNELS]));
        for (int i = 0; i < MSM_NKERNELS; i++) NWV_HIP(hipEventElapsedTime(&t[i], st->ev[i], st->ev[i + 1]));
        st->log[1].add((st->own.flags & NWV_FLAG_MSM_SPLIT_PREP) ? MSM_KERNEL_NAMES_SPLIT : MSM_KERNEL_NAMES, t,
                       MSM_NKERNELS);
        if (std::getenv("NWV_TAIL_STAMPS") && st->buf.m_stamps.p) {  // diagnostics: phase times, us
            std::vector<unsigned long long> h(8 * MSM_MAX_WINDOWS);
            NWV_HIP(hipMemcpy(h.data(), st->buf.m_stamps.p, 8 * h.size(), hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int w = 0; w < MSM_MAX_WINDOWS; w++)
                if (h[8 * w]) t0 = std::min(t0, h[8 * w]);
            std::fprintf(stderr, "nwv-tail-stamps n=%zu", st->n);
            for (int w = 0; w < MSM_MAX_WINDOWS; w++) {
                if (!h[8 * w]) continue;
                std::fprintf(stderr, " | w%d", w);
                for (int k = 0; k < 8; k++)
                    std::fprintf(stderr, " %.1f", h[8 * w + k] ? (double)(h[8 * w + k] - t0) / 100.0 : -1.0);
            }
            std::fprintf(stderr, "\n");
        }
    } else {
        NWV_HIP(hipEventSynchronize(st->ev[3]));
        for (int i = 0; i < 3; i++) NWV_HIP(hipEventElapsedTime(&t[i], st->ev[i], st->ev[i + 1]));
        st->log[0].add(ED_KERNEL_NAMES, t, 3);
    }
    st->pending_timing = false;
    return NWV_OK;
}

// Capture the batch MSM of a staged batch once into a HIP graph (buffers and plan are fixed for
// the batch; the per-run seed lives in device memory), so a run is one seed copy + one graph
// launch instead of ~13 kernel launches.
static int staged_graph(nwv_staged* st) {
    if (st->graph || st->graph_failed) return NWV_OK;
    hipGraph_t g = nullptr;
    NWV_HIP(hipStreamBeginCapture(st->stream, hipStreamCaptureModeThreadLocal));
    const int rc = msm_launch(st->own, st->buf, st->n, nullptr, st->stream, nullptr, false);
    const hipError_t e = hipStreamEndCapture(st->stream, &g);
    if (rc || e != hipSuccess || !g || hipGraphInstantiate(&st->graph, g, nullptr, nullptr, 0) != hipSuccess) {
        st->graph = nullptr;
        st->graph_failed = true;  // replay through direct launches
        (void)hipGetLastError();
    }
    if (g) (void)hipGraphDestroy(g);
    return NWV_OK;
}

// Staged runs chain their preps (NWV_STAGE_CHAIN = k, default 3, 0 = off): run r's k_msm_prep
// starts only once run r - k's has finished on the device.  Batches issued back to back then
// start staggered, each prep sharing the chip with at most k - 1 others and with the sorts,
// buckets and tails of the batches ahead, instead of 12 preps running side by side and every
// batch's latency-bound tail landing at once.  The driver's 20-step headline: 194 -> 201 M
// sigs/s (k = 3; k = 2: 203 M, steady state -4 %; k = 1: 172 M); the steady state moves by
// -1.5 % at k = 3 (profiles/round5_stage_chain_experiment.json).
int stage_chain_depth() {  // read per run: tests switch it between runs
    const char* e = std::getenv("NWV_STAGE_CHAIN");
    return e ? std::max(0, std::min(64, std::atoi(e))) : 3;
}

// a replay's coefficient seed: into the next pinned slot, then one asynchronous copy
static int staged_seed_copy(nwv_staged* st, const uint8_t seed[32]) {
    const int slot = (int)(st->seed_runs++ % nwv_staged::SEED_SLOTS);
    int rc = st->seeds.ensure(32 * nwv_staged::SEED_SLOTS);
    if (rc) return rc;
    if (!st->seed_ev[slot]) NWV_HIP(hipEventCreateWithFlags(&st->seed_ev[slot], hipEventDisableTiming));
    else NWV_HIP(hipEventSynchronize(st->seed_ev[slot]));  // the slot's copy of 64 runs ago
    uint8_t* hs = static_cast<uint8_t*>(st->seeds.p) + 32 * slot;
    std::memcpy(hs, seed, 32);
    NWV_HIP(hipMemcpyAsync(st->buf.m_state.as<uint32_t>() + 8, hs, 32, hipMemcpyHostToDevice, st->stream));
    NWV_HIP(hipEventRecord(st->seed_ev[slot], st->stream));
    return NWV_OK;
}

int nwv_staged_run(nwv_staged* st, int mode, const uint8_t seed32[32]) {
    const bool timed = (mode & NWV_RUN_TIMED) != 0;
    mode &= ~NWV_RUN_TIMED;
    if (!st || (mode != 0 && mode != 1)) return set_err(NWV_ERR_ARG, "bad staged/mode");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = with_device(st->own);
    if (rc) return rc;
    if ((rc = staged_collect_times(st))) return rc;
    if (mode == 1) {
        uint8_t seed[32];
        fill_seed(seed32, seed);
        if (!st->tally_ready && st->n) {
            // the run tally (m_state[2..4)) starts at zero and no run ever resets it
            const size_t na = msm_na(st->buf, st->n);
            if ((rc = msm_alloc(st->buf, msm_plan(st->n, na, st->buf.kc_split, (st->own.flags & NWV_FLAG_MSM_SORT2) ? 1 : 0),
                                st->n)))
                return rc;
            NWV_HIP(hipMemsetAsync(st->buf.m_state.as<uint32_t>() + 2, 0, 8, st->stream));
            st->tally_ready = true;
        }
        const int chain_k = stage_chain_depth();
        const bool replay = !timed && st->n && (chain_k > 0 ? st->chain_ready : st->graph != nullptr);
        if (replay && (rc = staged_seed_copy(st, seed))) return rc;
        if (replay && chain_k > 0) {
            // run r's k_msm_prep waits for run r - k's on this device (direct launches: the
            // event pair changes from run to run)
            Gpu& G = *st->gpu;
            std::lock_guard<std::mutex> lk(G.chain_mu);
            if (G.chain_ev.size() != (size_t)chain_k) {
                for (hipEvent_t e : G.chain_ev) (void)hipEventDestroy(e);  // (released once their records complete)
                G.chain_ev.assign(chain_k, nullptr);
                for (auto& e : G.chain_ev) NWV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                G.chain_runs = 0;
            }
            hipEvent_t ce = G.chain_ev[G.chain_runs % chain_k];
            st->own.chain_wait = G.chain_runs >= (uint64_t)chain_k ? ce : nullptr;
            st->own.chain_rec = ce;
            G.chain_runs++;
            rc = msm_launch(st->own, st->buf, st->n, nullptr, st->stream, nullptr, false);
            st->own.chain_wait = st->own.chain_rec = nullptr;
        } else if (replay) {
            NWV_HIP(hipGraphLaunch(st->graph, st->stream));
        } else {
            // first run of the batch (allocates its buffers) or a timed run; an untimed first run
            // also captures the graph the later runs replay (unchained form)
            rc = msm_launch(st->own, st->buf, st->n, seed, st->stream, timed ? st->ev : nullptr, false);
            if (!rc && !timed && st->n) {
                if (chain_k > 0) st->chain_ready = true;
                else rc = staged_graph(st);
            }
        }
    } else {
        rc = ed_launch(st->own, st->buf, st->n, st->stream, timed ? st->ev : nullptr);
    }
    if (rc) return rc;
    st->last_mode = mode;
    st->pending_timing = timed && st->n > 0;
    return NWV_OK;
}

static int staged_sync_locked(nwv_staged* st) {
    int rc = with_device(st->own);
    if (rc) return rc;
    NWV_HIP(hipStreamSynchronize(st->stream));
    return staged_collect_times(st);
}

int nwv_staged_sync(nwv_staged* st) {
    if (!st) return set_err(NWV_ERR_ARG, "null staged");
    std::lock_guard<std::mutex> g(st->mu);
    return staged_sync_locked(st);
}

// Verdicts of the last run.  After a batch run (mode 1) that rejected, the per-signature
// pipeline runs here to pinpoint the bad indices.
int nwv_staged_fetch(nwv_staged* st, uint64_t* verdict_bits, int* all_valid) {
    if (!st) return set_err(NWV_ERR_ARG, "null staged");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = staged_sync_locked(st);
    if (rc) return rc;
    const size_t words = (st->n + 63) / 64;
    std::vector<uint64_t> tmp;
    uint64_t* bits = verdict_bits;
    if (!bits) {
        tmp.assign(words + 1, 0);
        bits = tmp.data();
    }
    if (st->last_mode == 1 && st->n) {
        uint32_t state[2] = {0, 0};
        NWV_HIP(hipMemcpyAsync(state, st->buf.m_state.p, 8, hipMemcpyDeviceToHost, st->stream));
        NWV_HIP(hipStreamSynchronize(st->stream));
        if (state[1] == 1) {
            std::memset(bits, 0, 8 * words);
            set_ones(bits, 0, st->n);
            if (all_valid) *all_valid = 1;
            return NWV_OK;
        }
        if ((rc = ed_launch(st->own, st->buf, st->n, st->stream, nullptr, msm_reusable(st->own, st->buf, true))))
            return rc;
    }
    if (words && !st->buf.verdict.p) return set_err(NWV_ERR_ARG, "staged batch has not run");
    if (words) NWV_HIP(hipMemcpyAsync(bits, st->buf.verdict.p, 8 * words, hipMemcpyDeviceToHost, st->stream));
    NWV_HIP(hipStreamSynchronize(st->stream));
    if (all_valid) *all_valid = verdicts_all_valid(bits, st->n) ? 1 : 0;
    return NWV_OK;
}

int nwv_staged_kernel_ms(nwv_staged* st, double* avg_ms, int reset) {
    if (!st || !avg_ms) return set_err(NWV_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = staged_sync_locked(st);
    if (rc) return rc;
    const KernelLog& l = st->log[0];
    for (int k = 0; k < 3; k++) avg_ms[k] = l.runs ? l.ms[k] / l.runs : 0.0;
    if (reset) st->log[0] = KernelLog{};
    return NWV_OK;
}

int nwv_staged_kernel_times(nwv_staged* st, int mode, int cap, const char** names, double* avg_ms,
                            int reset) {
    if (!st || (mode != 0 && mode != 1) || cap < 0) return set_err(NWV_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = staged_sync_locked(st);
    if (rc) return rc;
    KernelLog& l = st->log[mode];
    const int k = std::min<int>(cap, (int)l.names.size());
    for (int i = 0; i < k; i++) {
        if (names) names[i] = l.names[i];
        if (avg_ms) avg_ms[i] = l.runs ? l.ms[i] / l.runs : 0.0;
    }
    const int total = (int)l.names.size();
    if (reset) l = KernelLog{};
    return total;
}

int nwv_staged_run_tally(nwv_staged* st, uint64_t out[2]) {
    if (!st || !out) return set_err(NWV_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = staged_sync_locked(st);
    if (rc) return rc;
    out[0] = out[1] = 0;
    if (!st->tally_ready) return NWV_OK;
    uint32_t w[2] = {0, 0};
    NWV_HIP(hipMemcpyAsync(w, st->buf.m_state.as<uint32_t>() + 2, 8, hipMemcpyDeviceToHost, st->stream));
    NWV_HIP(hipStreamSynchronize(st->stream));
    out[0] = w[0];
    out[1] = w[1];
    return NWV_OK;
}

int nwv_staged_msm_stats(nwv_staged* st, uint64_t out[8]) {
    if (!st || !out) return set_err(NWV_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = staged_sync_locked(st);
    if (rc) return rc;
    std::memset(out, 0, 8 * sizeof(uint64_t));
    if (!st->n) return NWV_OK;
    const size_t na = msm_na(st->buf, st->n);
    const MsmPlan p = msm_plan(st->n, na, st->buf.kc_split, (st->own.flags & NWV_FLAG_MSM_SORT2) ? 1 : 0);
    out[0] = p.np;
    out[1] = (uint64_t)p.lay.nw;
    out[2] = (uint64_t)p.lay.nw_z;
    out[3] = p.nkeys;
    out[5] = p.chunks;
    out[6] = p.seg;
    out[7] = na;
    if (st->buf.m_tiles.p && st->buf.m_tiles.cap >= 4 * ((size_t)MSM_MAX_WINDOWS + 1)) {
        uint32_t total = 0;  // entries = nonzero digits over all windows
        NWV_HIP(hipMemcpyAsync(&total, st->buf.m_tiles.as<uint32_t>() + MSM_MAX_WINDOWS, 4, hipMemcpyDeviceToHost,
                               st->stream));
        NWV_HIP(hipStreamSynchronize(st->stream));
        out[4] = total;
    }
    return NWV_OK;
}

int nwv_staged_mark(nwv_staged* st, int slot) {
    if (!st || slot < 0 || slot >= 65536) return set_err(NWV_ERR_ARG, "bad staged/slot");
    std::lock_guard<std::mutex> g(st->mu);
    int rc = with_device(st->own);
    if (rc) return rc;
    if ((size_t)slot >= st->marks.size()) st->marks.resize((size_t)slot + 1, nullptr);
    if (!st->marks[slot]) NWV_HIP(hipEventCreate(&st->marks[slot]));
    NWV_HIP(hipEventRecord(st->marks[slot], st->stream));
    return NWV_OK;
}

int nwv_staged_mark_elapsed(nwv_staged* a, int slot_a, nwv_staged* b, int slot_b, float* ms) {
    if (!a || !b || !ms || slot_a < 0 || slot_b < 0 || (size_t)slot_a >= a->marks.size() ||
        (size_t)slot_b >= b->marks.size() || !a->marks[slot_a] || !b->marks[slot_b])
        return set_err(NWV_ERR_ARG, "bad marks");
    NWV_HIP(hipEventSynchronize(b->marks[slot_b]));
    NWV_HIP(hipEventSynchronize(a->marks[slot_a]));
    NWV_HIP(hipEventElapsedTime(ms, a->marks[slot_a], b->marks[slot_b]));
    return NWV_OK;
}

void nwv_staged_free(nwv_staged* st) {
    if (!st) return;
    {
        std::lock_guard<std::mutex> g(st->mu);
        (void)hipSetDevice(st->own.ordinal);
        if (st->stream) (void)hipStreamSynchronize(st->stream);
        if (st->graph) (void)hipGraphExecDestroy(st->graph);
        for (auto& e : st->seed_ev)
            if (e) (void)hipEventDestroy(e);
        st->seeds.release();
        st->buf.release();
        for (auto& e : st->ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : st->marks)
            if (e) (void)hipEventDestroy(e);
        if (st->stream) (void)hipStreamDestroy(st->stream);
        st->own.stream = nullptr;
    }
    delete st;
}

// ---- BLAKE2b-256 --------------------------------------------------------------------
// Messages of at least this many bytes (the longest of the call) go 4 lanes per message
static uint64_t b2_quad_min() {
    static const uint64_t v = [] {
        const char* e = std::getenv("NWV_B2_QUAD_MIN");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)1024;
    }();
    return v;
}
// few messages (a types-layer call's header / vote / certificate preimages): the quad form too,
// for latency -- one lane's compression chain is ~4x the quad's, and m quads fill no more of the
// chip than the call has messages (NWV_B2_QUAD_MAX_M, default 4,096 messages)
static uint64_t b2_quad_max_m() {
    static const uint64_t v = [] {
        const char* e = std::getenv("NWV_B2_QUAD_MAX_M");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)4096;
    }();
    return v;
}
// out2 (optional): a second copy of the digests, e.g. straight into coherent pinned host memory
static void b2_launch(Lane& d, size_t m, uint64_t maxlen, const uint8_t* base, const uint64_t* off,
                      const uint64_t* len, uint32_t* out, uint32_t* out2 = nullptr) {
    if (maxlen >= b2_quad_min() || m <= b2_quad_max_m())
        hipLaunchKernelGGL(k_blake2b_quad, dim3((unsigned)((m + 15) / 16)), dim3(64), 0, d.stream,
                           (uint64_t)m, base, off, len, out, out2);
    else
        hipLaunchKernelGGL(k_blake2b_many, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, d.stream,
                           (uint64_t)m, base, off, len, out, out2);
}

// device pointers of a staged digest batch (views into b2_in, or the b2_base/off/len buffers)
struct B2Staged {
    const uint8_t* base;
    const uint64_t* off;
    const uint64_t* len;
};

static int b2_stage(Lane& d, size_t n, const uint8_t* base, const uint64_t* off,
                    const uint64_t* len, size_t lo, size_t hi, std::vector<uint64_t>& roff, B2Staged& st) {
    uint64_t mlo = UINT64_MAX, mhi = 0;
    for (size_t i = lo; i < hi; i++) {
        mlo = std::min<uint64_t>(mlo, off[i]);
        mhi = std::max<uint64_t>(mhi, off[i] + len[i]);
    }
    if (mhi < mlo) { mlo = 0; mhi = 0; }
    const size_t m = hi - lo, bytes = (size_t)(mhi - mlo);
    roff.resize(m);
    for (size_t i = 0; i < m; i++) roff[i] = off[lo + i] - mlo;
    int rc;
    (void)n;
    // small batches (header / vote / certificate preimages): offsets, lengths and bytes packed into
    // pinned memory and sent as ONE copy; large ones (worker batches) keep the driver's pipelined
    // pageable path, which overlaps its own staging with the DMA
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_len = up(8 * m + 8), o_bytes = o_len + up(8 * m + 8), total = o_bytes + bytes + MSG_PAD;
    if (total <= ((size_t)4 << 20)) {
        if ((rc = d.b2_in.ensure(total)) || (rc = d.b2_out.ensure(32 * m + 32))) return rc;
        NWV_HIP(hipEventSynchronize(d.b2stage_ev));
        if ((rc = d.b2stage.ensure(total))) return rc;
        uint8_t* h = static_cast<uint8_t*>(d.b2stage.p);
        std::memcpy(h, roff.data(), 8 * m);
        std::memcpy(h + o_len, len + lo, 8 * m);
        if (bytes) std::memcpy(h + o_bytes, base + mlo, bytes);
        std::memset(h + o_bytes + bytes, 0, MSG_PAD);
        NWV_HIP(nwv_stage::stage_h2d(d.b2_in.p, h, total, d.stream));  // small calls: through kernel arguments
        NWV_HIP(hipEventRecord(d.b2stage_ev, d.stream));
        const uint8_t* g = d.b2_in.as<uint8_t>();
        st = B2Staged{g + o_bytes, reinterpret_cast<const uint64_t*>(g), reinterpret_cast<const uint64_t*>(g + o_len)};
        return NWV_OK;
    }
    if ((rc = d.b2_base.ensure(bytes + MSG_PAD)) || (rc = d.b2_off.ensure(8 * m + 8)) ||
        (rc = d.b2_len.ensure(8 * m + 8)) || (rc = d.b2_out.ensure(32 * m + 32)))
        return rc;
    if (bytes) NWV_HIP(hipMemcpyAsync(d.b2_base.p, base + mlo, bytes, hipMemcpyHostToDevice, d.stream));
    NWV_HIP(hipMemsetAsync(d.b2_base.as<uint8_t>() + bytes, 0, MSG_PAD, d.stream));
    NWV_HIP(hipMemcpyAsync(d.b2_off.p, roff.data(), 8 * m, hipMemcpyHostToDevice, d.stream));
    NWV_HIP(hipMemcpyAsync(d.b2_len.p, len + lo, 8 * m, hipMemcpyHostToDevice, d.stream));
    st = B2Staged{d.b2_base.as<uint8_t>(), d.b2_off.as<uint64_t>(), d.b2_len.as<uint64_t>()};
    return NWV_OK;
}

int nwv_blake2b256_many(nwv_ctx* ctx, size_t n, const uint8_t* base, const uint64_t* off,
                        const uint64_t* len, uint8_t* out) {
    if (!ctx || (n && (!off || !len || !out))) return set_err(NWV_ERR_ARG, "null argument");
    if (n == 0) return NWV_OK;
    static const uint8_t empty[1] = {0};
    if (!base) base = empty;
    const auto ranges = nwv::shard_ranges(n, ctx->devs.size(), ctx->b2_shard_min, 1);
    return nwv::for_ranges(ranges, [&](size_t k, size_t lo, size_t hi) -> int {
        LaneRef lane(*ctx->devs[k]);
        Lane& d = *lane;
        std::vector<uint64_t> roff;
        int rc = lane.rc();
        B2Staged st{};
        if (!rc) rc = b2_stage(d, n, base, off, len, lo, hi, roff, st);
        if (!rc) {
            const size_t m = hi - lo;
            uint64_t maxlen = 0;
            for (size_t k2 = lo; k2 < hi; k2++) maxlen = std::max<uint64_t>(maxlen, len[k2]);
            b2_launch(d, m, maxlen, st.base, st.off, st.len, d.b2_out.as<uint32_t>());
            hipError_t e = hipGetLastError();
            if (e == hipSuccess) e = hipMemcpyAsync(out + 32 * lo, d.b2_out.p, 32 * m, hipMemcpyDeviceToHost, d.stream);
            if (e == hipSuccess) e = hipStreamSynchronize(d.stream);
            if (e != hipSuccess) rc = set_err(NWV_ERR_HIP, hipGetErrorString(e));
        }
        return rc;
    });
}

int nwv_ed25519_verify_batch_keyed_digests(nwv_ctx* ctx, size_t n_pre, const uint8_t* pre_base,
                                           const uint64_t* pre_off, const uint64_t* pre_len,
                                           uint8_t* digests_out, size_t n_keys, const uint8_t* keys,
                                           size_t n, const uint32_t* key_idx, const uint8_t* sig,
                                           const uint32_t* digest_idx, const uint8_t seed32[32],
                                           int* all_valid, uint64_t* verdict_bits_or_null) {
    if (!ctx || !all_valid || (n_pre && (!pre_off || !pre_len || !digests_out)) ||
        (n && (!keys || !key_idx || !sig || !digest_idx)))
        return set_err(NWV_ERR_ARG, "null argument");
    for (size_t i = 0; i < n; i++)
        if (digest_idx[i] >= n_pre) return set_err(NWV_ERR_ARG, "digest index out of range");
    *all_valid = 1;
    // message i = digest digest_idx[i]: 32 bytes at 32 * digest_idx[i] of the digest array
    thread_local std::vector<uint64_t> moff;
    thread_local std::vector<uint32_t> mlen;
    moff.resize(n);
    mlen.assign(n, 32u);
    for (size_t i = 0; i < n; i++) moff[i] = 32ull * digest_idx[i];
    if (nwv::ed_shard_ranges(n, ctx->devs.size(), ctx->shard_min).size() > 1 || n_pre == 0 || n == 0) {
        // a batch that splits over several devices: the digests come back to the host and the
        // signatures are sharded (a smaller one stays fused on device 0, below)
        int rc = nwv_blake2b256_many(ctx, n_pre, pre_base, pre_off, pre_len, digests_out);
        if (rc || n == 0) return rc;
        return nwv_ed25519_verify_batch_keyed(ctx, n_keys, keys, n, key_idx, sig, digests_out, moff.data(),
                                              mlen.data(), seed32, all_valid, verdict_bits_or_null);
    }
    static const uint8_t empty[1] = {0};
    if (!pre_base) pre_base = empty;
    uint8_t seed[32];
    fill_seed(seed32, seed);
    LaneRef lane(*ctx->devs[0]);
    Lane& d = *lane;
    int rc = lane.rc();
    std::vector<uint64_t> roff;
    B2Staged st{};
    if (!rc) rc = b2_stage(d, n_pre, pre_base, pre_off, pre_len, 0, n_pre, roff, st);
    if (rc) return rc;
    // the digests stay on the device as the message arena of the batch; the over-read slack past
    // them needs no particular contents (SHA-512 and BLAKE2b mask the bytes past a message)
    if ((rc = d.b2_out.ensure(32 * n_pre + 4 * MSG_PAD))) return rc;
    uint64_t maxlen = 0;
    for (size_t k = 0; k < n_pre; k++) maxlen = std::max<uint64_t>(maxlen, pre_len[k]);
    // the batch is staged before the hash launch (its copy does not depend on the digests), so
    // hash and verification run back to back; no host round trip between them
    rc = ed_stage_keyed(d, d.ed, 0, n, n_keys, keys, key_idx, sig, nullptr, moff.data(), mlen.data(), seed,
                        &d.b2_out);
    if (rc) return rc;
    // the hash also writes the digests straight into coherent pinned host memory (no copy back)
    if ((rc = d.b2dig.ensure(32 * n_pre, hipHostMallocCoherent | hipHostMallocMapped))) return rc;
    b2_launch(d, n_pre, maxlen, st.base, st.off, st.len, d.b2_out.as<uint32_t>(), static_cast<uint32_t*>(d.b2dig.p));
    NWV_HIP(hipGetLastError());
    int ok = 1;
    rc = batch_on_device(d, d.ed, n, seed, d.stream, &ok, verdict_bits_or_null, true);
    if (rc) return rc;
    if (!ok) *all_valid = 0;
    NWV_HIP(hipStreamSynchronize(d.stream));  // already synchronised by the verdict read
    std::memcpy(digests_out, d.b2dig.p, 32 * n_pre);
    return NWV_OK;
}

int nwv_batch_digest_serialized(nwv_ctx* ctx, size_t n, const uint8_t* base, const uint64_t* off,
                                const uint64_t* len, uint8_t* out, int64_t* err_offset) {
    if (!ctx || (n && (!base || !off || !len || !out || !err_offset)))
        return set_err(NWV_ERR_ARG, "null argument");
    if (n == 0) return NWV_OK;
    LaneRef lane(*ctx->devs[0]);
    Lane& d = *lane;
    int rc = lane.rc();
    std::vector<uint64_t> roff;
    B2Staged st{};
    if (!rc) rc = b2_stage(d, n, base, off, len, 0, n, roff, st);
    if (rc) return rc;
    size_t bytes = 0;
    for (size_t i = 0; i < n; i++) bytes = std::max<size_t>(bytes, roff[i] + len[i]);
    if ((rc = d.b2_packed.ensure(bytes + MSG_PAD)) || (rc = d.b2_plen.ensure(8 * n + 8)) ||
        (rc = d.b2_err.ensure(8 * n + 8)))
        return rc;
    NWV_HIP(hipMemsetAsync(d.b2_packed.p, 0, bytes + MSG_PAD, d.stream));
    hipLaunchKernelGGL(k_batch_compact, dim3((unsigned)n), dim3(256), 0, d.stream, (uint64_t)n,
                       st.base, st.off, st.len, d.b2_packed.as<uint8_t>(), d.b2_plen.as<uint64_t>(), d.b2_err.as<int64_t>());
    uint64_t maxlen = 0;
    for (size_t k2 = 0; k2 < n; k2++) maxlen = std::max<uint64_t>(maxlen, len[k2]);
    b2_launch(d, n, maxlen, d.b2_packed.as<uint8_t>(), st.off, d.b2_plen.as<uint64_t>(),
              d.b2_out.as<uint32_t>());
    NWV_HIP(hipGetLastError());
    NWV_HIP(hipMemcpyAsync(out, d.b2_out.p, 32 * n, hipMemcpyDeviceToHost, d.stream));
    NWV_HIP(hipMemcpyAsync(err_offset, d.b2_err.p, 8 * n, hipMemcpyDeviceToHost, d.stream));
    NWV_HIP(hipStreamSynchronize(d.stream));
    for (size_t i = 0; i < n; i++)
        if (err_offset[i] >= 0) return set_err(NWV_ERR_ARG, "malformed serialized batch");
    return NWV_OK;
}

// ---- synthetic signing ----------------------------------------------------------------
int nwv_ed25519_sign_many(nwv_ctx* ctx, size_t n, const uint8_t* seeds, const uint8_t* msg_base,
                          const uint64_t* msg_off, const uint32_t* msg_len, uint8_t* pk_out,
                          uint8_t* sig_out) {
    if (!ctx || (n && (!seeds || !msg_off || !msg_len || !pk_out || !sig_out)))
        return set_err(NWV_ERR_ARG, "null argument");
    if (n == 0) return NWV_OK;
    static const uint8_t empty[1] = {0};
    if (!msg_base) msg_base = empty;
    return for_shards(ctx, n, [&](Lane& d, size_t lo, size_t hi) -> int {
        // messages via the Ed25519 staging; seeds go to kbuf, outputs come back in pk / sig
        int rc = ed_stage(d, d.ed, lo, hi, nullptr, nullptr, msg_base, msg_off, msg_len, nullptr);
        if (rc) return rc;
        const size_t m = hi - lo;
        if ((rc = d.ed.kbuf.ensure(32 * m + 16))) return rc;
        NWV_HIP(hipMemcpyAsync(d.ed.kbuf.p, seeds + 32 * lo, 32 * m, hipMemcpyHostToDevice, d.stream));
        hipLaunchKernelGGL(k_sign, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, d.stream,
                           (uint64_t)m, d.ed.kbuf.as<uint8_t>(), d.ed.msg.as<uint8_t>(),
                           d.ed.off.as<uint64_t>(), d.ed.len.as<uint32_t>(), d.btab().as<uint32_t>(),
                           d.ed.pk.as<uint8_t>(), d.ed.sig.as<uint8_t>());
        NWV_HIP(hipGetLastError());
        NWV_HIP(hipMemcpyAsync(pk_out + 32 * lo, d.ed.pk.p, 32 * m, hipMemcpyDeviceToHost, d.stream));
        NWV_HIP(hipMemcpyAsync(sig_out + 64 * lo, d.ed.sig.p, 64 * m, hipMemcpyDeviceToHost, d.stream));
        NWV_HIP(hipStreamSynchronize(d.stream));
        return NWV_OK;
    });
}

}  // extern "C"
