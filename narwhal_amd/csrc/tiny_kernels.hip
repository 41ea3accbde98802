// tiny_kernels.hip -- one-launch verification of tiny keyed batches (gfx950), for the per-call
// paths of SURVEY.md §8 a1-a3: Certificate::verify (types/src/primary.rs:487-537, a committee's
// quorum of vote signatures plus the header's), Header::verify / Vote::verify (:150-183, :307-328).
//
// A batch of at most TINY_MAX signatures whose keys are registered committee keys is checked
// signature by signature -- ZIP-215's cofactored equation [8](R - ([s]B - [k]A)) = 0, exactly the
// per-signature verdict, so no random coefficients and no fallback pass -- in ONE launch:
//   wave 0   R's decompression on a 16-lane row (msm_kernels.hip row_decompress; the one long
//            dependent chain, ~250 row squarings)
//   wave 1   lane 0: k = SHA-512(R || A || M) mod l, s < l, the signed radix-16 digits of s and k;
//            then, while R still decompresses, [s]B - [k]A from two fixed-base combs -- B's (per
//            device) and the key's (i 16^j A, built once at key registration, k_key_comb_fill) --
//            one table entry of each per lane and a six-level tree of quad-lane additions in LDS:
//            no doubling chain at all; then [8] of that sum (three quad-lane doublings), while
//            wave 0 doubles R three times on its rows; [8] R = [8]([s]B - [k]A) tested projectively
//   last     the last workgroup to arrive (one per signature, grid <= 64) collects the verdict bits,
//            writes the batch verdict and stores both into the lane's polled host word
// Against the batch MSM path for these sizes (five launches: prep, sort, bucket, tail's 128-
// doubling row chain), the device time is the R decompression plus ~10 us.
#include "msm.h"

using namespace nwv;

static constexpr int TINY_MAX = 64;
struct TinyArgs {
    const uint8_t* pk;      // [n][32] each signature's key (the hash's A bytes)
    const uint8_t* sig;     // [n][64]
    const uint8_t* msg;     // message arena; off[n] / len[n] index it
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* kc;     // key cache records: word MSM_PT_WORDS - 1 of a slot = A did not decode
    const uint32_t* combs;  // per-key comb tables (COMB_WORDS words each)
    const uint32_t* bcomb;  // B's comb table
    // workspace, zero between calls: [0, 2) accumulated verdict bits, [2] arrivals (the last
    // workgroup resets both); results: [4, 6) verdict bits, [6] batch verdict
    uint32_t* ws;
    uint32_t* hword;        // the lane's polled host word or null: [0] (hseq << 2) | code, [2, 4) bits
    uint32_t n, hseq;
    unsigned long long* stamps;  // diagnostics (NWV_TINY_STAMPS): workgroup 0's phase times, or null
    uint32_t kslot[TINY_MAX];  // signature i's key cache slot
    uint32_t cidx[TINY_MAX];   // signature i's comb table
};

namespace {
// signed radix-16 digits of c (msm.h comb_digits), straight into LDS
__device__ __forceinline__ void tiny_digits(const uint32_t c[8], int* out) {
    int carry = 0;
#pragma unroll 4
    for (int j = 0; j < COMB_TABLES; j++) {
        int v = (int)((c[j >> 3] >> (4 * (j & 7))) & 15u) + carry;
        carry = 0;
        if (j + 1 < COMB_TABLES && v >= 8) {
            v -= 16;
            carry = 1;
        }
        out[j] = v;
    }
}
}  // namespace

// One workgroup of two waves per signature (a CU each: nothing else competes for their SIMDs).
// Wave 0 decompresses R on a row -- the critical chain -- and doubles it three times there; wave 1
// hashes on one lane, then sums the signature's comb terms on all 64 lanes and multiplies the sum
// by 8 while R is still decompressing; after the barrier lane 0 compares the two projectively
// (was: subtract R, three doublings, identity test, all after the barrier: 50.5 us to the verdict).
// Phase stamps of workgroup 0 with NWV_TINY_STAMPS: [1] R decoded, [3] [8] R, [2] hashed, [4]
// [8] of the comb sum, [5] barrier, [6] verdict.
static constexpr int TINY_WAVES = 2;
// s_memrealtime (100 MHz) into stamp slot k, by lane 0 of a wave of workgroup 0
#define NWV_TINY_STAMP(k)                                                                       \
    do {                                                                                        \
        if (a.stamps && blockIdx.x == 0 && lane == 0) a.stamps[k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
extern "C" __global__ void __launch_bounds__(64 * TINY_WAVES) k_ed_tiny(TinyArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ uint32_t rsh[4 * 48];     // wave 0's rows (48 words each; row 0 is R)
    __shared__ uint32_t rrec[32];        // [8] R: X | Y | Z (10 limbs each); word 31: 1 = R does not decode
    __shared__ int dg[2][COMB_TABLES];   // digits of s and of k
    __shared__ uint32_t hok;             // s < l
    __shared__ uint32_t pts[64 * P3_WORDS];  // the 64 comb terms, summed in place
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const uint32_t i = blockIdx.x;       // this workgroup's signature (grid = n)
    if (wv == 0) {
        NWV_TINY_STAMP(0);
        const int row = lane >> 4, limb = lane & 15;
        // every row decompresses R (the row products are wave-wide anyway); row 0 keeps it
        const uint32_t y16 = reinterpret_cast<const uint16_t*>(a.sig + 64 * (size_t)i)[limb];
        uint32_t* sh = rsh + 48 * row;
        const bool ok = row_decompress(y16, lane, row, limb, sh);
        NWV_TINY_STAMP(1);
        // [8] R on the rows while wave 1 finishes [8]([s]B - [k]A): three row doublings (one
        // multiply latency each) from (2x : 2y : 2) = ((y+x) - (y-x) : (y+x) + (y-x) : 2)
        rowf::RowConsts k = rowf::row_consts();
        k.rot = 1;
        const uint32_t ypx = sh[limb], ymx = sh[16 + limb];
        rowf::RowP3 d{rowf::carry32(rowf::sub(ypx, ymx, k), k), rowf::carry32(ypx + ymx, k),
                      rowf::sel(rowf::limb_is(0), 0u, 2u), 0u};
#pragma unroll 1
        for (int r = 0; r < 3; r++) d = rowf::row_dbl(d, k);
        rowf::lds_order();
        sh[limb] = d.X;
        sh[16 + limb] = d.Y;
        sh[32 + limb] = d.Z;
        rowf::lds_order();
        if (row == 0 && limb < 3) store_fe(&rrec[10 * limb], fe_from_limbs16(sh + 16 * limb));  // X | Y | Z
        if (lane == 0) rrec[31] = ok ? 0u : 1u;
        NWV_TINY_STAMP(3);
    } else {
        if (lane == 0) {
            uint32_t Aw[8], Rw[8], Sw[8], k[8];
            msm_load8(a.pk + 32 * (size_t)i, Aw);
            msm_load8(a.sig + 64 * (size_t)i, Rw);
            msm_load8(a.sig + 64 * (size_t)i + 32, Sw);
            const bool sok = lane_hash(Aw, Rw, Sw, a.msg + a.off[i], a.len[i], k) == FLAG_S_OK;
            hok = sok ? 1u : 0u;
            if (!sok) {  // s >= l fails the signature; its digits would index past the tables
#pragma unroll
                for (int q = 0; q < 8; q++) Sw[q] = 0u;
            }
            tiny_digits(Sw, dg[0]);
            tiny_digits(k, dg[1]);
        }
        rowf::lds_order();
        NWV_TINY_STAMP(2);
        const int ds = dg[0][lane], dk = dg[1][lane];
        ge_p3 P = ge_p3_identity();
        if (ds) {
            const int m = ds < 0 ? -ds : ds;
            P = ge_p1p1_to_p3(ge_madd(P, msm_load_point(a.bcomb + MSM_PT_WORDS * (COMB_ENTRIES * lane + m - 1), ds < 0)));
        }
        if (dk) {  // -[k]A: the entry negated for a positive digit
            const int m = dk < 0 ? -dk : dk;
            const uint32_t* ct = a.combs + (size_t)COMB_WORDS * a.cidx[i];
            P = ge_p1p1_to_p3(ge_madd(P, msm_load_point(ct + MSM_PT_WORDS * (COMB_ENTRIES * lane + m - 1), dk > 0)));
        }
        // the 64 terms summed by lane quads (msm_kernels.hip quad_p3_add: three multiply
        // latencies an addition instead of nine), a tree in place: level o adds slot i + o into i
        store_p3(pts + P3_WORDS * lane, P);
        rowf::lds_order();
        const int q = lane & 3;
#pragma unroll 1
        for (int o = 1; o < 64; o <<= 1) {
#pragma unroll 1
            for (int g = lane >> 2; g < 32 / o; g += 16) quad_p3_add(pts, 2 * o * g, o, q);
            rowf::lds_order();
        }
        // [8] P as three doublings on the first quad (an addition of the slot to itself)
        if (lane < 4)
#pragma unroll 1
            for (int r = 0; r < 3; r++) {
                quad_p3_add(pts, 0, 0, lane);
                rowf::lds_order();
            }
        NWV_TINY_STAMP(4);
    }
    __syncthreads();  // [8] R and [8]([s]B - [k]A) done
    if (wv == 1) {
        NWV_TINY_STAMP(5);
        // the cofactored equation [8](R - ([s]B - [k]A)) = 0 as [8] R = [8] P, projectively: the four
        // cross products on lanes 0..3 (P.X RZ, RX P.Z, P.Y RZ, RY P.Z), canonical words into LDS
        // (wave 0's rows, free after the barrier), compared by lane 0
        if (lane < 4) {
            const uint32_t* u = ((lane & 1) ? rrec : pts) + (lane < 2 ? 0 : 10);
            const uint32_t* v = ((lane & 1) ? pts : rrec) + 20;
            fe_freeze(fe_mul(load_fe(u), load_fe(v)), rsh + 8 * lane);
        }
        rowf::lds_order();
        if (lane == 0) {
            bool id = true;
#pragma unroll
            for (int q = 0; q < 8; q++) id = id && rsh[q] == rsh[8 + q] && rsh[16 + q] == rsh[24 + q];
            const bool aok = a.kc[(size_t)KC_SLOT_WORDS * a.kslot[i] + MSM_PT_WORDS - 1] == 0u;
            const bool ok = id && aok && hok && rrec[31] == 0u;
            NWV_TINY_STAMP(6);
            unsigned long long* acc = reinterpret_cast<unsigned long long*>(a.ws);
            if (ok) atomicOr(acc, 1ull << i);
            __threadfence();
            const uint32_t arrived = atomicAdd(a.ws + 2, 1u);
            if (arrived == gridDim.x - 1) {  // the last workgroup: every verdict bit is in
                __threadfence();
                const unsigned long long bits = atomicExch(acc, 0ull);
                a.ws[2] = 0u;
                const unsigned long long want = a.n >= 64 ? ~0ull : ((1ull << a.n) - 1ull);
                const bool all = bits == want;
                a.ws[4] = (uint32_t)bits;
                a.ws[5] = (uint32_t)(bits >> 32);
                a.ws[6] = all ? 1u : 0u;
                if (a.hword) {
                    a.hword[2] = (uint32_t)bits;
                    a.hword[3] = (uint32_t)(bits >> 32);
                    __hip_atomic_store(a.hword, (a.hseq << 2) | (all ? 1u : 2u), __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
#endif
}

// Per-key comb tables of newly registered keys: lane e of key q = entry e of its table, i 16^j A
// (j = e / 8, i = e % 8 + 1): the key's decompression and a chain of 4 j doublings per lane.  Once
// per key (nwv_keycache_register); a key that does not decode gets the identity's table (its
// signatures fail on the cache record's decode flag before the table matters).
extern "C" __global__ void __launch_bounds__(64) k_key_comb_fill(uint32_t cnt, const uint8_t* __restrict__ keys,
                                                                 const uint32_t* __restrict__ cidx,
                                                                 uint32_t* __restrict__ combs) {
    const uint32_t e = blockIdx.x * 64 + threadIdx.x;
    const uint32_t q = e / (COMB_TABLES * COMB_ENTRIES), r = e % (COMB_TABLES * COMB_ENTRIES);
    if (q >= cnt) return;
    uint32_t w[8];
    msm_load8(keys + 32 * (size_t)q, w);
    ge_p3 A;
    if (!ge_decompress(w, A)) A = ge_p3_identity();
    comb_entry_of(A, (int)(r / COMB_ENTRIES), (int)(r % COMB_ENTRIES) + 1,
                  combs + (size_t)COMB_WORDS * cidx[q] + (size_t)MSM_PT_WORDS * r);
}
