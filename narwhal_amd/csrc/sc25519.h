// sc25519.h -- scalars mod l = 2^252 + 27742317777372353535851937790883648493 on 32-bit VALU.
//
// Replaces curve25519-dalek-ng's Scalar::from_hash (512-bit reduction) and
// Scalar::from_canonical_bytes (s < l, top bit clear) used by ed25519-consensus 2.0.1
// (SURVEY.md Appendix A steps 2 and 4).  Reduction is Barrett (HAC 14.42) with b = 2^32,
// k = 8, mu = floor(2^512 / l) (9 words); every partial product is one v_mad_u64_u32.
#pragma once
#include "fe25519.h"

namespace nwv {

NWV_HD uint32_t sc_l(int i) {
    const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                           0u, 0u, 0u, 0x10000000u};
    return L[i];
}
NWV_HD uint32_t sc_mu(int i) {
    const uint32_t MU[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                            0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
    return MU[i];
}

// s < l (and therefore bit 255 clear): Scalar::from_canonical_bytes
NWV_HD bool sc_is_canonical(const uint32_t s[8]) {
    bool lt = false, decided = false;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
        const uint32_t a = s[i], b = sc_l(i);
        if (!decided && a != b) { lt = a < b; decided = true; }
    }
    return lt;
}

// r = x mod l for a 512-bit x (16 little-endian words)
NWV_HD void sc_reduce512(const uint32_t x[16], uint32_t r[8]) {
    uint32_t q2[18];
#pragma unroll
    for (int i = 0; i < 18; i++) q2[i] = 0;
    // q2 = (x >> 224) * mu  (9 x 9 words)
#pragma unroll
    for (int i = 0; i < 9; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < 9; j++) {
            uint64_t t = (uint64_t)x[7 + i] * sc_mu(j) + q2[i + j] + carry;
            q2[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        q2[i + 9] = (uint32_t)carry;
    }
    // r2 = (q3 * l) mod 2^288, q3 = q2 >> 288
    uint32_t r2[9];
#pragma unroll
    for (int i = 0; i < 9; i++) r2[i] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (i + j < 9) {
                uint64_t t = (uint64_t)q2[9 + i] * sc_l(j) + r2[i + j] + carry;
                r2[i + j] = (uint32_t)t;
                carry = t >> 32;
            }
        }
        if (i + 8 < 9) r2[i + 8] += (uint32_t)carry;
    }
    // rr = (x mod 2^288) - r2 (mod 2^288)
    uint32_t rr[9];
    uint64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        uint64_t t = (uint64_t)x[i] - r2[i] - borrow;
        rr[i] = (uint32_t)t;
        borrow = (t >> 63) & 1;
    }
    // at most two conditional subtractions of l
#pragma unroll
    for (int rep = 0; rep < 2; rep++) {
        uint32_t t[9];
        uint64_t b = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            uint64_t d = (uint64_t)rr[i] - (i < 8 ? sc_l(i) : 0u) - b;
            t[i] = (uint32_t)d;
            b = (d >> 63) & 1;
        }
        const bool keep = b != 0;  // rr < l
#pragma unroll
        for (int i = 0; i < 9; i++) rr[i] = keep ? rr[i] : t[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = rr[i];
}

// r = a * b mod l (a, b < 2^256)
NWV_HD void sc_mul(const uint32_t a[8], const uint32_t b[8], uint32_t r[8]) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
            x[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        x[i + 8] = (uint32_t)carry;
    }
    sc_reduce512(x, r);
}

// r = a + b mod l (a, b < l)
NWV_HD void sc_add(const uint32_t a[8], const uint32_t b[8], uint32_t r[8]) {
    uint32_t x[16];
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t t = (uint64_t)a[i] + b[i] + carry;
        x[i] = (uint32_t)t;
        carry = t >> 32;
    }
    x[8] = (uint32_t)carry;
#pragma unroll
    for (int i = 9; i < 16; i++) x[i] = 0;
    sc_reduce512(x, r);
}

// 256-bit add of the constant sum_i c * 2^(w i), the signed-digit recoding offset:
// with y = x + sum_i (2^(w-1)) 2^(w i), digit_i = window_i(y) - 2^(w-1) in [-2^(w-1), 2^(w-1))
NWV_HD void sc_recode_offset(const uint32_t x[8], uint32_t y[8], uint32_t pattern) {
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t t = (uint64_t)x[i] + pattern + carry;
        y[i] = (uint32_t)t;
        carry = t >> 32;
    }
}

}  // namespace nwv
