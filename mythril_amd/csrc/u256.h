// u256.h — 256-bit two's-complement arithmetic on 8 x 32-bit limbs held in VGPRs.
//
// One lane holds one candidate's value; limbs are little-endian (x[0] = bits 0..31).
// Everything is fully unrolled so the limbs stay in registers; carry chains map onto
// v_add_co_u32 / v_addc_co_u32 (__builtin_addc) and products onto v_mad_u64_u32.
// Widths w < 256 are handled by the callers (mask / sign-extend at the op boundary).
// Semantics follow SMT-LIB2 (z3) — see oracle/pyoracle.py for the CPU restatement.
#pragma once
#include <stdint.h>

#define PF_INL __device__ __forceinline__

namespace pf {

struct u256 {
    uint32_t l[8];
};

PF_INL u256 zero256() {
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = 0;
    return r;
}

PF_INL u256 ones256() {
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = 0xffffffffu;
    return r;
}

PF_INL u256 add256(const u256& a, const u256& b) {
    u256 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t co;
        r.l[i] = __builtin_addc(a.l[i], b.l[i], c, &co);
        c = co;
    }
    return r;
}

// a + b, returns carry-out in *cout
PF_INL u256 add256c(const u256& a, const u256& b, uint32_t* cout) {
    u256 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t co;
        r.l[i] = __builtin_addc(a.l[i], b.l[i], c, &co);
        c = co;
    }
    *cout = c;
    return r;
}

PF_INL u256 sub256(const u256& a, const u256& b) {
    u256 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t co;
        r.l[i] = __builtin_subc(a.l[i], b.l[i], c, &co);
        c = co;
    }
    return r;
}

// a - b, returns borrow-out (1 iff a < b unsigned)
PF_INL u256 sub256b(const u256& a, const u256& b, uint32_t* bout) {
    u256 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t co;
        r.l[i] = __builtin_subc(a.l[i], b.l[i], c, &co);
        c = co;
    }
    *bout = c;
    return r;
}

PF_INL uint32_t ult256(const u256& a, const u256& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t co;
        (void)__builtin_subc(a.l[i], b.l[i], c, &co);
        c = co;
    }
    return c;
}

PF_INL uint32_t eq256(const u256& a, const u256& b) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d |= a.l[i] ^ b.l[i];
    return d == 0;
}

PF_INL uint32_t iszero256(const u256& a) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d |= a.l[i];
    return d == 0;
}

PF_INL u256 neg256(const u256& a) { return sub256(zero256(), a); }

PF_INL u256 not256(const u256& a) {
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = ~a.l[i];
    return r;
}

PF_INL u256 sel256(uint32_t c, const u256& a, const u256& b) {
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = c ? a.l[i] : b.l[i];
    return r;
}

// truncated 256 x 256 -> 256 product (36 partial products)
PF_INL u256 mul256(const u256& a, const u256& b) {
    u256 r = zero256();
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8 - i; j++) {
            uint64_t t = (uint64_t)a.l[i] * b.l[j] + r.l[i + j] + carry;
            r.l[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
    }
    return r;
}

// full product high half is non-zero? (a * b >= 2^256).  Used for bvumul_noovfl.
PF_INL uint32_t mul256_overflows(const u256& a, const u256& b) {
    // any a[i]*b[j] with i+j >= 8 non-zero, or carry out of the truncated product.
    uint32_t hi = 0;
    u256 r = zero256();
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (i + j < 8) {
                uint64_t t = (uint64_t)a.l[i] * b.l[j] + r.l[i + j] + carry;
                r.l[i + j] = (uint32_t)t;
                carry = t >> 32;
            } else {
                hi |= (a.l[i] != 0u && b.l[j] != 0u) ? 1u : 0u;
            }
        }
        hi |= (carry != 0) ? 1u : 0u;
    }
    return hi;
}

// logical shift left by s (per lane, any value); s >= 256 -> 0
PF_INL u256 shl256(const u256& a, uint32_t s, uint32_t big) {
    u256 x = a;
    // limb moves by 4, 2, 1 limbs
    if (__builtin_expect(1, 1)) {
        uint32_t m = (s >> 7) & 1;
#pragma unroll
        for (int i = 7; i >= 0; i--) x.l[i] = m ? (i >= 4 ? x.l[i - 4] : 0u) : x.l[i];
        m = (s >> 6) & 1;
#pragma unroll
        for (int i = 7; i >= 0; i--) x.l[i] = m ? (i >= 2 ? x.l[i - 2] : 0u) : x.l[i];
        m = (s >> 5) & 1;
#pragma unroll
        for (int i = 7; i >= 0; i--) x.l[i] = m ? (i >= 1 ? x.l[i - 1] : 0u) : x.l[i];
    }
    uint32_t bs = s & 31;
    u256 r;
#pragma unroll
    for (int i = 7; i >= 1; i--) r.l[i] = bs ? ((x.l[i] << bs) | (x.l[i - 1] >> (32 - bs))) : x.l[i];
    r.l[0] = x.l[0] << bs;
    if (big) r = zero256();
    return r;
}

// shift right by s with fill word f (0 = logical, 0xffffffff = arithmetic fill); s < 256
PF_INL u256 shr256(const u256& a, uint32_t s, uint32_t f) {
    u256 x = a;
    uint32_t m = (s >> 7) & 1;
#pragma unroll
    for (int i = 0; i < 8; i++) x.l[i] = m ? (i + 4 < 8 ? x.l[i + 4] : f) : x.l[i];
    m = (s >> 6) & 1;
#pragma unroll
    for (int i = 0; i < 8; i++) x.l[i] = m ? (i + 2 < 8 ? x.l[i + 2] : f) : x.l[i];
    m = (s >> 5) & 1;
#pragma unroll
    for (int i = 0; i < 8; i++) x.l[i] = m ? (i + 1 < 8 ? x.l[i + 1] : f) : x.l[i];
    uint32_t bs = s & 31;
    u256 r;
#pragma unroll
    for (int i = 0; i < 7; i++) r.l[i] = bs ? ((x.l[i] >> bs) | (x.l[i + 1] << (32 - bs))) : x.l[i];
    r.l[7] = bs ? ((x.l[7] >> bs) | (f << (32 - bs))) : x.l[7];
    return r;
}

PF_INL uint32_t clz256(const u256& a) {
    uint32_t n = 0, done = 0;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
        uint32_t z = a.l[i] ? (uint32_t)__builtin_clz(a.l[i]) : 32u;
        n += done ? 0u : z;
        done |= (a.l[i] != 0u);
    }
    return n;  // 256 for zero
}

// unsigned divide: q = a / b, r = a % b, with z3 conventions for b == 0 (q = ~0, r = a).
// Restoring binary division over only the bits where the quotient can be non-zero:
// per lane (clz(b) - clz(a) + 1) steps; the wave runs the maximum over its lanes.
PF_INL void udivrem256(const u256& a, const u256& b, u256* q, u256* r) {
    uint32_t bz = iszero256(b);
    uint32_t ca = clz256(a), cb = clz256(b);
    int32_t steps = bz ? -1 : ((int32_t)cb - (int32_t)ca);  // quotient bit positions sh..0
    u256 rem = a;
    u256 quo = zero256();
    if (steps >= 0) {
        uint32_t sh = (uint32_t)steps;
        u256 d = shl256(b, sh, 0u);
        for (int32_t i = steps; i >= 0; i--) {
            uint32_t borrow;
            u256 t = sub256b(rem, d, &borrow);
            uint32_t ge = borrow ^ 1u;
            rem = sel256(ge, t, rem);
            // set quotient bit i
            uint32_t li = (uint32_t)i >> 5, bit = 1u << ((uint32_t)i & 31);
#pragma unroll
            for (int k = 0; k < 8; k++) quo.l[k] |= (ge && (uint32_t)k == li) ? bit : 0u;
            // d >>= 1
#pragma unroll
            for (int k = 0; k < 7; k++) d.l[k] = (d.l[k] >> 1) | (d.l[k + 1] << 31);
            d.l[7] >>= 1;
        }
    }
    *q = bz ? ones256() : quo;
    *r = rem;  // b == 0 -> a
}

}  // namespace pf
