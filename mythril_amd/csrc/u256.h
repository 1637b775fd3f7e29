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

// truncated square: 16 cross products (i < j, i + j <= 7), doubled, plus the 4 diagonal
// squares a_i^2 (2i <= 7) — 20 partial products instead of mul256's 36.
PF_INL u256 sqr256(const u256& a) {
    u256 r = zero256();
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t carry = 0;
#pragma unroll
        for (int j = i + 1; j <= 7 - i; j++) {
            uint64_t t = (uint64_t)a.l[i] * a.l[j] + r.l[i + j] + carry;
            r.l[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
    }
#pragma unroll
    for (int i = 7; i >= 1; i--) r.l[i] = (r.l[i] << 1) | (r.l[i - 1] >> 31);
    r.l[0] <<= 1;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t t = (uint64_t)a.l[i] * a.l[i] + r.l[2 * i] + c;
        r.l[2 * i] = (uint32_t)t;
        uint64_t t2 = (t >> 32) + r.l[2 * i + 1];
        r.l[2 * i + 1] = (uint32_t)t2;
        c = t2 >> 32;
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

// (q, r) = (min(num / v, 2^32 - 1), num - q * v) for a normalised divisor v >= 2^31:
// an f64 quotient estimate (off by at most one) corrected exactly in integers — far
// cheaper than a generic 64-bit division.  With q clamped, r may exceed v (Knuth D3
// then only refines q downwards, as it must).
PF_INL void div64_norm(uint64_t num, uint32_t v, uint64_t* q_out, uint64_t* r_out) {
    const double dn = (double)(uint32_t)(num >> 32) * 4294967296.0 + (double)(uint32_t)num;
    const double dv = (double)v;
    uint64_t q = (uint64_t)(dn / dv);
    int64_t r = (int64_t)(num - q * (uint64_t)v);
    if (r < 0) {
        q -= 1;
        r += (int64_t)v;
    }
    if (r < 0) {
        q -= 1;
        r += (int64_t)v;
    }
    if (r >= (int64_t)v) {
        q += 1;
        r -= (int64_t)v;
    }
    if (q > 0xffffffffull) {
        q = 0xffffffffull;
        r = (int64_t)(num - q * (uint64_t)v);
    }
    *q_out = q;
    *r_out = (uint64_t)r;
}

// unsigned divide: q = a / b, r = a % b, with z3 conventions for b == 0 (q = ~0, r = a).
// Knuth algorithm D on 32-bit limbs: normalise b so its top bit is set (shift s = clz(b)),
// then produce the 8 quotient digits from the top down; each digit is estimated from the top
// two limbs of the running remainder divided by the top divisor limb, refined with the
// second limb (at most two decrements), and fixed by at most one add-back after the
// multiply-subtract.  Digits whose remainder window is below the divisor in every lane of
// the wave are skipped (wave-uniform branch), so similar-magnitude operands cost one or two
// digits.  All limb indices are compile-time (fully unrolled): no scratch.
PF_INL void udivrem256(const u256& a, const u256& b, u256* q, u256* r) {
    const uint32_t bz = iszero256(b);
    const uint32_t s = bz ? 0u : clz256(b);
    const u256 B = shl256(b, s, 0u);
    const u256 lo = shl256(a, s, 0u);
    u256 hi = zero256();
    if (s != 0u) hi = shr256(a, 256u - s, 0u);  // bits of a shifted out of the top
    uint32_t u[17];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u[i] = lo.l[i];
        u[8 + i] = hi.l[i];
    }
    u[16] = 0u;
    u256 Q = zero256();
    const uint32_t b7 = B.l[7], b6 = B.l[6];
#pragma unroll
    for (int j = 7; j >= 0; j--) {
        const uint32_t u2 = u[j + 8], u1 = u[j + 7], u0 = u[j + 6];
        const bool need = (u2 != 0u) || (u1 >= b7);
        if (__ballot(need && !bz) == 0ull) continue;  // digit is 0 in every lane
        // estimate: (u2:u1) / b7, clamped to 2^32 - 1 (u2 <= b7 by the invariant)
        const uint64_t num = ((uint64_t)u2 << 32) | u1;
        uint64_t qh, rh;
        div64_norm(num, b7, &qh, &rh);
        // refine with the second divisor limb (Knuth D3): at most two decrements
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const bool big = (rh >> 32) == 0ull &&
                             qh * (uint64_t)b6 > ((rh << 32) | (uint64_t)u0);
            qh -= big ? 1ull : 0ull;
            rh += big ? (uint64_t)b7 : 0ull;
        }
        uint32_t qd = need ? (uint32_t)qh : 0u;
        // multiply-subtract: u[j .. j+8] -= qd * B
        uint64_t carry = 0;
        uint32_t borrow = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint64_t p = (uint64_t)qd * B.l[i] + carry;
            carry = p >> 32;
            uint32_t bo;
            u[j + i] = __builtin_subc(u[j + i], (uint32_t)p, borrow, &bo);
            borrow = bo;
        }
        uint32_t bo;
        u[j + 8] = __builtin_subc(u[j + 8], (uint32_t)carry, borrow, &bo);
        // went negative: add B back once (D6)
        if (bo) {
            qd -= 1u;
            uint32_t c = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                uint32_t co;
                u[j + i] = __builtin_addc(u[j + i], B.l[i], c, &co);
                c = co;
            }
            u[j + 8] += c;
        }
        Q.l[j] = qd;
    }
    u256 R;
#pragma unroll
    for (int i = 0; i < 8; i++) R.l[i] = u[i];
    R = shr256(R, s, 0u);
    *q = bz ? ones256() : Q;
    *r = bz ? a : R;
}

// base^e mod 2^256, left-to-right over 2-bit exponent digits: one square per bit and one
// multiply per digit (table base, base^2, base^3) — ~1.06 products per exponent bit
// instead of square-and-always-multiply's 2.  `nbits` (wave-uniform) must be >= every
// lane's bitlen(e); the digit loop is uniform, lanes differ only in the selected factor.
PF_INL u256 exp256(const u256& base, const u256& e, uint32_t nbits) {
    const u256 b2 = sqr256(base);
    const u256 b3 = mul256(b2, base);
    nbits = (nbits + 1u) & ~1u;
    // align the top digit at bits 255..254 (nbits == 0 runs no digit)
    u256 ex = shl256(e, (256u - nbits) & 255u, 0u);
    u256 r = zero256();
    r.l[0] = 1u;
#pragma unroll 1
    for (uint32_t i = 0; i < nbits; i += 2u) {
        if (i) {
            r = sqr256(r);
            r = sqr256(r);
        }
        const uint32_t d = ex.l[7] >> 30;
#pragma unroll
        for (int k = 7; k >= 1; k--) ex.l[k] = (ex.l[k] << 2) | (ex.l[k - 1] >> 30);
        ex.l[0] <<= 2;
        const u256 m = d == 1u ? base : (d == 2u ? b2 : b3);
        const u256 p = mul256(r, m);
        r = sel256(d, p, r);
    }
    return r;
}


}  // namespace pf
