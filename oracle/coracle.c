/*
 * ORACLE — test infrastructure only (checker and bench.py's cpu_baseline leg).
 *
 * C restatement of oracle/pyoracle.py: SMT-LIB2 / z3 bit-vector semantics of the bytecode in
 * include/pf_bytecode.h (what z3's model.eval(..., model_completion=True) computes for the terms
 * built by mythril/laser/smt/bitvec.py:63-246, bitvec_helper.py:31-245, bool.py:98-134), and the
 * candidate-generator contract of include/pf_bytecode.h.  The SAT criterion is
 * ModelCache.check_quick_sat's (mythril/support/support_utils.py:57-71): the conjunction
 * evaluates to true.  4 x 64-bit limbs with unsigned __int128 intermediates — an independent
 * arithmetic formulation from the kernel's 8 x 32-bit limbs.  OpenMP over candidates.
 * Nothing in mythril_amd/ links or calls this file.
 */
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t w[4]; } v256;

static v256 Z(void) { v256 r = {{0, 0, 0, 0}}; return r; }
static v256 ONES(void) { v256 r = {{~0ull, ~0ull, ~0ull, ~0ull}}; return r; }
static v256 mask_of(uint32_t w) {
    v256 r = Z();
    for (int i = 0; i < 4; i++) {
        uint32_t lo = 64u * i;
        r.w[i] = w >= lo + 64 ? ~0ull : (w <= lo ? 0ull : ((1ull << (w - lo)) - 1ull));
    }
    return r;
}
static v256 andv(v256 a, v256 b) { for (int i = 0; i < 4; i++) a.w[i] &= b.w[i]; return a; }
static v256 orv(v256 a, v256 b) { for (int i = 0; i < 4; i++) a.w[i] |= b.w[i]; return a; }
static v256 xorv(v256 a, v256 b) { for (int i = 0; i < 4; i++) a.w[i] ^= b.w[i]; return a; }
static v256 notv(v256 a) { for (int i = 0; i < 4; i++) a.w[i] = ~a.w[i]; return a; }
static int iszero(v256 a) { return !(a.w[0] | a.w[1] | a.w[2] | a.w[3]); }
static int eqv(v256 a, v256 b) { return iszero(xorv(a, b)); }
static v256 addv(v256 a, v256 b, int* carry) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) { c += (u128)a.w[i] + b.w[i]; a.w[i] = (uint64_t)c; c >>= 64; }
    if (carry) *carry = (int)c;
    return a;
}
static v256 subv(v256 a, v256 b) { return addv(addv(a, notv(b), 0), (v256){{1, 0, 0, 0}}, 0); }
static v256 negv(v256 a) { return subv(Z(), a); }
static int ultv(v256 a, v256 b) {
    for (int i = 3; i >= 0; i--) if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return 0;
}
static v256 mulv(v256 a, v256 b, int* overflow) {
    uint64_t r[8] = {0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a.w[i] * b.w[j] + r[i + j];
            r[i + j] = (uint64_t)c;
            c >>= 64;
        }
        r[i + 4] = (uint64_t)c;
    }
    if (overflow) *overflow = (r[4] | r[5] | r[6] | r[7]) != 0;
    v256 o = {{r[0], r[1], r[2], r[3]}};
    return o;
}
static int bitlen(v256 a) {
    for (int i = 3; i >= 0; i--) if (a.w[i]) return 64 * i + 64 - __builtin_clzll(a.w[i]);
    return 0;
}
static v256 shlv(v256 a, uint32_t s) {
    if (s >= 256) return Z();
    v256 r = Z();
    uint32_t q = s / 64, b = s % 64;
    for (int i = 3; i >= (int)q; i--) {
        uint64_t v = a.w[i - q] << b;
        if (b && i - (int)q - 1 >= 0) v |= a.w[i - q - 1] >> (64 - b);
        r.w[i] = v;
    }
    return r;
}
static v256 shrv(v256 a, uint32_t s, uint64_t fill) {
    if (s >= 256) { v256 f = {{fill, fill, fill, fill}}; return f; }
    v256 r;
    uint32_t q = s / 64, b = s % 64;
    for (int i = 0; i < 4; i++) {
        uint64_t lo = (i + q < 4) ? a.w[i + q] : fill;
        uint64_t hi = (i + q + 1 < 4) ? a.w[i + q + 1] : fill;
        r.w[i] = b ? ((lo >> b) | (hi << (64 - b))) : lo;
    }
    return r;
}
/* restoring division; z3: x / 0 = ~0, x % 0 = x */
static void udivremv(v256 a, v256 b, v256* q, v256* r) {
    if (iszero(b)) { *q = ONES(); *r = a; return; }
    int la = bitlen(a), lb = bitlen(b);
    v256 qq = Z(), rr = a;
    for (int i = la - lb; i >= 0; i--) {
        v256 d = shlv(b, (uint32_t)i);
        if (!ultv(rr, d)) { rr = subv(rr, d); qq.w[i / 64] |= 1ull << (i % 64); }
    }
    *q = qq; *r = rr;
}
static int msb(v256 a, uint32_t w) { return (int)((a.w[(w - 1) / 64] >> ((w - 1) % 64)) & 1); }
static v256 sext(v256 a, uint32_t wsrc, uint32_t w) {
    if (msb(a, wsrc)) a = orv(a, andv(notv(mask_of(wsrc)), mask_of(w)));
    return andv(a, mask_of(w));
}
static v256 sdivfam(v256 a, v256 b, uint32_t w, int which) {
    v256 M = mask_of(w);
    int sa = msb(a, w), sb = msb(b, w);
    v256 ua = sa ? andv(negv(a), M) : a, ub = sb ? andv(negv(b), M) : b, q, r;
    udivremv(ua, ub, &q, &r);
    q = andv(q, M);
    if (which == 0) return (sa ^ sb) ? andv(negv(q), M) : q;
    if (which == 1) return sa ? andv(negv(r), M) : r;
    if (iszero(r) || (!sa && !sb)) return r;
    if (sa && !sb) return andv(addv(negv(r), b, 0), M);
    if (!sa && sb) return andv(addv(r, b, 0), M);
    return andv(negv(r), M);
}
static v256 expv(v256 a, v256 e, uint32_t w) {
    v256 r = {{1, 0, 0, 0}};
    for (uint32_t i = 0; i < w; i++) {
        if ((e.w[i / 64] >> (i % 64)) & 1) r = mulv(r, a, 0);
        a = mulv(a, a, 0);
    }
    return andv(r, mask_of(w));
}
static int ge_w(v256 b, uint32_t w) { return b.w[1] || b.w[2] || b.w[3] || b.w[0] >= w; }

/* ---- Philox4x32-10 and the candidate generator ------------------------------------ */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; i++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
static v256 from32(const uint32_t* p) {
    v256 r;
    for (int i = 0; i < 4; i++) r.w[i] = (uint64_t)p[2 * i] | ((uint64_t)p[2 * i + 1] << 32);
    return r;
}
static v256 pow2(uint32_t k) { v256 r = Z(); r.w[k / 64] = 1ull << (k % 64); return r; }
static v256 pow2m1(uint32_t k) { return subv(pow2(k), (v256){{1, 0, 0, 0}}); }

typedef struct {
    const uint32_t *code, *consts, *schema, *parents;
    uint32_t n_ins, n_const, n_vars, seed;
} SetV;

static v256 gen(const SetV* S, uint32_t v, uint32_t cand, uint64_t gseed) {
    const uint32_t* sc = S->schema + 4 * v;
    uint32_t kind = sc[0] & 0xff, w = (sc[0] >> 8) & 0x3ff, h0 = sc[1], h1 = sc[2], slot = sc[3];
    v256 M = mask_of(w);
    if (cand == 0 && slot != 0xffffffffu) return andv(from32(S->parents + 8 * (size_t)slot), M);
    uint32_t k0 = (uint32_t)gseed ^ S->seed, k1 = (uint32_t)(gseed >> 32);
    uint32_t r[8], m[4];
    uint32_t c0[4] = {cand, v, 0, 0}, c1[4] = {cand, v, 1, 0}, c2[4] = {cand, v, 2, 0};
    philox(c0, k0, k1); philox(c1, k0, k1); philox(c2, k0, k1);
    memcpy(r, c0, 16); memcpy(r + 4, c1, 16); memcpy(m, c2, 16);
    if (slot != 0xffffffffu && (cand & 1u) && (m[3] & ((4u << ((cand >> 1) & 3u)) - 1u)) != 0u)
        return andv(from32(S->parents + 8 * (size_t)slot), M); /* neighbourhood candidate */
    v256 rv = from32(r), out;
    if (kind == 2) { /* keccak slot */
        v256 k = Z();
        k.w[0] = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
        k.w[1] = ((uint64_t)r[2] | ((uint64_t)r[3] << 32)) & ((1ull << 53) - 1);
        return andv(addv(from32(S->consts + 8 * (size_t)h0), shlv(k, 6), 0), M);
    }
    if (kind == 3) {
        out = Z();
        if ((m[0] & 16u) && h0 >= 4u && h0 != 0xffffffffu) out.w[0] = 4u + 32u * (r[1] % ((h0 - 4u) / 32u + 1u));
        else out.w[0] = (h0 == 0xffffffffu) ? r[0] : r[0] % (h0 + 1);
        return andv(out, M);
    }
    if (kind == 6 && (m[0] & 16u)) return Z(); /* call value: 0 in half the candidates */
    if (kind == 4) { out = Z(); out.w[0] = r[0] & 1; return out; }
    if (kind == 1 && (m[1] % 4) < h1) return andv(from32(S->consts + 8 * (size_t)(h0 + m[1] % 4)), M);
    uint32_t wk = (h0 >> 8) & 0xfffu, ws = h0 >> 20;
    if (wk == 0) { wk = S->n_const; ws = 0; }
    if (kind == 5 && wk) { /* calldata byte: one constant per (candidate, ABI word) */
        uint32_t u = cand ^ k0 ^ (h1 * 0x9E3779B9u);
        u ^= u >> 16; u *= 0x7feb352du; u ^= u >> 15; u *= 0x846ca68bu; u ^= u >> 16;
        if (u & 1u) {
            const uint32_t sh = h0 & 0xffu;
            v256 c = from32(S->consts + 8 * (size_t)(ws + (u >> 1) % wk));
            uint32_t d = u >> 30;
            if (d == 1) c = addv(c, (v256){{1, 0, 0, 0}}, 0);
            if (d == 2) c = addv(c, ONES(), 0);
            out = Z();
            out.w[0] = (c.w[(sh >> 6) & 3u] >> (sh & 63u)) & 0xffu;
            return andv(out, M);
        }
    }
    uint32_t sel = m[0] & 15;
    if (sel <= 4) out = rv;
    else if (sel <= 8) {
        uint32_t j = m[1] % 12, k = m[2] % w;
        v256 one = {{1, 0, 0, 0}};
        switch (j) {
            case 0: case 1: case 2: case 3: out = Z(); out.w[0] = j; break;
            case 4: out = M; break;
            case 5: out = subv(M, one); break;
            case 6: out = pow2(w - 1); break;
            case 7: out = pow2m1(w - 1); break;
            case 8: out = pow2(k); break;
            case 9: out = pow2m1(k); break;
            case 10: out = addv(pow2(k), one, 0); break;
            default: out = pow2m1(160); break;
        }
    } else if (sel <= 11) {
        if (S->n_const) {
            out = from32(S->consts + 8 * (size_t)(m[1] % S->n_const));
            uint32_t d = m[2] % 3;
            if (d == 1) out = addv(out, (v256){{1, 0, 0, 0}}, 0);
            if (d == 2) out = addv(out, ONES(), 0);
        } else out = rv;
    } else if (sel <= 13) {
        if (slot != 0xffffffffu) {
            out = from32(S->parents + 8 * (size_t)slot);
            if ((m[1] & 3) == 0) out = xorv(out, pow2(m[2] % w));
        } else { out = Z(); out.w[0] = r[0] & 0xff; }
    } else { out = Z(); out.w[0] = r[0] & ((1ull << (1 + m[1] % 16)) - 1); }
    return andv(out, M);
}

/* values: optional explicit assignment [n_vars] (NULL = generate candidate cand) */
static int eval_one(const SetV* S, const v256* values, uint32_t cand, uint64_t gseed) {
    v256 W[16], SP[64]; /* SP: spill slots (PF_W_SPILL / PF_W_FILL / PF_B_SPILL / PF_B_FILL) */
    uint8_t B[32];
    memset(SP, 0, sizeof SP);
    memset(W, 0, sizeof W);
    memset(B, 0, sizeof B);
    int root = 1;
    for (uint32_t pc = 0; pc < S->n_ins; pc++) {
        const uint32_t* I = S->code + 4 * (size_t)pc;
        uint32_t op = I[0] & 0xff, w = (I[0] >> 8) & 0x3ff;
        uint32_t d = I[1] & 0xff, a = (I[1] >> 8) & 0xff, b = (I[1] >> 16) & 0xff, c = (I[1] >> 24) & 0xff;
        v256 M = mask_of(w), x = W[a & 15], y = W[b & 15], q, r;
        int ov;
        switch (op) {
            case 0: return root;
            case 1: W[d] = andv(from32(S->consts + 8 * (size_t)I[2]), M); break;
            case 2: W[d] = andv(values ? values[I[2]] : gen(S, I[2], cand, gseed), M); break;
            case 3: W[d] = andv(x, M); break;
            case 4: W[d] = andv(addv(x, y, 0), M); break;
            case 5: W[d] = andv(subv(x, y), M); break;
            case 6: W[d] = andv(mulv(x, y, 0), M); break;
            case 7: udivremv(x, y, &q, &r); W[d] = andv(q, M); break;
            case 8: udivremv(x, y, &q, &r); W[d] = andv(r, M); break;
            case 9: W[d] = sdivfam(x, y, w, 0); break;
            case 10: W[d] = sdivfam(x, y, w, 1); break;
            case 11: W[d] = sdivfam(x, y, w, 2); break;
            case 12: W[d] = andv(x, y); break;
            case 13: W[d] = orv(x, y); break;
            case 14: W[d] = xorv(x, y); break;
            case 15: W[d] = andv(notv(x), M); break;
            case 16: W[d] = andv(negv(x), M); break;
            case 17: W[d] = ge_w(y, w) ? Z() : andv(shlv(x, (uint32_t)y.w[0]), M); break;
            case 18: W[d] = ge_w(y, w) ? Z() : shrv(x, (uint32_t)y.w[0], 0); break;
            case 19: {
                v256 sx = sext(x, w, 256);
                uint64_t f = msb(x, w) ? ~0ull : 0ull;
                W[d] = andv(ge_w(y, w) ? (v256){{f, f, f, f}} : shrv(sx, (uint32_t)y.w[0], f), M);
                break;
            }
            case 20: W[d] = expv(x, y, w); break;
            case 21: W[d] = andv(shrv(x, I[2], 0), M); break;
            case 22: W[d] = andv(orv(shlv(x, I[2]), y), M); break;
            case 23: W[d] = sext(x, I[2], w); break;
            case 24: W[d] = B[c & 31] ? x : y; break;
            case 25: {
                uint32_t xs[8], h[4], g[4];
                for (int k = 0; k < 4; k++) { xs[2 * k] = (uint32_t)x.w[k]; xs[2 * k + 1] = (uint32_t)(x.w[k] >> 32); }
                memcpy(h, xs, 16);
                philox(h, I[2], 0x5BD1E995u);
                for (int k = 0; k < 4; k++) g[k] = xs[4 + k] ^ h[k];
                philox(g, I[2], 0x27D4EB2Fu);
                uint32_t o[8] = {h[0], h[1], h[2], h[3], g[0], g[1], g[2], g[3]};
                W[d] = andv(from32(o), M);
                break;
            }
            case 26: SP[I[2] & 63] = x; break;
            case 27: W[d] = andv(SP[I[2] & 63], M); break;
            case 40: B[d] = I[2] & 1; break;
            case 41: B[d] = (uint8_t)((values ? values[I[2]] : gen(S, I[2], cand, gseed)).w[0] & 1); break;
            case 42: B[d] = eqv(x, y); break;
            case 43: B[d] = ultv(x, y); break;
            case 44: B[d] = !ultv(y, x); break;
            case 45: case 46: {
                v256 sx = sext(x, w, 256), sy = sext(y, w, 256);
                sx.w[3] ^= 1ull << 63; sy.w[3] ^= 1ull << 63;
                B[d] = (op == 45) ? ultv(sx, sy) : !ultv(sy, sx);
                break;
            }
            case 47: B[d] = B[a] & B[b]; break;
            case 48: B[d] = B[a] | B[b]; break;
            case 49: B[d] = B[a] ^ B[b]; break;
            case 50: B[d] = !B[a]; break;
            case 51: B[d] = B[c] ? B[a] : B[b]; break;
            case 52: { int cy; v256 s = addv(x, y, &cy); B[d] = !cy && eqv(andv(s, M), s); break; }
            case 53: { v256 p = mulv(x, y, &ov); B[d] = !ov && eqv(andv(p, M), p); break; }
            case 54: B[d] = (uint8_t)(SP[I[2] & 63].w[0] & 1); break;
            case 55: SP[I[2] & 63] = Z(); SP[I[2] & 63].w[0] = B[a]; break;
            case 60: root &= B[a]; break;
            default: return -1;
        }
    }
    return root;
}

static SetV view(const uint32_t* code, const uint32_t* consts, const uint32_t* schema,
                 const uint32_t* parents, const uint32_t* descs, uint32_t s) {
    const uint32_t* D = descs + 8 * (size_t)s;
    SetV S = {code + 4 * (size_t)D[0], consts + 8 * (size_t)D[2], schema + 4 * (size_t)D[4],
              parents, D[1], D[3], D[5], D[6]};
    return S;
}

/* SAT flag of candidates [cand0, cand0 + n) of set s (generated) */
int co_eval_generated(const uint32_t* code, const uint32_t* consts, const uint32_t* schema,
                      const uint32_t* parents, const uint32_t* descs, uint32_t s, uint64_t gseed,
                      uint32_t cand0, uint32_t n, uint8_t* out) {
    SetV S = view(code, consts, schema, parents, descs, s);
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (uint32_t i = 0; i < n; i++) {
        int r = eval_one(&S, 0, cand0 + i, gseed);
        if (r < 0) bad = 1;
        out[i] = (uint8_t)(r > 0);
    }
    return bad ? -1 : 0;
}

/* SAT flag of explicit assignments: values [n][n_vars][8] u32 */
int co_eval_explicit(const uint32_t* code, const uint32_t* consts, const uint32_t* schema,
                     const uint32_t* parents, const uint32_t* descs, uint32_t s,
                     const uint32_t* values, uint32_t n, uint8_t* out) {
    SetV S = view(code, consts, schema, parents, descs, s);
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (uint32_t i = 0; i < n; i++) {
        v256 vals[256];
        for (uint32_t v = 0; v < S.n_vars && v < 256; v++) vals[v] = from32(values + ((size_t)i * S.n_vars + v) * 8);
        int r = eval_one(&S, vals, 0, 0);
        if (r < 0) bad = 1;
        out[i] = (uint8_t)(r > 0);
    }
    return bad ? -1 : 0;
}

/* generated values of variable v for candidates [cand0, cand0+n): out [n][8] u32 */
void co_gen_values(const uint32_t* code, const uint32_t* consts, const uint32_t* schema,
                   const uint32_t* parents, const uint32_t* descs, uint32_t s, uint32_t v,
                   uint64_t gseed, uint32_t cand0, uint32_t n, uint32_t* out) {
    SetV S = view(code, consts, schema, parents, descs, s);
    for (uint32_t i = 0; i < n; i++) {
        v256 x = gen(&S, v, cand0 + i, gseed);
        for (int k = 0; k < 4; k++) {
            out[8 * (size_t)i + 2 * k] = (uint32_t)x.w[k];
            out[8 * (size_t)i + 2 * k + 1] = (uint32_t)(x.w[k] >> 32);
        }
    }
}

/* ---- Keccak-256 (original Keccak padding 0x01..0x80, as eth_hash / support_utils.sha3,
 * mythril/support/support_utils.py:93-101) — FIPS 202 Keccak-f[1600] restated with 64-bit
 * lanes; the checker and CPU baseline for pf_keccak_*_kernel.  OpenMP over messages. */
static const uint64_t KRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int KROT[5][5] = {{0, 36, 3, 41, 18}, {1, 44, 10, 45, 2}, {62, 6, 43, 15, 61},
                               {28, 55, 25, 21, 56}, {27, 20, 39, 8, 14}}; /* [x][y] */

static uint64_t rol(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }

static void keccak_f(uint64_t A[25]) { /* A[x + 5y] */
    for (int r = 0; r < 24; r++) {
        uint64_t C[5], B[25];
        for (int x = 0; x < 5; x++) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; x++) {
            uint64_t D = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
            for (int y = 0; y < 5; y++) A[x + 5 * y] ^= D;
        }
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rol(A[x + 5 * y], KROT[x][y]);
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= KRC[r];
    }
}

static void keccak256_one(const uint8_t* p, uint64_t len, uint8_t* out) {
    uint64_t A[25];
    uint8_t blk[136];
    memset(A, 0, sizeof A);
    for (;;) {
        uint64_t take = len < 136 ? len : 136;
        memset(blk, 0, sizeof blk);
        memcpy(blk, p, take);
        int last = len < 136;
        if (last) { blk[take] ^= 0x01; blk[135] ^= 0x80; }
        for (int i = 0; i < 17; i++) {
            uint64_t lane = 0;
            for (int b = 0; b < 8; b++) lane |= (uint64_t)blk[8 * i + b] << (8 * b);
            A[i] ^= lane;
        }
        keccak_f(A);
        if (last) break;
        p += 136;
        len -= 136;
    }
    for (int i = 0; i < 4; i++)
        for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(A[i] >> (8 * b));
}

/* n fixed-length messages data[i*len .. (i+1)*len) -> out[32*i ..] */
void co_keccak256_fixed(const uint8_t* data, uint64_t len, uint64_t n, uint8_t* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) keccak256_one(data + (uint64_t)i * len, len, out + 32 * (uint64_t)i);
}
