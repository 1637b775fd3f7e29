// pf_seed.cpp — libpflower.so: constraint-directed hint models (include/pf_lower.h,
// pfl_hints).  The native form of mythril_amd/seed.py (Seeder), decision for decision: the
// same backward propagation of the roots' desires (values / bit masks / intervals through
// concat, extract, extensions, shifts and divisions by constants, logic, add / sub /
// odd-constant mul, not, neg), the same ordered choices for ite / or / and / xor / compares
// with the same snapshot-and-retry discipline, the same repair rounds — so the hint values
// are identical (tests/test_native_seed.py).  Values are 256-bit (4 x u64 limbs); interval
// bounds that can leave [0, 2^256) (c - 1, lo + c, 2^w - c, signed bounds) are 320-bit
// two's-complement.  Host code, no HIP.
#include <cstdint>
#include <cstring>

#include <string>
#include <vector>

#include "../../include/pf_bytecode.h"
#include "../../include/pf_lower.h"

namespace {

// ---- 256-bit unsigned --------------------------------------------------------------------
struct U {
    uint64_t w[4] = {0, 0, 0, 0};
    static U from32(const uint32_t* p) {
        U r;
        for (int i = 0; i < 4; i++) r.w[i] = (uint64_t)p[2 * i] | ((uint64_t)p[2 * i + 1] << 32);
        return r;
    }
    static U of(uint64_t v) {
        U r;
        r.w[0] = v;
        return r;
    }
    void to32(uint32_t* p) const {
        for (int i = 0; i < 4; i++) {
            p[2 * i] = (uint32_t)w[i];
            p[2 * i + 1] = (uint32_t)(w[i] >> 32);
        }
    }
    bool zero() const { return !(w[0] | w[1] | w[2] | w[3]); }
    bool operator==(const U& o) const { return w[0] == o.w[0] && w[1] == o.w[1] && w[2] == o.w[2] && w[3] == o.w[3]; }
    bool operator!=(const U& o) const { return !(*this == o); }
};

int cmp(const U& a, const U& b) {
    for (int i = 3; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}
bool lt(const U& a, const U& b) { return cmp(a, b) < 0; }
bool le(const U& a, const U& b) { return cmp(a, b) <= 0; }
U uand(const U& a, const U& b) { U r; for (int i = 0; i < 4; i++) r.w[i] = a.w[i] & b.w[i]; return r; }
U uor(const U& a, const U& b) { U r; for (int i = 0; i < 4; i++) r.w[i] = a.w[i] | b.w[i]; return r; }
U uxor(const U& a, const U& b) { U r; for (int i = 0; i < 4; i++) r.w[i] = a.w[i] ^ b.w[i]; return r; }
U unot(const U& a) { U r; for (int i = 0; i < 4; i++) r.w[i] = ~a.w[i]; return r; }
U add(const U& a, const U& b, uint64_t* carry = nullptr) {
    U r;
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (unsigned __int128)a.w[i] + b.w[i];
        r.w[i] = (uint64_t)c;
        c >>= 64;
    }
    if (carry) *carry = (uint64_t)c;
    return r;
}
U sub(const U& a, const U& b) {
    U r;
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
        const uint64_t x = a.w[i], y = b.w[i];
        const uint64_t d = x - y - br;
        br = (x < y) || (x - y < br);
        r.w[i] = d;
    }
    return r;
}
U neg(const U& a) { return sub(U(), a); }
U shl(const U& a, unsigned k) {
    U r;
    if (k >= 256) return r;
    const unsigned q = k / 64, s = k % 64;
    for (int i = 3; i >= 0; i--) {
        const int j = i - (int)q;
        uint64_t v = 0;
        if (j >= 0) {
            v = a.w[j] << s;
            if (s && j >= 1) v |= a.w[j - 1] >> (64 - s);
        }
        r.w[i] = v;
    }
    return r;
}
U shr(const U& a, unsigned k) {
    U r;
    if (k >= 256) return r;
    const unsigned q = k / 64, s = k % 64;
    for (int i = 0; i < 4; i++) {
        const unsigned j = i + q;
        uint64_t v = 0;
        if (j < 4) {
            v = a.w[j] >> s;
            if (s && j + 1 < 4) v |= a.w[j + 1] << (64 - s);
        }
        r.w[i] = v;
    }
    return r;
}
U mask_slow(unsigned w) {
    if (w >= 256) return unot(U());
    return sub(shl(U::of(1), w), U::of(1));
}
struct MaskTable {
    U m[257];
    MaskTable() {
        for (unsigned w = 0; w <= 256; w++) m[w] = mask_slow(w);
    }
};
const U& mask(unsigned w) {  // 2^w - 1
    static const MaskTable t;
    return t.m[w >= 256 ? 256 : w];
}
U mw(const U& a, unsigned w) { return uand(a, mask(w)); }
unsigned bitlen(const U& a) {
    for (int i = 3; i >= 0; i--)
        if (a.w[i]) return 64 * i + 64 - __builtin_clzll(a.w[i]);
    return 0;
}
bool bit(const U& a, unsigned k) { return k < 256 && ((a.w[k / 64] >> (k % 64)) & 1u); }
// full 512-bit product (lo, hi)
void mul_full(const U& a, const U& b, U* lo, U* hi) {
    uint64_t r[8] = {0};
    for (int i = 0; i < 4; i++) {
        unsigned __int128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (unsigned __int128)a.w[i] * b.w[j] + r[i + j];
            r[i + j] = (uint64_t)c;
            c >>= 64;
        }
        r[i + 4] = (uint64_t)c;
    }
    for (int i = 0; i < 4; i++) {
        lo->w[i] = r[i];
        hi->w[i] = r[i + 4];
    }
}
U mul(const U& a, const U& b) {
    U lo, hi;
    mul_full(a, b, &lo, &hi);
    return lo;
}
void divmod(const U& a, const U& b, U* q, U* r) {  // b != 0
    if (lt(a, b)) {
        *q = U();
        *r = a;
        return;
    }
    if (!(b.w[1] | b.w[2] | b.w[3])) {  // one-limb divisor: 128/64 steps
        const uint64_t d = b.w[0];
        U Q;
        unsigned __int128 rem = 0;
        for (int i = 3; i >= 0; i--) {
            const unsigned __int128 cur = (rem << 64) | a.w[i];
            Q.w[i] = (uint64_t)(cur / d);
            rem = cur % d;
        }
        *q = Q;
        *r = U::of((uint64_t)rem);
        return;
    }
    // restoring division from the first quotient bit that can be set (the bits of a above
    // it are below b)
    const int k0 = (int)bitlen(a) - (int)bitlen(b);
    U Q, R = shr(a, (unsigned)k0 + 1u);
    for (int k = k0; k >= 0; k--) {
        R = shl(R, 1);
        if (bit(a, (unsigned)k)) R.w[0] |= 1;
        if (!lt(R, b)) {
            R = sub(R, b);
            Q.w[k / 64] |= 1ull << (k % 64);
        }
    }
    *q = Q;
    *r = R;
}
U powmod(U a, const U& e, unsigned w) {  // a^e mod 2^w
    U r = U::of(1);
    const unsigned n = bitlen(e);
    for (unsigned k = 0; k < n; k++) {
        if (bit(e, k)) r = mul(r, a);
        a = mul(a, a);
    }
    return mw(r, w);
}
bool negw(const U& a, unsigned w) { return w >= 1 && bit(a, w - 1); }
U absw(const U& a, unsigned w) { return negw(a, w) ? mw(neg(a), w) : a; }

uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)PF_PHILOX_M0 * c[0], p1 = (uint64_t)PF_PHILOX_M1 * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1,
                       n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += PF_PHILOX_W0;
        k1 += PF_PHILOX_W1;
    }
}
U uf_hash(const U& x, uint32_t salt) {  // PF_W_HASH
    uint32_t xs[8];
    x.to32(xs);
    uint32_t h[4] = {xs[0], xs[1], xs[2], xs[3]};
    philox(h, salt, PF_HASH_K1A);
    uint32_t g[4] = {xs[4] ^ h[0], xs[5] ^ h[1], xs[6] ^ h[2], xs[7] ^ h[3]};
    philox(g, salt, PF_HASH_K1B);
    uint32_t o[8] = {h[0], h[1], h[2], h[3], g[0], g[1], g[2], g[3]};
    return U::from32(o);
}

// ---- 320-bit two's complement for interval bounds ----------------------------------------
struct S {
    U lo;
    int64_t hi = 0;  // value = hi * 2^256 + lo
    static S of(const U& u) { S s; s.lo = u; return s; }
    static S pow2(unsigned k) {  // 2^k, k <= 256
        S s;
        if (k >= 256) s.hi = 1; else s.lo = shl(U::of(1), k);
        return s;
    }
};
S sadd(const S& a, const S& b) {
    S r;
    uint64_t c;
    r.lo = add(a.lo, b.lo, &c);
    r.hi = a.hi + b.hi + (int64_t)c;
    return r;
}
S sneg(const S& a) {
    S r;
    r.lo = neg(a.lo);
    r.hi = -a.hi - (a.lo.zero() ? 0 : 1);
    return r;
}
S ssub(const S& a, const S& b) { return sadd(a, sneg(b)); }
S ssmall(int64_t v) { S s; if (v >= 0) s.lo = U::of((uint64_t)v); else s = sneg(S::of(U::of((uint64_t)(-v)))); return s; }
int scmp(const S& a, const S& b) {
    if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
    return cmp(a.lo, b.lo);
}
S smax(const S& a, const S& b) { return scmp(a, b) >= 0 ? a : b; }
S smin(const S& a, const S& b) { return scmp(a, b) <= 0 ? a : b; }
S sgn(const U& x, unsigned w) {  // x as a signed w-bit value
    return negw(x, w) ? ssub(S::of(x), S::pow2(w)) : S::of(x);
}

struct Conflict {};

struct Node {
    uint32_t kind, width, nargs, args[3], aux, is_bool;
};
bool is_leaf(uint32_t k) { return k >= PFL_K_VAR && k <= PFL_K_BVAR; }

// Adjacency lists in compressed-row form: row r is idx[off[r] .. off[r + 1]) — two allocations
// for the whole DAG where a vector per node cost one each (the hint solver runs per bucket,
// and a single query's lowering spent ~16 % of its samples in the allocator)
struct Csr {
    std::vector<int> off, idx;
    struct Row {
        const int *b, *e;
        const int* begin() const { return b; }
        const int* end() const { return e; }
    };
    Row operator[](size_t r) const { return Row{idx.data() + off[r], idx.data() + off[r + 1]}; }
};

class Seeder {
   public:
    static constexpr int MAX_CHOICES = 4096;
    static constexpr int REPAIR_ROUNDS = 4;

    Seeder(const Node* nodes, size_t nn, const U* pool, const uint32_t* widths, size_t nv,
           const U* soft)
        : N(nodes), nn(nn), pool(pool), vw(widths, widths + nv), soft(soft, soft + nv), nv(nv),
          has_bits(nv, 0), bits_v(nv), bits_m(nv), has_rng(nv, 0), rng_lo(nv), rng_hi(nv),
          memo(nn), have(nn, 0), hv(nn, -1) {
        // two passes per list: counts, then each row filled in node order (the order the
        // per-node vectors had)
        users.off.assign(nn + 1, 0);
        leaf.off.assign(nv + 1, 0);
        auto each_user = [&](auto&& f) {
            for (size_t i = 0; i < nn; i++) {
                const Node& n = N[i];
                for (uint32_t k = 0; k < n.nargs; k++) {
                    bool dup = false;
                    for (uint32_t j = 0; j < k; j++) dup |= n.args[j] == n.args[k];
                    if (!dup) f(n.args[k], (int)i);
                }
            }
        };
        each_user([&](uint32_t a, int) { users.off[a + 1]++; });
        for (size_t i = 0; i < nn; i++)
            if (N[i].kind == PFL_K_VAR || N[i].kind == PFL_K_BVAR) leaf.off[N[i].aux + 1]++;
        for (size_t r = 0; r < nn; r++) users.off[r + 1] += users.off[r];
        for (size_t r = 0; r < nv; r++) leaf.off[r + 1] += leaf.off[r];
        users.idx.resize(users.off[nn]);
        leaf.idx.resize(leaf.off[nv]);
        std::vector<int> fill(users.off.begin(), users.off.end() - 1);
        each_user([&](uint32_t a, int i) { users.idx[fill[a]++] = i; });
        fill.assign(leaf.off.begin(), leaf.off.end() - 1);
        for (size_t i = 0; i < nn; i++)
            if (N[i].kind == PFL_K_VAR || N[i].kind == PFL_K_BVAR) leaf.idx[fill[N[i].aux]++] = (int)i;
    }

    std::vector<U> run(const uint32_t* roots, size_t n_roots, int* n_sat) {
        std::vector<int> rs;
        for (size_t i = 0; i < n_roots; i++) {
            bool seen = false;
            for (int r : rs) seen |= r == (int)roots[i];
            if (!seen) rs.push_back((int)roots[i]);
        }
        for (int r : rs) try_([&] { want_bool(r, true); });
        drain();
        for (int round = 0; round < REPAIR_ROUNDS; round++) {
            std::vector<int> bad;
            for (int r : rs)
                if (!truth(r)) bad.push_back(r);
            if (bad.empty()) break;
            force = true;
            for (int r : bad) {
                try {
                    want_bool(r, true);
                    drain();
                } catch (const Conflict&) {
                }
            }
            force = false;
        }
        std::vector<U> out(nv);
        for (size_t v = 0; v < nv; v++) out[v] = value_of_var((int)v);
        *n_sat = 0;
        for (int r : rs) *n_sat += truth(r) ? 1 : 0;
        return out;
    }

   private:
    const Node* N;
    size_t nn;
    const U* pool;
    std::vector<uint32_t> vw;
    std::vector<U> soft;
    size_t nv;
    // hint state: bits (value, known mask) and unsigned interval per variable
    std::vector<char> has_bits;
    std::vector<U> bits_v, bits_m;
    std::vector<char> has_rng;
    std::vector<U> rng_lo, rng_hi;
    // undo journal: (kind 0 = bits / 1 = rng, var, had, old a, old b)
    struct J {
        int kind, v;
        char had;
        U a, b;
    };
    std::vector<J> journal;
    std::vector<std::pair<int, bool>> queue;
    size_t qhead = 0;
    bool force = false;
    std::vector<U> memo;
    std::vector<char> have;
    Csr users, leaf;
    std::vector<signed char> hv;                      // has_var memo: -1 unknown
    std::vector<int> ev_stack, ch_stack, hv_stack;    // scratch (none of these recurse)
    std::vector<int> rs_leaves, rs_stack;

    // ---- evaluation under the current hint model -------------------------------------
    U value_of_var(int v) {
        const unsigned w = vw[v];
        const U M = mask(w);
        const U val = has_bits[v] ? bits_v[v] : U(), msk = has_bits[v] ? bits_m[v] : U();
        U x = uand(uor(uand(soft[v], unot(msk)), val), M);
        if (has_rng[v] && !(le(rng_lo[v], x) && le(x, rng_hi[v]))) {
            if (msk.zero()) {
                x = rng_lo[v];
            } else {
                U y = uand(val, M);
                if (lt(y, rng_lo[v])) {
                    const U fr = uand(unot(msk), M);
                    y = uand(uor(y, uand(rng_lo[v], fr)), M);
                }
                if (le(rng_lo[v], y) && le(y, rng_hi[v])) x = y;
            }
        }
        return x;
    }

    bool truth(int n) { return !ev(n).zero(); }

    const U& ev(int n) {
        if (have[n]) return memo[n];
        std::vector<int>& stack = ev_stack;
        stack.assign(1, n);
        while (!stack.empty()) {
            const int i = stack.back();
            if (have[i]) {
                stack.pop_back();
                continue;
            }
            const Node& nd = N[i];
            bool pend = false;
            for (uint32_t k = 0; k < nd.nargs; k++)
                if (!have[nd.args[k]]) {
                    stack.push_back((int)nd.args[k]);
                    pend = true;
                }
            if (pend) continue;
            stack.pop_back();
            memo[i] = ev1(nd);
            have[i] = 1;
        }
        return memo[n];
    }

    U ev1(const Node& nd) {
        const uint32_t k = nd.kind;
        const unsigned w = nd.width;
        auto A = [&](int j) -> const U& { return memo[nd.args[j]]; };
        auto B = [](bool b) { return U::of(b ? 1 : 0); };
        switch (k) {
            case PFL_K_VAR: return value_of_var((int)nd.aux);
            case PFL_K_CONST: return mw(pool[nd.aux], w);
            case PFL_K_BCONST: return B(nd.aux != 0);
            case PFL_K_BVAR: return B(value_of_var((int)nd.aux).w[0] & 1);
            case PF_W_ADD: return mw(add(A(0), A(1)), w);
            case PF_W_SUB: return mw(sub(A(0), A(1)), w);
            case PF_W_MUL: return mw(mul(A(0), A(1)), w);
            case PF_W_UDIV: {
                if (A(1).zero()) return mask(w);
                U q, r;
                divmod(A(0), A(1), &q, &r);
                return mw(q, w);
            }
            case PF_W_UREM: {
                if (A(1).zero()) return mw(A(0), w);
                U q, r;
                divmod(A(0), A(1), &q, &r);
                return mw(r, w);
            }
            case PF_W_SDIV: {
                const bool na = negw(A(0), w), nb = negw(A(1), w);
                if (A(1).zero()) return na ? U::of(1) : mask(w);
                U q, r;
                divmod(absw(A(0), w), absw(A(1), w), &q, &r);
                return mw(na == nb ? q : neg(q), w);
            }
            case PF_W_SREM: {
                if (A(1).zero()) return mw(A(0), w);
                const bool na = negw(A(0), w);
                U q, r;
                divmod(absw(A(0), w), absw(A(1), w), &q, &r);
                return mw(na ? neg(r) : r, w);
            }
            case PF_W_SMOD: {  // Python floor mod of the signed values: sign of the divisor
                if (A(1).zero()) return mw(A(0), w);
                const bool na = negw(A(0), w), nb = negw(A(1), w);
                const U mb = absw(A(1), w);
                U q, r;
                divmod(absw(A(0), w), mb, &q, &r);
                if (r.zero()) return U();
                U res;
                if (!na && !nb) res = r;
                else if (na && !nb) res = sub(mb, r);
                else if (!na && nb) res = neg(sub(mb, r));
                else res = neg(r);
                return mw(res, w);
            }
            case PF_W_AND: return mw(uand(A(0), A(1)), w);
            case PF_W_OR: return mw(uor(A(0), A(1)), w);
            case PF_W_XOR: return mw(uxor(A(0), A(1)), w);
            case PF_W_SHL: return (lt(A(1), U::of(w))) ? mw(shl(A(0), (unsigned)A(1).w[0]), w) : U();
            case PF_W_LSHR: return (lt(A(1), U::of(w))) ? mw(shr(A(0), (unsigned)A(1).w[0]), w) : U();
            case PF_W_ASHR: {
                const bool na = negw(A(0), w);
                if (!lt(A(1), U::of(w))) return na ? mask(w) : U();
                const unsigned s = (unsigned)A(1).w[0];
                U r = shr(A(0), s);
                if (na) r = uor(r, uand(mask(w), unot(mask(w - s))));
                return mw(r, w);
            }
            case PF_W_EXP: return powmod(A(0), A(1), w);
            case PF_W_NOT: return mw(unot(A(0)), w);
            case PF_W_NEG: return mw(neg(A(0)), w);
            case PF_W_MOV: return mw(A(0), w);
            case PF_W_EXTRACT: return mw(shr(A(0), nd.aux), w);
            case PF_W_CONCAT: return mw(uor(shl(A(0), nd.aux), A(1)), w);
            case PF_W_SEXT: {
                const U x = mw(A(0), nd.aux);
                return mw(negw(x, nd.aux) ? sub(x, shl(U::of(1), nd.aux)) : x, w);
            }
            case PF_W_ITE: return A(0).zero() ? A(2) : A(1);
            case PF_W_HASH: return mw(uf_hash(A(0), nd.aux), w);
            case PF_B_AND: return B(!A(0).zero() && !A(1).zero());
            case PF_B_OR: return B(!A(0).zero() || !A(1).zero());
            case PF_B_XOR: return B(A(0).zero() != A(1).zero());
            case PF_B_NOT: return B(A(0).zero());
            case PF_B_ITE: return A(0).zero() ? A(2) : A(1);
            case PF_B_EQ: return B(A(0) == A(1));
            case PF_B_ULT: return B(lt(A(0), A(1)));
            case PF_B_ULE: return B(le(A(0), A(1)));
            case PF_B_SLT: return B(scmp(sgn(A(0), w), sgn(A(1), w)) < 0);
            case PF_B_SLE: return B(scmp(sgn(A(0), w), sgn(A(1), w)) <= 0);
            case PF_B_UADD_NOOVF: {
                uint64_t c;
                const U s = add(A(0), A(1), &c);
                return B(!c && le(s, mask(w)));
            }
            case PF_B_UMUL_NOOVF: {
                U lo, hi;
                mul_full(A(0), A(1), &lo, &hi);
                return B(hi.zero() && le(lo, mask(w)));
            }
            default: throw Conflict{};  // cannot evaluate: the caller's try absorbs it
        }
    }

    void changed(int v) {
        std::vector<int>& stack = ch_stack;
        stack.clear();
        for (int i : leaf[v])
            if (have[i]) stack.push_back(i);
        while (!stack.empty()) {
            const int i = stack.back();
            stack.pop_back();
            have[i] = 0;
            for (int u : users[i])
                if (have[u]) stack.push_back(u);
        }
    }

    // ---- variable-level desires ----------------------------------------------------------
    void set_bits(int v, U val, U msk) {
        const unsigned w = vw[v];
        msk = mw(msk, w);
        val = uand(val, msk);
        if (msk.zero()) return;
        U ov = has_bits[v] ? bits_v[v] : U(), om = has_bits[v] ? bits_m[v] : U();
        const U om0 = om;
        if (!uand(uand(uxor(ov, val), om), msk).zero()) {
            if (!force) throw Conflict{};
            ov = uand(ov, unot(msk));
        }
        const U nvv = uor(uand(ov, unot(msk)), val), nm = uor(om0, msk);
        if (!(nvv == ov && nm == om0)) {
            journal.push_back({0, v, has_bits[v], bits_v[v], bits_m[v]});
            has_bits[v] = 1;
            bits_v[v] = nvv;
            bits_m[v] = nm;
            changed(v);
        }
    }

    void set_range(int v, const U& lo, const U& hi) {
        const U olo = has_rng[v] ? rng_lo[v] : U(), ohi = has_rng[v] ? rng_hi[v] : mask(vw[v]);
        U nlo = lt(olo, lo) ? lo : olo, nhi = lt(hi, ohi) ? hi : ohi;
        if (lt(nhi, nlo)) {
            if (!force) throw Conflict{};
            nlo = lo;
            nhi = hi;
        }
        if (!(nlo == olo && nhi == ohi) || !has_rng[v]) {
            journal.push_back({1, v, has_rng[v], rng_lo[v], rng_hi[v]});
            has_rng[v] = 1;
            rng_lo[v] = nlo;
            rng_hi[v] = nhi;
            changed(v);
        }
    }

    bool cst(int n, U* out) const {
        const Node& nd = N[n];
        if (nd.kind != PFL_K_CONST) return false;
        *out = mw(pool[nd.aux], nd.width);
        return true;
    }

    // ---- W desires: node value has bits `val` on `msk` -----------------------------------
    void want_val(int n, U val, U msk) {
        const Node& nd = N[n];
        const uint32_t k = nd.kind;
        const unsigned w = nd.width;
        msk = mw(msk, w);
        val = uand(val, msk);
        if (msk.zero()) return;
        if (k == PFL_K_VAR) {
            set_bits((int)nd.aux, val, msk);
            return;
        }
        if (k == PFL_K_CONST) {
            if (!uand(uxor(mw(pool[nd.aux], w), val), msk).zero()) throw Conflict{};
            return;
        }
        const uint32_t* a = nd.args;
        const bool full = msk == mask(w);
        if (k == PF_W_CONCAT) {
            const unsigned wl = nd.aux;
            want_val(a[1], mw(val, wl), mw(msk, wl));
            want_val(a[0], shr(val, wl), shr(msk, wl));
        } else if (k == PF_W_EXTRACT) {
            want_val(a[0], shl(val, nd.aux), shl(msk, nd.aux));
        } else if (k == PF_W_MOV || k == PF_W_SEXT) {
            const unsigned ws = k == PF_W_MOV ? N[a[0]].width : nd.aux;
            if (k == PF_W_MOV && !shr(val, ws).zero()) throw Conflict{};
            want_val(a[0], mw(val, ws), mw(msk, ws));
        } else if (k == PF_W_ITE) {
            choice_w(n, val, msk);
        } else if (k == PF_W_NOT) {
            want_val(a[0], unot(val), msk);
        } else if (k == PF_W_NEG && full) {
            want_val(a[0], neg(val), msk);
        } else if (k == PF_W_LSHR || k == PF_W_SHL || k == PF_W_UDIV) {
            U c;
            if (!cst(a[1], &c)) {
                if (k == PF_W_UDIV) return;
                // a shift by a computed amount (a window lookup's byte, to_dag._window):
                // propagate through the amount's current value
                c = ev((int)a[1]);
            }
            unsigned cs;
            if (k == PF_W_UDIV) {
                if (c.zero()) return;
                if (!uand(c, sub(c, U::of(1))).zero()) {  // general divisor
                    if (full) want_val(a[0], mul(val, c), mask(w));
                    return;
                }
                cs = bitlen(c) - 1;
            } else {
                if (!lt(c, U::of(w))) {
                    if (!uand(val, msk).zero()) throw Conflict{};
                    return;
                }
                cs = (unsigned)c.w[0];
            }
            if (cs >= w) {
                if (!uand(val, msk).zero()) throw Conflict{};
                return;
            }
            if (k == PF_W_SHL) {
                if (!uand(uand(val, msk), mask(cs)).zero()) throw Conflict{};
                want_val(a[0], shr(val, cs), shr(msk, cs));
            } else {
                if (!shr(uand(val, msk), w - cs).zero()) throw Conflict{};
                want_val(a[0], shl(val, cs), shl(msk, cs));
            }
        } else if (k == PF_W_AND || k == PF_W_OR || k == PF_W_XOR || k == PF_W_ADD || k == PF_W_SUB ||
                   k == PF_W_MUL) {
            U c0, c1;
            const bool h0 = cst(a[0], &c0), h1 = cst(a[1], &c1);
            if (!h0 && !h1) {
                eval_propagate(n, val, msk);
                return;
            }
            const int x = h1 ? (int)a[0] : (int)a[1];
            const U c = h1 ? c1 : c0;
            if (k == PF_W_AND) {
                if (!uand(uand(val, unot(c)), msk).zero()) throw Conflict{};
                want_val(x, uand(val, c), uand(msk, c));
            } else if (k == PF_W_OR) {
                if (!uand(uand(unot(val), c), msk).zero()) throw Conflict{};
                want_val(x, uand(val, unot(c)), uand(msk, unot(c)));
            } else if (k == PF_W_XOR) {
                want_val(x, uxor(val, c), msk);
            } else {
                if (!uand(add(msk, U::of(1)), msk).zero()) return;  // msk is not a run of low bits
                const unsigned wl = bitlen(msk);
                if (k == PF_W_ADD) {
                    want_val(x, sub(val, c), msk);
                } else if (k == PF_W_SUB) {
                    want_val(x, x == (int)a[0] ? add(val, c) : sub(c, val), msk);
                } else if (c.w[0] & 1) {  // odd constant: multiply by its inverse mod 2^wl
                    U inv = U::of(1);      // Newton: inv <- inv * (2 - c * inv), 9 steps to 2^256
                    for (int it = 0; it < 9; it++) inv = mul(inv, sub(U::of(2), mul(c, inv)));
                    want_val(x, mul(val, mw(inv, wl)), msk);
                }
            }
        }
    }

    void eval_propagate(int n, const U& val, const U& msk) {
        const Node& nd = N[n];
        if (msk != mask(nd.width)) return;
        const uint32_t k = nd.kind;
        const int x = (int)nd.args[0], y = (int)nd.args[1];
        const unsigned w = nd.width;
        const int tg[2] = {x, y}, ot[2] = {y, x};
        for (int p = 0; p < 2; p++) {
            const int tgt = tg[p], other = ot[p];
            const U o = ev(other);
            U need;
            if (k == PF_W_ADD) need = sub(val, o);
            else if (k == PF_W_XOR) need = uxor(val, o);
            else if (k == PF_W_SUB) need = tgt == x ? add(val, o) : sub(o, val);
            else return;
            if (has_var(tgt)) {
                const U nm = mw(need, w);
                try_([&] { want_val(tgt, nm, mask(w)); });
                if (ev(n) == val) return;
            }
        }
    }

    // does the sub-DAG under n reach a variable leaf?  (memoised: the DAG is immutable)
    bool has_var(int n) {
        if (hv[n] >= 0) return hv[n] != 0;
        std::vector<int>& stack = hv_stack;
        stack.assign(1, n);
        while (!stack.empty()) {
            const int i = stack.back();
            if (hv[i] >= 0) {
                stack.pop_back();
                continue;
            }
            const Node& nd = N[i];
            if (nd.kind == PFL_K_VAR || nd.kind == PFL_K_BVAR) {
                hv[i] = 1;
                stack.pop_back();
                continue;
            }
            bool pend = false;
            for (uint32_t k = 0; k < nd.nargs; k++)
                if (hv[nd.args[k]] < 0) {
                    stack.push_back((int)nd.args[k]);
                    pend = true;
                }
            if (pend) continue;
            stack.pop_back();
            char r = 0;
            for (uint32_t k = 0; k < nd.nargs; k++) r |= hv[nd.args[k]];
            hv[i] = r;
        }
        return hv[n] != 0;
    }

    // ---- W interval desires -------------------------------------------------------------
    void want_range(int n, S lo, S hi) {
        const Node& nd = N[n];
        const unsigned w = nd.width;
        const S M = S::of(mask(w));
        lo = smax(lo, S());
        hi = smin(hi, M);
        if (scmp(lo, hi) > 0) throw Conflict{};
        const U cur = ev(n);
        if (nd.kind == PFL_K_VAR) {
            set_range((int)nd.aux, lo.lo, hi.lo);
            return;
        }
        if (scmp(lo, S::of(cur)) <= 0 && scmp(S::of(cur), hi) <= 0) return;
        if (nd.kind == PFL_K_CONST) throw Conflict{};
        if (nd.kind == PF_W_MOV) {
            const unsigned ws = N[nd.args[0]].width;
            want_range((int)nd.args[0], lo, smin(hi, S::of(mask(ws))));
            return;
        }
        if (nd.kind == PF_W_ITE) {
            const int c = (int)nd.args[0], a = (int)nd.args[1], b = (int)nd.args[2];
            alternatives([&] { want_bool(c, true); want_range(a, lo, hi); },
                         [&] { want_bool(c, false); want_range(b, lo, hi); });
            return;
        }
        if (nd.kind == PF_W_ADD || nd.kind == PF_W_SUB) {
            U c1;
            if (cst((int)nd.args[1], &c1)) {
                const S d = nd.kind == PF_W_SUB ? S::of(c1) : sneg(S::of(c1));
                const S nlo = sadd(lo, d), nhi = sadd(hi, d);
                if (scmp(S(), nlo) <= 0 && scmp(nhi, M) <= 0) {
                    want_range((int)nd.args[0], nlo, nhi);
                    return;
                }
            }
        }
        want_val(n, lo.lo, mask(w));  // a representative point
    }

    void want_srange(int n, S slo, S shi) {
        const unsigned w = N[n].width;
        slo = smax(slo, sneg(S::pow2(w - 1)));
        shi = smin(shi, ssub(S::pow2(w - 1), ssmall(1)));
        if (scmp(slo, shi) > 0) throw Conflict{};
        if (scmp(slo, S()) >= 0) {
            want_range(n, slo, shi);
        } else if (scmp(shi, S()) < 0) {
            want_range(n, sadd(slo, S::pow2(w)), sadd(shi, S::pow2(w)));
        } else {
            alternatives([&] { want_range(n, S(), shi); },
                         [&] { want_range(n, sadd(slo, S::pow2(w)), S::of(mask(w))); });
        }
    }

    // ---- Bool desires -------------------------------------------------------------------
    void want_bool(int n, bool v) {
        const Node& nd = N[n];
        const uint32_t k = nd.kind;
        if (k == PFL_K_BCONST) {
            if ((nd.aux != 0) != v) throw Conflict{};
            return;
        }
        if (k == PFL_K_BVAR) {
            set_bits((int)nd.aux, U::of(v ? 1 : 0), U::of(1));
            return;
        }
        const uint32_t* a = nd.args;
        if (k == PF_B_NOT) {
            want_bool((int)a[0], !v);
        } else if ((k == PF_B_AND && v) || (k == PF_B_OR && !v)) {
            want_bool((int)a[0], v);
            want_bool((int)a[1], v);
        } else if (k == PF_B_AND || k == PF_B_OR || k == PF_B_XOR || k == PF_B_ITE) {
            queue.push_back({n, v});
        } else if (k == PF_B_EQ) {
            want_eq(n, v);
        } else if (k == PF_B_ULT || k == PF_B_ULE || k == PF_B_SLT || k == PF_B_SLE) {
            want_cmp(n, v);
        } else if ((k == PF_B_UADD_NOOVF || k == PF_B_UMUL_NOOVF) && !v) {
            U c;
            if (cst((int)a[1], &c) && !c.zero()) {
                S need;
                if (k == PF_B_UADD_NOOVF) {
                    need = ssub(S::pow2(nd.width), S::of(c));
                } else {  // ceil(2^w / c) = floor((2^w - 1) / c) + 1
                    U q, r;
                    divmod(mask(nd.width), c, &q, &r);
                    need = sadd(S::of(q), ssmall(1));
                }
                want_range((int)a[0], need, S::of(mask(nd.width)));
            }
        }
    }

    void want_eq(int n, bool v) {
        const Node& nd = N[n];
        const int x = (int)nd.args[0], y = (int)nd.args[1];
        const unsigned w = nd.width;
        U cx, cy;
        const bool hx = cst(x, &cx), hy = cst(y, &cy);
        if (v) {
            if (hy) want_val(x, cy, mask(w));
            else if (hx) want_val(y, cx, mask(w));
            else queue.push_back({n, v});
            return;
        }
        if (!truth(n)) return;
        if (hy || hx) {
            const int t = hy ? x : y;
            const U c = hy ? cy : cx;
            const Node& tn = N[t];
            if (tn.kind == PF_W_ITE) {
                const int cc = (int)tn.args[0], p = (int)tn.args[1], q = (int)tn.args[2];
                U cp, cq;
                const bool hp = cst(p, &cp), hq = cst(q, &cq);
                if (hp && cp != c) {
                    want_bool(cc, true);
                    return;
                }
                if (hq && cq != c) {
                    want_bool(cc, false);
                    return;
                }
            }
            queue.push_back({n, v});
        }
    }

    static uint32_t flip(uint32_t k) {
        switch (k) {
            case PF_B_ULT: return PF_B_ULE;
            case PF_B_ULE: return PF_B_ULT;
            case PF_B_SLT: return PF_B_SLE;
            default: return PF_B_SLT;
        }
    }

    void want_cmp(int n, bool v) {
        const Node& nd = N[n];
        uint32_t k = nd.kind;
        int x = (int)nd.args[0], y = (int)nd.args[1];
        const unsigned w = nd.width;
        if (!v) {
            k = flip(k);
            std::swap(x, y);
        }
        const int strict = (k == PF_B_ULT || k == PF_B_SLT) ? 1 : 0;
        const bool sg = k == PF_B_SLT || k == PF_B_SLE;
        U cx, cy;
        const bool hx = cst(x, &cx), hy = cst(y, &cy);
        if (!hx && !hy) {
            queue.push_back({n, v});
            return;
        }
        if (sg) {
            const S top = ssub(S::pow2(w - 1), ssmall(1)), bot = sneg(S::pow2(w - 1));
            if (hy) want_srange(x, bot, ssub(sgn(cy, w), ssmall(strict)));
            else want_srange(y, sadd(sgn(cx, w), ssmall(strict)), top);
        } else {
            if (hy) want_range(x, S(), ssub(S::of(cy), ssmall(strict)));
            else want_range(y, sadd(S::of(cx), ssmall(strict)), S::of(mask(w)));
        }
    }

    // ---- choices ------------------------------------------------------------------------
    void choice_w(int n, const U& val, const U& msk) {
        const Node& nd = N[n];
        const int c = (int)nd.args[0], a = (int)nd.args[1], b = (int)nd.args[2];
        U ca, cb;
        const bool ha = cst(a, &ca), hb = cst(b, &cb);
        auto alt_a = [&] { want_bool(c, true); want_val(a, val, msk); };
        auto alt_b = [&] { want_bool(c, false); want_val(b, val, msk); };
        const bool cur = truth(c);
        bool a_first;
        if (uand(uxor(ev(n), val), msk).zero()) {
            a_first = cur;
        } else if (hb && uand(uxor(cb, val), msk).zero() && !(ha && uand(uxor(ca, val), msk).zero())) {
            a_first = false;
        } else if (ha && uand(uxor(ca, val), msk).zero()) {
            a_first = true;
        } else {
            a_first = cur;
        }
        if (a_first) alternatives(alt_a, alt_b);
        else alternatives(alt_b, alt_a);
    }

    struct Snap {
        size_t jlen, qlen;
    };
    Snap snapshot() const { return {journal.size(), queue.size() - qhead}; }

    void restore(const Snap& s) {
        while (journal.size() > s.jlen) {
            const J& j = journal.back();
            if (j.kind == 0) {
                has_bits[j.v] = j.had;
                bits_v[j.v] = j.a;
                bits_m[j.v] = j.b;
            } else {
                has_rng[j.v] = j.had;
                rng_lo[j.v] = j.a;
                rng_hi[j.v] = j.b;
            }
            changed(j.v);
            journal.pop_back();
        }
        queue.resize(qhead + s.qlen);
    }

    template <typename F>
    bool try_(F&& fn) {
        const Snap s = snapshot();
        try {
            fn();
            return true;
        } catch (const Conflict&) {
            restore(s);
            return false;
        }
    }

    // First alternative that applies without a conflict wins; under `force` the first one is
    // applied regardless.  Variadic (no std::function / vector allocation per choice).
    template <typename F0, typename... Fs>
    void alternatives(F0&& f0, Fs&&... fs) {
        if (try_(f0)) return;
        if ((try_(fs) || ...)) return;
        if (force) {
            f0();
            return;
        }
        throw Conflict{};
    }

    void resolve(int n, bool v) {
        if (truth(n) == v) return;
        const Node& nd = N[n];
        uint32_t k = nd.kind;
        const uint32_t* a = nd.args;
        if (k == PF_B_AND || k == PF_B_OR) {
            // one conjunct / disjunct over the flattened tree, in left-to-right order
            std::vector<int>&leaves = rs_leaves, &stack = rs_stack;  // resolve() does not nest
            leaves.clear();
            stack.assign(1, n);
            while (!stack.empty()) {
                const int i = stack.back();
                stack.pop_back();
                if (N[i].kind == k) {
                    for (int j = (int)N[i].nargs - 1; j >= 0; j--) stack.push_back((int)N[i].args[j]);
                } else {
                    leaves.push_back(i);
                }
            }
            for (int x : leaves)
                if (try_([&] { want_bool(x, v); })) return;
            if (force && !leaves.empty()) {
                want_bool(leaves[0], v);
                return;
            }
            throw Conflict{};
        } else if (k == PF_B_XOR) {
            alternatives([&] { want_bool((int)a[0], v); want_bool((int)a[1], false); },
                         [&] { want_bool((int)a[0], !v); want_bool((int)a[1], true); });
        } else if (k == PF_B_ITE) {
            const int c = (int)a[0], p = (int)a[1], q = (int)a[2];
            alternatives([&] { want_bool(c, true); want_bool(p, v); },
                         [&] { want_bool(c, false); want_bool(q, v); });
        } else if (k == PF_B_EQ) {
            const int x = (int)a[0], y = (int)a[1];
            const unsigned w = nd.width;
            if (v) {
                want_eqw(x, y, 0);
            } else {
                const U vx = ev(x), vy = ev(y);
                alternatives([&] { want_val(x, uxor(vx, U::of(1)), mask(w)); },
                             [&] { want_val(y, uxor(vy, U::of(1)), mask(w)); },
                             [&] { want_val(x, uxor(vx, shl(U::of(1), w - 1)), mask(w)); });
            }
        } else if (k == PF_B_ULT || k == PF_B_ULE || k == PF_B_SLT || k == PF_B_SLE) {
            int x = (int)a[0], y = (int)a[1];
            const unsigned w = nd.width;
            U vx = ev(x), vy = ev(y);
            if (!v) {
                k = flip(k);
                std::swap(x, y);
                std::swap(vx, vy);
            }
            const int strict = (k == PF_B_ULT || k == PF_B_SLT) ? 1 : 0;
            if (k == PF_B_ULT || k == PF_B_ULE) {
                alternatives([&] { want_range(x, S(), ssub(S::of(vy), ssmall(strict))); },
                             [&] { want_range(y, sadd(S::of(vx), ssmall(strict)), S::of(mask(w))); });
            } else {
                alternatives([&] { want_srange(x, sneg(S::pow2(w - 1)), ssub(sgn(vy, w), ssmall(strict))); },
                             [&] { want_srange(y, sadd(sgn(vx, w), ssmall(strict)),
                                               ssub(S::pow2(w - 1), ssmall(1))); });
            }
        } else {
            want_bool(n, v);
        }
    }

    void want_eqw(int x, int y, int depth) {
        if (x == y || ev(x) == ev(y)) return;
        const unsigned w = N[x].width;
        U cx, cy;
        const bool hx = cst(x, &cx), hy = cst(y, &cy);
        if (hy) {
            want_val(x, cy, mask(w));
            return;
        }
        if (hx) {
            want_val(y, cx, mask(w));
            return;
        }
        const Node &nx = N[x], &ny = N[y];
        const bool structural = depth < 8 && nx.kind == ny.kind && nx.aux == ny.aux &&
                                nx.width == ny.width && nx.nargs == ny.nargs &&
                                nx.kind != PFL_K_VAR && nx.kind != PFL_K_CONST;
        auto by_args = [&] {
            for (uint32_t i = 0; i < nx.nargs; i++) {
                const int a = (int)nx.args[i], b = (int)ny.args[i];
                if (a == b) continue;
                if (N[a].is_bool) {
                    U dummy;
                    if (!cst(b, &dummy)) want_bool(a, truth(b));
                } else {
                    want_eqw(a, b, depth + 1);
                }
            }
        };
        const U vx = ev(x), vy = ev(y);
        auto x_to_y = [&] { want_val(x, vy, mask(w)); };
        auto y_to_x = [&] { want_val(y, vx, mask(w)); };
        if (structural) alternatives(by_args, x_to_y, y_to_x);
        else alternatives(x_to_y, y_to_x);
    }

    void drain() {
        int steps = 0;
        while (queue.size() > qhead && steps < MAX_CHOICES) {
            const auto item = queue[qhead++];
            steps++;
            try_([&] { resolve(item.first, item.second); });
        }
    }
};

}  // namespace

extern "C" int pfl_hints(const uint32_t* nodes, size_t n_nodes, const uint32_t* const_pool,
                         size_t n_pool, const uint32_t* roots, size_t n_roots,
                         const uint32_t* var_widths, size_t n_vars, const uint32_t* soft,
                         uint32_t* hints_out, int* n_sat_out) {
    const Node* N = reinterpret_cast<const Node*>(nodes);
    for (size_t i = 0; i < n_nodes; ++i) {
        const Node& n = N[i];
        if (n.nargs > 3) return -1;
        for (uint32_t k = 0; k < n.nargs; ++k)
            if (n.args[k] >= i) return -1;
        if ((n.kind == PFL_K_VAR || n.kind == PFL_K_BVAR) && n.aux >= n_vars) return -1;
        if (n.kind == PFL_K_CONST && n.aux >= n_pool) return -1;
    }
    for (size_t r = 0; r < n_roots; ++r)
        if (roots[r] >= n_nodes) return -1;
    std::vector<U> pool(n_pool), sv(n_vars);
    for (size_t i = 0; i < n_pool; i++) pool[i] = U::from32(const_pool + 8 * i);
    for (size_t i = 0; i < n_vars; i++) sv[i] = U::from32(soft + 8 * i);
    Seeder s(N, n_nodes, pool.data(), var_widths, n_vars, sv.data());
    int n_sat = 0;
    const std::vector<U> out = s.run(roots, n_roots, &n_sat);
    for (size_t v = 0; v < n_vars; v++) out[v].to32(hints_out + 8 * v);
    if (n_sat_out) *n_sat_out = n_sat;
    return 0;
}
