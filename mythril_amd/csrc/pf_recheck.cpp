// pf_recheck.cpp — libpflower.so: the host re-check of a GPU witness, natively
// (include/pf_lower.h, pflt_recheck).
//
// The native form of mythril_amd/smt/interp.py:Witness.ev — the same interpretation of
// every term the lowering accepts, bit for bit: SMT-LIB2 bit-vector semantics at any width
// (z3's total division), arrays read in the lowering's lookup order (the first read of the
// array whose index evaluates equal), keccak256_<n> as the registered concrete hash or
// base_n + 64 (H(x) mod 2^117), inverses by lookup among the set's applications, Power by
// argument value, other UFs as keyed hashes (PF_W_HASH).  gpu_check runs it on every bucket
// witness before trusting it (soundness: a GPU "sat" must satisfy the terms, not only the
// program); tests/test_native_terms.py checks it against Witness.ev.  Host code, no HIP.
#include <algorithm>
#include <initializer_list>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/pf_lower.h"
#include "pf_pool.h"

namespace {

// ---- values of any width: little-endian u32 limbs, exactly ceil(w / 32) of them ----------
// A small vector: up to 512 bits in place (every value of a <= 256-bit bucket and the
// 257..512-bit chunks), wider on the heap — the evaluator makes a value per node and op, and
// a heap allocation each was most of a re-check's time.
class V {
   public:
    V() = default;
    explicit V(size_t n) : V(n, 0u) {}
    V(size_t n, uint32_t x) {
        set_size(n);
        std::fill(p_, p_ + n, x);
    }
    V(std::initializer_list<uint32_t> il) {
        set_size(il.size());
        std::copy(il.begin(), il.end(), p_);
    }
    V(const uint32_t* b, const uint32_t* e) { assign(b, e); }
    V(const V& o) { assign(o.p_, o.p_ + o.n_); }
    V(V&& o) noexcept { take(o); }
    V& operator=(const V& o) {
        if (this != &o) assign(o.p_, o.p_ + o.n_);
        return *this;
    }
    V& operator=(V&& o) noexcept {
        if (this != &o) {
            release();
            take(o);
        }
        return *this;
    }
    ~V() { release(); }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    uint32_t& operator[](size_t i) { return p_[i]; }
    const uint32_t& operator[](size_t i) const { return p_[i]; }
    uint32_t& back() { return p_[n_ - 1]; }
    const uint32_t& back() const { return p_[n_ - 1]; }
    uint32_t* data() { return p_; }
    const uint32_t* data() const { return p_; }
    uint32_t* begin() { return p_; }
    uint32_t* end() { return p_ + n_; }
    const uint32_t* begin() const { return p_; }
    const uint32_t* end() const { return p_ + n_; }
    void push_back(uint32_t x) {
        if (n_ == cap_) grow(2 * cap_);
        p_[n_++] = x;
    }
    void assign(const uint32_t* b, const uint32_t* e) {
        const size_t n = (size_t)(e - b);
        set_size(n);
        std::copy(b, e, p_);
    }
    bool operator==(const V& o) const { return n_ == o.n_ && std::equal(p_, p_ + n_, o.p_); }
    bool operator!=(const V& o) const { return !(*this == o); }
    bool operator<(const V& o) const { return std::lexicographical_compare(p_, p_ + n_, o.p_, o.p_ + o.n_); }

   private:
    static constexpr size_t N = 16;
    uint32_t buf_[N];
    uint32_t* p_ = buf_;
    size_t n_ = 0, cap_ = N;
    void set_size(size_t n) {  // contents not kept
        if (n > cap_) {
            release();
            p_ = new uint32_t[n];
            cap_ = n;
        }
        n_ = n;
    }
    void grow(size_t c) {
        uint32_t* q = new uint32_t[c];
        std::copy(p_, p_ + n_, q);
        release();
        p_ = q;
        cap_ = c;
    }
    void release() {
        if (p_ != buf_) delete[] p_;
        p_ = buf_;
        cap_ = N;
    }
    void take(V& o) {
        n_ = o.n_;
        if (o.p_ == o.buf_) {
            p_ = buf_;
            cap_ = N;
            std::copy(o.buf_, o.buf_ + o.n_, buf_);
        } else {
            p_ = o.p_;
            cap_ = o.cap_;
            o.p_ = o.buf_;
            o.cap_ = N;
        }
        o.n_ = 0;
    }
};

size_t nl_of(uint32_t w) { return (w + 31) / 32; }

V vzero(uint32_t w) { return V(nl_of(w), 0u); }

V vmask(const V& a, uint32_t w) {
    V r(nl_of(w), 0u);
    for (size_t i = 0; i < r.size() && i < a.size(); i++) r[i] = a[i];
    if (w % 32 && !r.empty()) r.back() &= (1u << (w % 32)) - 1u;
    return r;
}

bool vbit(const V& a, uint32_t i) { return i / 32 < a.size() && ((a[i / 32] >> (i % 32)) & 1u); }

bool vis_zero(const V& a) {
    for (uint32_t x : a)
        if (x) return false;
    return true;
}

int vcmp(const V& a, const V& b) {  // unsigned
    const size_t n = std::max(a.size(), b.size());
    for (size_t i = n; i-- > 0;) {
        const uint32_t x = i < a.size() ? a[i] : 0u, y = i < b.size() ? b[i] : 0u;
        if (x != y) return x < y ? -1 : 1;
    }
    return 0;
}

V vadd(const V& a, const V& b, uint32_t w) {
    V r(nl_of(w), 0u);
    uint64_t c = 0;
    for (size_t i = 0; i < r.size(); i++) {
        c += (uint64_t)(i < a.size() ? a[i] : 0u) + (i < b.size() ? b[i] : 0u);
        r[i] = (uint32_t)c;
        c >>= 32;
    }
    return vmask(r, w);
}

V vnot(const V& a, uint32_t w) {
    V r(nl_of(w), 0u);
    for (size_t i = 0; i < r.size(); i++) r[i] = ~(i < a.size() ? a[i] : 0u);
    return vmask(r, w);
}

V vneg(const V& a, uint32_t w) {
    V one = vzero(w);
    if (!one.empty()) one[0] = 1;
    return vadd(vnot(a, w), one, w);
}

V vsub(const V& a, const V& b, uint32_t w) { return vadd(a, vneg(b, w), w); }

V vmul(const V& a, const V& b, uint32_t w) {
    const size_t n = nl_of(w);
    V r(n, 0u);
    for (size_t i = 0; i < n && i < a.size(); i++) {
        uint64_t c = 0;
        for (size_t j = 0; i + j < n; j++) {
            c += (uint64_t)a[i] * (j < b.size() ? b[j] : 0u) + r[i + j];
            r[i + j] = (uint32_t)c;
            c >>= 32;
        }
    }
    return vmask(r, w);
}

V vshl(const V& a, uint64_t s, uint32_t w) {
    V r = vzero(w);
    if (s >= w) return r;
    const size_t q = (size_t)(s / 32), b = (size_t)(s % 32);
    for (size_t i = r.size(); i-- > q;) {
        const size_t j = i - q;
        uint32_t x = j < a.size() ? a[j] << b : 0u;
        if (b && j >= 1 && j - 1 < a.size()) x |= a[j - 1] >> (32 - b);
        r[i] = x;
    }
    return vmask(r, w);
}

V vlshr(const V& a, uint64_t s, uint32_t w) {
    V r = vzero(w);
    if (s >= w) return r;
    const V m = vmask(a, w);
    const size_t q = (size_t)(s / 32), b = (size_t)(s % 32);
    for (size_t i = 0; i + q < m.size(); i++) {
        uint32_t x = m[i + q] >> b;
        if (b && i + q + 1 < m.size()) x |= m[i + q + 1] << (32 - b);
        r[i] = x;
    }
    return r;
}

bool vneg_sign(const V& a, uint32_t w) { return w && vbit(a, w - 1); }

V vashr(const V& a, uint64_t s, uint32_t w) {
    const bool neg = vneg_sign(a, w);
    if (s >= w) return neg ? vnot(vzero(w), w) : vzero(w);
    V r = vlshr(a, s, w);
    if (neg)
        for (uint32_t i = w - (uint32_t)s; i < w; i++) r[i / 32] |= 1u << (i % 32);
    return r;
}

void vdivmod(const V& a, const V& b, uint32_t w, V* q, V* r) {  // unsigned, b != 0
    const V A = vmask(a, w);
    *q = vzero(w);
    if (vcmp(A, b) < 0) {  // quotient 0
        *r = A;
        return;
    }
    bool wide_b = false;
    for (size_t i = 1; i < b.size(); i++) wide_b |= b[i] != 0u;
    if (!wide_b) {  // one-limb divisor: 64/32 steps from the top limb
        const uint64_t d = b[0];
        uint64_t rem = 0;
        for (size_t i = A.size(); i-- > 0;) {
            const uint64_t cur = (rem << 32) | A[i];
            (*q)[i] = (uint32_t)(cur / d);
            rem = cur % d;
        }
        *r = vzero(w);
        if (!r->empty()) (*r)[0] = (uint32_t)rem;
        return;
    }
    // restoring division in place, from A's top bit (the remainder stays below 2b)
    const size_t n = A.size() + 1;
    V R(n, 0u);
    uint32_t top = 0;
    for (size_t i = A.size(); i-- > 0;)
        if (A[i]) {
            top = 32u * (uint32_t)i + 32u - (uint32_t)__builtin_clz(A[i]);
            break;
        }
    for (uint32_t i = top; i-- > 0;) {
        for (size_t k = n; k-- > 1;) R[k] = (R[k] << 1) | (R[k - 1] >> 31);
        R[0] = (R[0] << 1) | ((A[i / 32] >> (i % 32)) & 1u);
        if (vcmp(R, b) >= 0) {
            uint64_t br = 0;
            for (size_t k = 0; k < n; k++) {
                const uint64_t x = (uint64_t)R[k] - (k < b.size() ? b[k] : 0u) - br;
                R[k] = (uint32_t)x;
                br = (x >> 63) & 1u;
            }
            (*q)[i / 32] |= 1u << (i % 32);
        }
    }
    *r = vmask(R, w);
}

uint64_t vsmall(const V& a, bool* big) {  // value if it fits 64 bits
    *big = false;
    for (size_t i = 2; i < a.size(); i++)
        if (a[i]) *big = true;
    return (uint64_t)(a.size() > 0 ? a[0] : 0u) | ((uint64_t)(a.size() > 1 ? a[1] : 0u) << 32);
}

V vabs(const V& a, uint32_t w) { return vneg_sign(a, w) ? vneg(a, w) : vmask(a, w); }

V binop(uint32_t op, const V& a, const V& b, uint32_t w) {  // terms._FOLD2
    switch (op) {
        case PFLT_BVADD: return vadd(a, b, w);
        case PFLT_BVSUB: return vsub(a, b, w);
        case PFLT_BVMUL: return vmul(a, b, w);
        case PFLT_BVAND: case PFLT_BVOR: case PFLT_BVXOR: {
            V r = vzero(w);
            for (size_t i = 0; i < r.size(); i++) {
                const uint32_t x = i < a.size() ? a[i] : 0u, y = i < b.size() ? b[i] : 0u;
                r[i] = op == PFLT_BVAND ? (x & y) : (op == PFLT_BVOR ? (x | y) : (x ^ y));
            }
            return r;
        }
        case PFLT_BVSHL: case PFLT_BVLSHR: case PFLT_BVASHR: {
            bool big;
            const uint64_t s = vsmall(b, &big);
            const uint64_t sh = big ? UINT64_MAX : s;
            return op == PFLT_BVSHL ? vshl(a, sh, w) : (op == PFLT_BVLSHR ? vlshr(a, sh, w) : vashr(a, sh, w));
        }
        case PFLT_BVUDIV: case PFLT_BVUREM: {
            if (vis_zero(b)) return op == PFLT_BVUDIV ? vnot(vzero(w), w) : vmask(a, w);
            V q, r;
            vdivmod(a, b, w, &q, &r);
            return op == PFLT_BVUDIV ? q : r;
        }
        case PFLT_BVSDIV: {
            const bool sa = vneg_sign(a, w), sb = vneg_sign(b, w);
            if (vis_zero(b)) {
                V one = vzero(w);
                one[0] = 1;
                return sa ? one : vnot(vzero(w), w);
            }
            V q, r;
            vdivmod(vabs(a, w), vabs(b, w), w, &q, &r);
            return sa == sb ? q : vneg(q, w);
        }
        case PFLT_BVSREM: {
            if (vis_zero(b)) return vmask(a, w);
            V q, r;
            vdivmod(vabs(a, w), vabs(b, w), w, &q, &r);
            return vneg_sign(a, w) ? vneg(r, w) : r;
        }
        case PFLT_BVSMOD: {  // Python's floor modulo of the signed values: sign of b
            if (vis_zero(b)) return vmask(a, w);
            V q, r;
            vdivmod(vabs(a, w), vabs(b, w), w, &q, &r);
            const bool sa = vneg_sign(a, w), sb = vneg_sign(b, w);
            if (vis_zero(r)) return r;
            V m = sa ? vneg(r, w) : r;  // truncated remainder, sign of a
            if (sa != sb) m = vadd(m, vmask(b, w), w);
            return m;
        }
        case PFLT_BVEXP: {
            V r = vzero(w), x = vmask(a, w);
            if (!r.empty()) r[0] = 1;
            if (w == 0) return r;
            const size_t eb = b.size() * 32;
            for (size_t i = 0; i < eb; i++) {
                if (vbit(b, (uint32_t)i)) r = vmul(r, x, w);
                x = vmul(x, x, w);
            }
            return vmask(r, w);
        }
        default: return vzero(w);
    }
}

bool cmpop(uint32_t op, const V& a, const V& b, uint32_t w) {  // terms._CMP
    switch (op) {
        case PFLT_BVULT: return vcmp(a, b) < 0;
        case PFLT_BVULE: return vcmp(a, b) <= 0;
        case PFLT_BVSLT: case PFLT_BVSLE: {
            const bool sa = vneg_sign(a, w), sb = vneg_sign(b, w);
            if (sa != sb) return sa;
            const int c = vcmp(a, b);
            return op == PFLT_BVSLT ? c < 0 : c <= 0;
        }
        case PFLT_BVUADD_NOOVF: {
            const V s = vadd(a, b, w + 1);
            return !vbit(s, w);
        }
        case PFLT_BVUMUL_NOOVF: {
            const V p = vmul(a, b, 2 * w + 1);
            for (uint32_t i = w; i < 2 * w + 1; i++)
                if (vbit(p, i)) return false;
            return true;
        }
        default: return false;
    }
}

// ---- PF_W_HASH (include/pf_bytecode.h) -----------------------------------------------------
void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

V uf_hash(const V& x8, uint32_t salt) {
    uint32_t xs[8];
    for (int i = 0; i < 8; i++) xs[i] = i < (int)x8.size() ? x8[i] : 0u;
    uint32_t h[4] = {xs[0], xs[1], xs[2], xs[3]};
    philox(h, salt, 0x5BD1E995u);
    uint32_t g[4] = {xs[4] ^ h[0], xs[5] ^ h[1], xs[6] ^ h[2], xs[7] ^ h[3]};
    philox(g, salt, 0x27D4EB2Fu);
    return V{h[0], h[1], h[2], h[3], g[0], g[1], g[2], g[3]};
}

uint32_t crc32_str(const std::string& s) {
    uint32_t c = 0xffffffffu;
    for (unsigned char ch : s) {
        c ^= ch;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return c ^ 0xffffffffu;
}

// chunks of a w-bit value: 256-bit pieces, LSB first (interp._chunks)
std::vector<V> chunks256(const V& v, uint32_t w) {
    std::vector<V> out;
    uint32_t off = 0;
    while (off < w) {
        const uint32_t cw = std::min<uint32_t>(256, w - off);
        out.push_back(vmask(vlshr(v, off, std::max<uint32_t>(w, 1)), cw));
        off += 256;
    }
    return out;
}

struct KSpec {
    bool has_lo;
    V base;
    std::vector<std::pair<V, V>> concrete;
};

struct Ev {
    // the term store is read through the public accessors of pf_terms.cpp
    void* st;
    std::unordered_map<std::string, V> vars;
    std::unordered_map<std::string, bool> bools;
    std::map<std::pair<uint32_t, uint32_t>, V> read_vals;  // (array id, index id) -> value
    std::unordered_map<uint32_t, V> app_vals;              // apply term id -> value
    std::map<std::string, std::vector<std::pair<uint32_t, uint32_t>>> reads;  // array name -> (arr, idx)
    std::vector<uint32_t> uf_apps;
    std::map<uint32_t, KSpec> kspecs;
    std::unordered_map<uint32_t, V> memo;

    pflt_term_view T(uint32_t id) const {
        pflt_term_view t;
        pflt_view(st, id, &t);
        return t;
    }
    std::string name_of(const pflt_term_view& t) const { return std::string(t.name ? t.name : ""); }
    uint32_t width(const pflt_term_view& t) const { return t.sortk == 1 ? t.w1 : 0; }

    static V of_limbs(const uint32_t* l, uint32_t n, uint32_t w) { return vmask(V(l, l + n), w); }

    static bool keccak_name(const std::string& f, uint32_t* n, bool* inv) {
        static const char pre[] = "keccak256_";
        if (f.compare(0, sizeof(pre) - 1, pre) != 0) return false;
        size_t i = sizeof(pre) - 1, j = i;
        while (j < f.size() && f[j] >= '0' && f[j] <= '9') j++;
        if (j == i) return false;
        *n = (uint32_t)strtoul(f.c_str() + i, nullptr, 10);
        if (j == f.size()) { *inv = false; return true; }
        if (f.compare(j, std::string::npos, "-1") == 0) { *inv = true; return true; }
        return false;
    }

    V keccak(uint32_t n, const V& x) {
        auto it = kspecs.find(n);
        if (it != kspecs.end())
            for (const auto& c : it->second.concrete)
                if (vcmp(c.first, vmask(x, n)) == 0) return vmask(c.second, 256);
        V h;
        bool first = true;
        const uint32_t salt = crc32_str("keccak256_" + std::to_string(n));
        for (const V& c : chunks256(x, n)) {
            V in = first ? vmask(c, 256) : binop(PFLT_BVXOR, h, vmask(c, 256), 256);
            h = uf_hash(in, salt);
            first = false;
        }
        if (it == kspecs.end() || !it->second.has_lo) return h;
        V k = vmask(h, 117);
        return vadd(it->second.base, vshl(k, 6, 256), 256);
    }

    V keccak_inv(uint32_t n, const V& y, uint32_t term) {
        size_t upto = uf_apps.size();
        for (size_t i = 0; i < uf_apps.size(); i++)
            if (uf_apps[i] == term) { upto = i; break; }
        const std::string fname = "keccak256_" + std::to_string(n), iname = fname + "-1";
        for (size_t i = 0; i < upto; i++) {
            const pflt_term_view a = T(uf_apps[i]);
            if (name_of(a) == fname) {
                const V x = ev(a.args[0]);
                if (vcmp(keccak(n, x), y) == 0) return x;
            }
        }
        for (size_t i = 0; i < upto; i++) {
            const pflt_term_view a = T(uf_apps[i]);
            if (name_of(a) == iname && app_vals.count(uf_apps[i]) && vcmp(ev(a.args[0]), y) == 0)
                return app_vals[uf_apps[i]];
        }
        auto it = app_vals.find(term);
        return it != app_vals.end() ? it->second : vzero(n);
    }

    V power(uint32_t t, const pflt_term_view& tv) {
        const V b = ev(tv.args[0]), e = ev(tv.args[1]);
        for (uint32_t app : uf_apps) {
            const pflt_term_view a = T(app);
            if (name_of(a) != "Power" || a.nargs != 2) continue;
            const pflt_term_view a0 = T(a.args[0]), a1 = T(a.args[1]);
            if (a0.op == PFLT_BV && a1.op == PFLT_BV &&
                vcmp(of_limbs(a0.limbs, a0.nlimbs, 256), b) == 0 && vcmp(of_limbs(a1.limbs, a1.nlimbs, 256), e) == 0)
                return binop(PFLT_BVEXP, b, e, 256);
        }
        V c256 = vzero(256);
        c256[0] = 256;
        if (vcmp(b, c256) == 0) {
            const uint32_t em = e.empty() ? 0u : (e[0] % 32u);
            return vshl(V{1u}, 8u * em, 256);
        }
        for (uint32_t app : uf_apps) {
            const pflt_term_view a = T(app);
            if (name_of(a) != "Power" || a.nargs != 2 || !app_vals.count(app)) continue;
            if (vcmp(ev(a.args[0]), b) == 0 && vcmp(ev(a.args[1]), e) == 0) return app_vals[app];
        }
        (void)t;
        V one = vzero(256);
        one[0] = 1;
        return one;
    }

    V apply(uint32_t t, const pflt_term_view& tv) {
        const std::string f = name_of(tv);
        uint32_t n;
        bool inv;
        if (keccak_name(f, &n, &inv)) {
            const pflt_term_view a = T(tv.args[0]);
            uint32_t an;
            bool ainv;
            if (inv && a.op == PFLT_APPLY && keccak_name(name_of(a), &an, &ainv) && !ainv && an == n)
                return ev(a.args[0]);
            const V x = ev(tv.args[0]);
            return inv ? keccak_inv(n, x, t) : keccak(n, x);
        }
        if (f == "Power" && tv.nargs == 2 && width(tv) == 256) return power(t, tv);
        V h;
        bool first = true;
        const uint32_t salt = crc32_str(f);
        for (uint32_t i = 0; i < tv.nargs; i++) {
            const pflt_term_view a = T(tv.args[i]);
            for (const V& c : chunks256(ev(tv.args[i]), width(a))) {
                V in = first ? vmask(c, 256) : binop(PFLT_BVXOR, h, vmask(c, 256), 256);
                h = uf_hash(in, salt);
                first = false;
            }
        }
        return vmask(h, width(tv));
    }

    // interp.Witness._first_table: once every index of an array has been evaluated (by the
    // scan's rules: a nested read of the same array meanwhile scans), the first read whose
    // index equals iv is a lookup — the scan's answer, as the read's own entry matches
    struct FirstTable {
        bool ok = false;
        std::map<V, V> first;  // index value (trailing zero limbs trimmed) -> value
    };
    std::unordered_map<std::string, FirstTable> tables;
    std::unordered_map<std::string, bool> building;

    static V trimmed(const V& v) {
        size_t n = v.size();
        while (n && v[n - 1] == 0) n--;
        return V(v.begin(), v.begin() + n);
    }

    const FirstTable* first_table(const std::string& name, const std::vector<std::pair<uint32_t, uint32_t>>& es,
                                  uint32_t w2) {
        auto it = tables.find(name);
        if (it != tables.end()) return it->second.ok ? &it->second : nullptr;
        if (building[name]) return nullptr;
        building[name] = true;
        FirstTable tab;
        try {
            for (const auto& e : es) {
                V key = trimmed(ev(e.second));
                if (tab.first.count(key)) continue;
                auto jt = read_vals.find(e);
                tab.first.emplace(std::move(key), jt != read_vals.end() ? jt->second : vzero(w2));
            }
            tab.ok = true;
        } catch (...) {
            tab.first.clear();
            tab.ok = false;
        }
        building[name] = false;
        auto& slot = tables[name] = std::move(tab);
        return slot.ok ? &slot : nullptr;
    }

    V array_read(uint32_t arr, uint32_t idx, const V& iv) {
        const pflt_term_view A = T(arr);
        const std::string name = name_of(A);
        auto it = reads.find(name);
        if (it == reads.end() || it->second.empty()) return vzero(A.w2);
        const auto& es = it->second;
        if (const FirstTable* tab = first_table(name, es, A.w2)) {
            auto jt = tab->first.find(trimmed(iv));
            return jt != tab->first.end() ? jt->second : vzero(A.w2);
        }
        size_t last = es.size() - 1;
        for (size_t i = 0; i < es.size(); i++)
            if (es[i].first == arr && es[i].second == idx) { last = i; break; }
        for (size_t i = 0; i <= last; i++) {
            if (vcmp(ev(es[i].second), iv) == 0) {
                auto jt = read_vals.find(es[i]);
                return jt != read_vals.end() ? jt->second : vzero(A.w2);
            }
        }
        return vzero(A.w2);
    }

    V select(uint32_t arr, const V& iv, uint32_t idx) {
        const pflt_term_view A = T(arr);
        if (A.op == PFLT_STORE) {
            if (vcmp(ev(A.args[1]), iv) == 0) return ev(A.args[2]);
            return select(A.args[0], iv, idx);
        }
        if (A.op == PFLT_K) return ev(A.args[0]);
        if (A.op == PFLT_ITE) return select(bool_of(ev(A.args[0])) ? A.args[1] : A.args[2], iv, idx);
        if (A.op == PFLT_ARRAY) return array_read(arr, idx, iv);
        throw 1;
    }

    static bool bool_of(const V& v) { return !vis_zero(v); }
    static V B(bool b) { return V{b ? 1u : 0u}; }

    // memoised: the reference stays valid (node-based map) while later terms are added
    const V& ev(uint32_t t) {
        auto it = memo.find(t);
        if (it != memo.end()) return it->second;
        V r = ev_(t);
        return memo.emplace(t, std::move(r)).first->second;
    }

    V ev_(uint32_t t) {
        const pflt_term_view tv = T(t);
        const uint32_t w = width(tv);
        switch (tv.op) {
            case PFLT_BV: return of_limbs(tv.limbs, tv.nlimbs, w);
            case PFLT_TRUE: return B(true);
            case PFLT_FALSE: return B(false);
            case PFLT_VAR: {
                auto jt = vars.find(name_of(tv));
                return jt != vars.end() ? vmask(jt->second, w) : vzero(w);
            }
            case PFLT_BVAR: {
                auto jt = bools.find(name_of(tv));
                return B(jt != bools.end() && jt->second);
            }
            case PFLT_BVNOT: return vnot(ev(tv.args[0]), w);
            case PFLT_BVNEG: return vneg(ev(tv.args[0]), w);
            case PFLT_EXTRACT: return vmask(vlshr(ev(tv.args[0]), (uint64_t)tv.i1, width(T(tv.args[0]))), w);
            case PFLT_CONCAT: {
                V v = vzero(w);
                uint32_t off = w;
                for (uint32_t i = 0; i < tv.nargs; i++) {
                    const uint32_t aw = width(T(tv.args[i]));
                    off -= aw;
                    v = binop(PFLT_BVOR, v, vshl(vmask(ev(tv.args[i]), aw), off, w), w);
                }
                return v;
            }
            case PFLT_ZERO_EXTEND: return vmask(ev(tv.args[0]), w);
            case PFLT_ITE: return bool_of(ev(tv.args[0])) ? ev(tv.args[1]) : ev(tv.args[2]);
            case PFLT_SELECT: return select(tv.args[0], ev(tv.args[1]), tv.args[1]);
            case PFLT_APPLY: return apply(t, tv);
            case PFLT_EQ: return B(vcmp(ev(tv.args[0]), ev(tv.args[1])) == 0);
            case PFLT_IFF: return B(bool_of(ev(tv.args[0])) == bool_of(ev(tv.args[1])));
            case PFLT_AND:
                for (uint32_t i = 0; i < tv.nargs; i++)
                    if (!bool_of(ev(tv.args[i]))) return B(false);
                return B(true);
            case PFLT_OR:
                for (uint32_t i = 0; i < tv.nargs; i++)
                    if (bool_of(ev(tv.args[i]))) return B(true);
                return B(false);
            case PFLT_NOT: return B(!bool_of(ev(tv.args[0])));
            case PFLT_XOR: return B(bool_of(ev(tv.args[0])) != bool_of(ev(tv.args[1])));
            default: break;
        }
        if (tv.op >= PFLT_BVADD && tv.op <= PFLT_BVEXP) return binop(tv.op, ev(tv.args[0]), ev(tv.args[1]), w);
        if (tv.op >= PFLT_BVULT && tv.op <= PFLT_BVUMUL_NOOVF) {
            const uint32_t aw = width(T(tv.args[0]));
            return B(cmpop(tv.op, ev(tv.args[0]), ev(tv.args[1]), aw));
        }
        throw 1;  // not evaluable: the caller reports "cannot evaluate"
    }
};

// registry blob: as for pflt_lower (actors first, unused here); throws on a short blob
void parse_registry(Ev& E, const uint32_t* registry, size_t n_registry) {
    size_t p = 0;
        auto take = [&]() -> uint32_t {
            if (p >= n_registry) throw 2;
            return registry[p++];
        };
        const uint32_t na = take();
        p += 8 * na;
        const uint32_t ns = take();
        for (uint32_t s = 0; s < ns; s++) {
            const uint32_t n = take();
            KSpec sp;
            sp.has_lo = take() != 0;
            V base(8);
            for (int k = 0; k < 8; k++) base[k] = take();
            sp.base = base;
            const uint32_t nc = take();
            for (uint32_t c = 0; c < nc; c++) {
                V v(nl_of(n));
                for (auto& x : v) x = take();
                V dg(8);
                for (auto& x : dg) x = take();
                sp.concrete.push_back({vmask(v, n), dg});
            }
            E.kspecs[n] = sp;
        }
}

// one part of a witness (interp.Witness.__init__): var descriptors (type, a, b, c) with values,
// its UF applications and array reads appended (Witness.union: the parts' arrays and keccak
// families are disjoint, their uf_apps concatenate in part order)
void add_part(Ev& E, const uint32_t* var_desc, size_t n_vars, const uint32_t* values, const uint32_t* uf_apps,
              size_t n_uf, const uint32_t* reads, size_t n_reads) {
        for (size_t i = 0; i < n_vars; i++) {
            const uint32_t* d = var_desc + 4 * i;
            const V val(values + 8 * i, values + 8 * i + 8);
            if (d[0] == PFLT_VT_TERM) {
                const pflt_term_view t = E.T(d[1]);
                if (t.op == PFLT_VAR)
                    E.vars[E.name_of(t)] = val;
                else if (t.op == PFLT_BVAR)
                    E.bools[E.name_of(t)] = (val[0] & 1u) != 0;
                else
                    E.app_vals[d[1]] = val;
            } else if (d[0] == PFLT_VT_SELECT) {
                E.read_vals[{d[1], d[2]}] = val;
            } else {  // one 256-bit chunk (lo = d[2]) of a wider free symbol
                const pflt_term_view t = E.T(d[1]);
                const uint32_t w = E.width(t);
                V& cur = E.vars[E.name_of(t)];
                if (cur.empty()) cur = vzero(w);
                cur = binop(PFLT_BVOR, cur, vshl(val, d[2], w), w);
            }
        }
        E.uf_apps.insert(E.uf_apps.end(), uf_apps, uf_apps + n_uf);
        for (size_t i = 0; i < n_reads; i++) {
            const uint32_t arr = reads[2 * i], idx = reads[2 * i + 1];
            E.reads[E.name_of(E.T(arr))].push_back({arr, idx});
        }
}

int recheck_core(void* store, const uint32_t* var_desc, size_t n_vars, const uint32_t* values,
                 const uint32_t* uf_apps, size_t n_uf, const uint32_t* reads, size_t n_reads,
                 const uint32_t* registry, size_t n_registry, const uint32_t* roots,
                 size_t n_roots, uint8_t* out) {
    try {
        Ev E;
        E.st = store;
        parse_registry(E, registry, n_registry);
        add_part(E, var_desc, n_vars, values, uf_apps, n_uf, reads, n_reads);
        for (size_t i = 0; i < n_roots; i++) out[i] = Ev::bool_of(E.ev(roots[i])) ? 1u : 0u;
        return 0;
    } catch (...) {
        return -1;
    }
}

// the witness metadata of one lowering result (pflt_result_get) into E, with its values
void add_result(Ev& E, void* R, const uint32_t* values) {
    uint64_t info[17];
    pflt_result_info(R, info);
    const size_t nvt = info[2], nuf = info[3], na = info[4], nr = info[5];
    std::vector<uint32_t> desc(4 * nvt + 1), ufs(nuf + 1), rd(na + 2 * nr + 1);
    pflt_result_get(R, PFLT_GET_VAR_TERMS, desc.data(), nullptr);
    pflt_result_get(R, PFLT_GET_UF_APPS, ufs.data(), nullptr);
    pflt_result_get(R, PFLT_GET_READS, rd.data(), nullptr);
    add_part(E, desc.data(), std::min<size_t>(nvt, info[0]), values, ufs.data(), nuf, rd.data() + na, nr);
}

}  // namespace

extern "C" int pflt_recheck(void* store, const uint32_t* var_desc, size_t n_vars, const uint32_t* values,
                            const uint32_t* uf_apps, size_t n_uf, const uint32_t* reads, size_t n_reads,
                            const uint32_t* registry, size_t n_registry, const uint32_t* roots,
                            size_t n_roots, uint8_t* out) {
    return recheck_core(store, var_desc, n_vars, values, uf_apps, n_uf, reads, n_reads, registry, n_registry,
                        roots, n_roots, out);
}

// the witness metadata of a lowering result (pflt_result_get), re-checked like pflt_recheck
extern "C" void pflt_recheck_many(void* store, void* const* results, size_t n, const uint32_t* values,
                                  const uint32_t* registry, size_t n_registry, uint32_t n_threads,
                                  int8_t* status) {
    std::vector<size_t> off(n + 1, 0);
    for (size_t j = 0; j < n; j++) {
        uint64_t info[17];
        pflt_result_info(results[j], info);
        off[j + 1] = off[j] + 8 * info[0];
    }
    auto one = [&](size_t j) {
        uint64_t info[17];
        void* R = results[j];
        pflt_result_info(R, info);
        const size_t nvt = info[2], nuf = info[3], na = info[4], nr = info[5], nro = info[14];
        std::vector<uint32_t> desc(4 * nvt + 1), ufs(nuf + 1), rd(na + 2 * nr + 1), roots(nro + 1);
        pflt_result_get(R, PFLT_GET_VAR_TERMS, desc.data(), nullptr);
        pflt_result_get(R, PFLT_GET_UF_APPS, ufs.data(), nullptr);
        pflt_result_get(R, PFLT_GET_READS, rd.data(), nullptr);
        pflt_result_get(R, PFLT_GET_IN_ROOTS, roots.data(), nullptr);
        // var_terms pair with the program's variables (interp.Witness zips them)
        const size_t nv = std::min<size_t>(nvt, info[0]);
        std::vector<uint8_t> out(nro + 1, 0);
        const int rc = recheck_core(store, desc.data(), nv, values + off[j], ufs.data(), nuf, rd.data() + na, nr,
                                    registry, n_registry, roots.data(), nro, out.data());
        if (rc != 0) {
            status[j] = -1;
            return;
        }
        int8_t ok = 1;
        for (size_t i = 0; i < nro; i++) ok &= out[i] ? 1 : 0;
        status[j] = ok;
    };
    pfpool::parallel_for(n, n_threads, one);
}

// ---- GPU witnesses kept natively for the GPU-resident ModelCache (mythril_amd/model_cache.py):
// a witness's interpretation (interp.Witness, bit for bit: the recheck's evaluator) built
// once from its parts' lowering results and values, with its evaluation memo kept across
// calls; pflt_witness_values evaluates the quick-sat leaf terms under many witnesses at once.
struct WitnessH {
    Ev E;
    uint64_t reg_serial = 0;  // the registry state its hash specs were parsed from
    // the values of the caller's leaf slots (dense: a leaf read again is a 32-byte copy, not a
    // memo lookup); state 0 unknown, 1 evaluated, 2 not evaluable natively
    uint64_t slot_epoch = 0;
    std::vector<uint32_t> slot_vals;
    std::vector<uint8_t> slot_state;
};

extern "C" void* pflt_witness_new(void* store, void* const* results, size_t n_parts, const uint32_t* values,
                                  const uint32_t* registry, size_t n_registry, uint64_t reg_serial) {
    WitnessH* W = new WitnessH();
    try {
        W->E.st = store;
        parse_registry(W->E, registry, n_registry);
        W->reg_serial = reg_serial;
        size_t off = 0;
        for (size_t j = 0; j < n_parts; j++) {
            uint64_t info[17];
            pflt_result_info(results[j], info);
            add_result(W->E, results[j], values + off);
            off += 8 * info[0];
        }
        return W;
    } catch (...) {
        delete W;
        return nullptr;
    }
}

extern "C" void pflt_witness_free(void* w) { delete (WitnessH*)w; }

// values of terms[0..n_terms) under each witness: out_limbs[(m * n_terms + i) * 8 ..], ok = 1
// where the term evaluated (0: the caller evaluates it another way); the witnesses in parallel
extern "C" void pflt_witness_values(void* const* witnesses, size_t n_models, const uint32_t* terms, size_t n_terms,
                                    const uint32_t* slots, uint64_t slot_epoch,
                                    const uint32_t* registry, size_t n_registry, uint64_t reg_serial,
                                    uint32_t n_threads, uint32_t* out_limbs, uint8_t* ok) {
    auto one = [&](size_t m) {
        WitnessH* W = (WitnessH*)witnesses[m];
        Ev& E = W->E;
        if (W->reg_serial != reg_serial) {
            // hashes registered since (interp.Witness reads its live registry): re-parse; the
            // memo stays, as the Python witness's does
            try {
                std::map<uint32_t, KSpec> old;
                old.swap(E.kspecs);
                try {
                    parse_registry(E, registry, n_registry);
                } catch (...) {
                    E.kspecs.swap(old);
                    throw;
                }
                W->reg_serial = reg_serial;
            } catch (...) {
                for (size_t i = 0; i < n_terms; i++) ok[m * n_terms + i] = 0;
                return;
            }
        }
        if (slots && W->slot_epoch != slot_epoch) {  // renumbered: drop the old slots' memory
            std::vector<uint32_t>().swap(W->slot_vals);
            std::vector<uint8_t>().swap(W->slot_state);
            W->slot_epoch = slot_epoch;
        }
        for (size_t i = 0; i < n_terms; i++) {
            uint32_t* o = out_limbs + (m * n_terms + i) * 8;
            const uint32_t s = slots ? slots[i] : 0u;
            if (slots && s < W->slot_state.size() && W->slot_state[s]) {
                if (W->slot_state[s] == 1) std::copy(&W->slot_vals[8 * (size_t)s], &W->slot_vals[8 * (size_t)s] + 8, o);
                ok[m * n_terms + i] = W->slot_state[s] == 1;
                continue;
            }
            uint8_t st = 2;
            try {
                const uint32_t w = E.width(E.T(terms[i]));
                const V v = vmask(E.ev(terms[i]), w ? std::min<uint32_t>(w, 256) : 256);
                for (size_t k = 0; k < 8; k++) o[k] = k < v.size() ? v[k] : 0u;
                st = 1;
            } catch (...) {
            }
            ok[m * n_terms + i] = st == 1;
            if (slots) {
                if (s >= W->slot_state.size()) {
                    W->slot_state.resize((size_t)s + 1 + s / 2, 0);
                    W->slot_vals.resize(8 * W->slot_state.size(), 0);
                }
                W->slot_state[s] = st;
                if (st == 1) std::copy(o, o + 8, &W->slot_vals[8 * (size_t)s]);
            }
        }
    };
    pfpool::parallel_for(n_models, n_threads, one);
}
