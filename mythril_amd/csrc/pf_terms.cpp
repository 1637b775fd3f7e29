// pf_terms.cpp — libpflower.so: constraint terms -> bytecode DAG -> program, natively
// (include/pf_lower.h, "term store" section).
//
// The native form of mythril_amd/smt/to_dag.py:TermLowering and mythril_amd/lower.py:Dag —
// node for node: the same hash-consed node table (same order, same word-slicing rewrites),
// the same variables (names, kinds, schema hints, parents), the same by-construction
// interpretation of arrays, keccak256_<n> / inverse and Power, the same chunked wide values —
// and then the hint derivation (pfl_hints) and register allocation (pfl_lower) of the same
// library, so a bucket goes from terms to a program without a Python DAG in between.
// tests/test_native_terms.py checks the node tables, variables, witness metadata and
// programs against the Python lowering.  Host code, no HIP.
//
// Terms live in a store the host fills once per term (hash-consed Python terms are immortal,
// so a term's store id never changes): children before parents.  A lowering call names the
// bucket's roots, the keccak registry, the parent models and the program seed.
#include <algorithm>
#include <array>
#include <cctype>
#include <cstdlib>
#include <tuple>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <list>
#include <deque>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/pf_bytecode.h"
#include "../../include/pf_lower.h"
#include "pf_pool.h"

namespace {

thread_local std::string t_err;

struct TermError {
    int rc;
};

#ifndef PF_MAX_TERM_DEPTH
#define PF_MAX_TERM_DEPTH 5000u
#endif

[[noreturn]] void lerr(const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_err = buf;
    throw TermError{-2};
}

// ---- big unsigned integers (term constants: any width) ---------------------------------
typedef std::vector<uint32_t> Big;  // little-endian limbs, no trailing-zero normalisation

uint32_t limb(const Big& v, size_t i) { return i < v.size() ? v[i] : 0u; }

Big mask_big(const Big& v, uint32_t w) {
    const size_t nl = (w + 31) / 32;
    Big r(nl, 0u);
    for (size_t i = 0; i < nl; i++) r[i] = limb(v, i);
    if (w % 32 && nl) r[nl - 1] &= (1u << (w % 32)) - 1u;
    return r;
}

Big shr_big(const Big& v, uint32_t s) {
    const size_t q = s / 32, b = s % 32;
    Big r;
    for (size_t i = q; i < v.size(); i++) {
        uint32_t x = v[i] >> b;
        if (b && i + 1 < v.size()) x |= v[i + 1] << (32 - b);
        r.push_back(x);
    }
    return r;
}

bool big_eq(const Big& a, const Big& b) {
    const size_t n = std::max(a.size(), b.size());
    for (size_t i = 0; i < n; i++)
        if (limb(a, i) != limb(b, i)) return false;
    return true;
}

bool big_zero(const Big& a) {
    for (uint32_t x : a)
        if (x) return false;
    return true;
}

uint32_t bitlen(const Big& a) {
    for (size_t i = a.size(); i-- > 0;)
        if (a[i]) return (uint32_t)(32 * i + 32 - __builtin_clz(a[i]));
    return 0;
}

// ---- 256-bit constants (DAG constant nodes) ------------------------------------------------
struct C8 {
    uint32_t l[8];
    bool operator==(const C8& o) const { return memcmp(l, o.l, sizeof(l)) == 0; }
};

C8 c8_of(const Big& v, uint32_t w) {  // v masked to w <= 256 bits
    C8 c;
    const Big m = mask_big(v, w);
    for (int i = 0; i < 8; i++) c.l[i] = limb(m, i);
    return c;
}

C8 c8_small(uint64_t x, uint32_t w) {
    Big b = {(uint32_t)x, (uint32_t)(x >> 32)};
    return c8_of(b, w);
}

Big big_of(const C8& c) { return Big(c.l, c.l + 8); }

// a * b mod 2^256 and b^e mod 2^256 (Power's concrete facts, pow(c1, c2, 1 << 256))
C8 mul8(const C8& a, const C8& b) {
    uint32_t r[8] = {0};
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
        for (int j = 0; i + j < 8; j++) {
            c += (uint64_t)a.l[i] * b.l[j] + r[i + j];
            r[i + j] = (uint32_t)c;
            c >>= 32;
        }
    }
    C8 o;
    memcpy(o.l, r, sizeof(r));
    return o;
}

C8 pow8(const C8& b, const C8& e) {
    C8 r = c8_small(1, 256), x = b;
    for (int i = 0; i < 256; i++) {
        if ((e.l[i / 32] >> (i % 32)) & 1u) r = mul8(r, x);
        x = mul8(x, x);
    }
    return r;
}

uint32_t crc32_of(const std::string& s) {  // zlib.crc32 (to_dag.salt_of)
    uint32_t c = 0xffffffffu;
    for (unsigned char ch : s) {
        c ^= ch;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return c ^ 0xffffffffu;
}

// ---- the term store -------------------------------------------------------------------
struct TermRec {
    uint32_t op, sortk, w1, w2;
    uint32_t depth = 1;  // nesting depth (1 + the deepest argument's), set by pflt_add
    std::vector<uint32_t> args;
    int64_t i0, i1;
    Big val;
    std::string name;
};

// Parent model of one bucket: values by symbol name (any width) and by base-array read
// (array id, index id) — pflt_lower's par_* arguments, or gpu_check._recent_parent's dict.
struct Parents {
    std::unordered_map<std::string, Big> names;
    std::map<std::pair<uint32_t, uint32_t>, C8> reads;
    std::vector<std::string> name_order;                      // dump order (tests)
    std::vector<std::pair<uint32_t, uint32_t>> read_order;
    bool empty() const { return names.empty() && reads.empty(); }
    void set_name(const std::string& n, const Big& v) {
        if (names.emplace(n, v).second) name_order.push_back(n);
        else names[n] = v;
    }
    void set_read(std::pair<uint32_t, uint32_t> k, const C8& v) {
        if (reads.emplace(k, v).second) read_order.push_back(k);
        else reads[k] = v;
    }
};

// A least-recently-updated map (Python's OrderedDict with move_to_end on every write and
// popitem(last=False) to trim) — gpu_check._RECENT_VARS / _RECENT_READS.
template <class K, class V, class H = std::hash<K>>
struct Lru {
    std::list<K> order;
    std::unordered_map<K, std::pair<typename std::list<K>::iterator, V>, H> m;
    V& touch(const K& k) {  // get-or-create, moved to the newest end
        auto it = m.find(k);
        if (it != m.end()) {
            order.splice(order.end(), order, it->second.first);
            return it->second.second;
        }
        order.push_back(k);
        return m.emplace(k, std::make_pair(std::prev(order.end()), V())).first->second.second;
    }
    const V* get(const K& k) const {
        auto it = m.find(k);
        return it == m.end() ? nullptr : &it->second.second;
    }
    void trim(size_t n) {
        while (m.size() > n) {
            m.erase(order.front());
            order.pop_front();
        }
    }
    void clear() {
        order.clear();
        m.clear();
    }
};

struct PairHash {
    size_t operator()(const std::pair<uint32_t, uint32_t>& p) const {
        return std::hash<uint64_t>()(((uint64_t)p.first << 32) | p.second);
    }
};

struct Recent {  // newest accepted witness / z3-model values, for parent models
    Lru<std::string, Big> vars;
    // per array name: (array id, index id) of a base-array read -> value
    Lru<std::string, Lru<std::pair<uint32_t, uint32_t>, C8, PairHash>> reads;
};

struct Store {
    std::vector<TermRec> t;
    Recent recent;
    // independence keys (smt/independence.py), memoised per term: sorted key ids and the
    // widths whose inverse keccak the term applies to a non-application
    std::vector<int32_t> kmemo;  // term id -> index into keysets (-1: not computed)
    std::vector<std::vector<uint32_t>> keysets, finvs;
    std::unordered_map<std::string, uint32_t> key_ids;
    std::vector<std::string> key_names;
    // per key id, for pflt_buckets: the id of the keccak family a "k:<n>" key belongs to (the
    // key "<n>"), -2 for any other key, -1 while "<n>" has no id yet (looked up again), -3 not
    // classified yet; and the per-call union-find / group scratch, indexed by key id (-1 =
    // untouched; reset through the touched list after each call)
    std::vector<int32_t> kfam, uf, ugrp;
};

// ---- the DAG (mythril_amd/lower.py Dag) ---------------------------------------------------
constexpr uint32_t K_VAR = PFL_K_VAR, K_CONST = PFL_K_CONST, K_BCONST = PFL_K_BCONST,
                   K_BVAR = PFL_K_BVAR;

struct DNode {
    uint32_t kind, width, nargs;
    int32_t args[3];
    uint32_t aux;
    C8 cv;  // K_CONST value
    bool is_bool;
};

struct DVar {
    std::string name;
    uint32_t width, kind, hint0, hint1;
    bool has_parent;
    C8 parent;
};

struct NodeKey {  // the hash-consing key of a node (lower.py Node tuple)
    uint32_t kind, width, nargs, aux;
    int32_t args[3];
    uint32_t is_bool;
    C8 cv;
    bool operator==(const NodeKey& o) const { return memcmp(this, &o, sizeof(NodeKey)) == 0; }
};

struct NodeKeyHash {
    size_t operator()(const NodeKey& k) const {
        const uint32_t* w = (const uint32_t*)&k;
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (size_t i = 0; i < sizeof(NodeKey) / 4; i++) h = (h ^ w[i]) * 0x100000001B3ull;
        return (size_t)(h ^ (h >> 29));
    }
};

// Hash-consing table of a DAG: open addressing over node ids (the key is the node itself),
// linear probing, grown at half load.  A std::unordered_map<NodeKey, id> allocated one
// 80-byte node per DAG node and, reserved for 4,096 entries per job, zeroed a 32 KB bucket
// array for buckets of a few dozen nodes — allocation churn that was a large share of a
// single query's lowering.
struct NodeTable {
    std::vector<int32_t> slot;   // -1 = empty
    size_t used = 0;
    void clear() { std::vector<int32_t>().swap(slot); used = 0; }
};

inline uint64_t node_hash(uint32_t kind, uint32_t width, uint32_t nargs, const int32_t* args, uint32_t aux,
                          bool is_bool, const C8* cv) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    auto mix = [&](uint32_t w) { h = (h ^ w) * 0x100000001B3ull; };
    mix(kind);
    mix(width);
    mix(nargs);
    mix(aux);
    for (uint32_t i = 0; i < nargs; i++) mix((uint32_t)args[i]);
    mix(is_bool ? 1u : 0u);
    if (kind == K_CONST)  // a constant without a value given is the zero constant
        for (int i = 0; i < 8; i++) mix(cv ? cv->l[i] : 0u);
    // fmix64: the table indexes with the low bits, which the FNV products alone spread poorly
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 33);
}

struct Dag {
    std::vector<DNode> nodes;
    std::vector<int32_t> roots;
    std::vector<DVar> vars;
    std::vector<C8> forced;
    NodeTable memo;
    std::unordered_map<std::string, int32_t> var_index;

    explicit Dag(size_t reserve = 64) {
        size_t cap = 16;
        while (cap < 2 * reserve) cap <<= 1;
        memo.slot.assign(cap, -1);
        nodes.reserve(reserve);
    }

    bool same(const DNode& n, uint32_t kind, uint32_t width, const int32_t* args, uint32_t nargs, uint32_t aux,
              bool is_bool, const C8* cv) const {
        if (n.kind != kind || n.width != width || n.nargs != nargs || n.aux != aux || n.is_bool != is_bool) return false;
        for (uint32_t i = 0; i < nargs; i++)
            if (n.args[i] != args[i]) return false;
        if (kind == K_CONST) {
            static const C8 zero{};
            return memcmp(n.cv.l, (cv ? cv : &zero)->l, sizeof(n.cv.l)) == 0;
        }
        return true;
    }

    void grow() {
        std::vector<int32_t> old;
        old.swap(memo.slot);
        memo.slot.assign(old.size() * 2, -1);
        const size_t mask = memo.slot.size() - 1;
        for (int32_t id : old) {
            if (id < 0) continue;
            const DNode& n = nodes[(size_t)id];
            size_t h = (size_t)node_hash(n.kind, n.width, n.nargs, n.args, n.aux, n.is_bool, &n.cv) & mask;
            while (memo.slot[h] >= 0) h = (h + 1) & mask;
            memo.slot[h] = id;
        }
    }

    int32_t add_n(uint32_t kind, uint32_t width, const int32_t* args, uint32_t nargs, uint32_t aux,
                  bool is_bool, const C8* cv = nullptr) {
        if (memo.slot.empty()) memo.slot.assign(16, -1);
        const size_t mask = memo.slot.size() - 1;
        size_t h = (size_t)node_hash(kind, width, nargs, args, aux, is_bool, cv) & mask;
        for (;;) {
            const int32_t id = memo.slot[h];
            if (id < 0) break;
            if (same(nodes[(size_t)id], kind, width, args, nargs, aux, is_bool, cv)) return id;
            h = (h + 1) & mask;
        }
        DNode n;
        memset(&n, 0, sizeof(n));
        n.kind = kind;
        n.width = width;
        n.nargs = nargs;
        for (uint32_t i = 0; i < nargs; i++) n.args[i] = args[i];
        n.aux = aux;
        if (cv) n.cv = *cv;
        n.is_bool = is_bool;
        const int32_t id = (int32_t)nodes.size();
        nodes.push_back(n);
        memo.slot[h] = id;
        if (2 * ++memo.used > memo.slot.size()) grow();
        return id;
    }

    int32_t add(uint32_t kind, uint32_t width, std::initializer_list<int32_t> args, uint32_t aux,
                bool is_bool, const C8* cv = nullptr) {
        return add_n(kind, width, args.begin(), (uint32_t)args.size(), aux, is_bool, cv);
    }

    uint32_t force_consts(const std::vector<C8>& vals) {
        const uint32_t start = (uint32_t)forced.size();
        forced.insert(forced.end(), vals.begin(), vals.end());
        return start;
    }

    int32_t var(const std::string& name, uint32_t width, uint32_t kind, uint32_t h0, uint32_t h1,
                bool has_parent, const C8& parent, bool* created) {
        auto it = var_index.find(name);
        uint32_t idx;
        *created = false;
        if (it == var_index.end()) {
            idx = (uint32_t)vars.size();
            DVar v{name, width, kind, h0, h1, has_parent, parent};
            vars.push_back(v);
            var_index.emplace(name, (int32_t)idx);
            *created = true;
        } else {
            idx = (uint32_t)it->second;
        }
        if (kind == PF_VK_BOOL) return add(K_BVAR, 1, {}, idx, true);
        return add(K_VAR, width, {}, idx, false);
    }

    int32_t cnst(const C8& v, uint32_t width) {
        if (width == 256) return add(K_CONST, width, {}, 0, false, &v);
        C8 m = c8_of(big_of(v), width);
        return add(K_CONST, width, {}, 0, false, &m);
    }
    int32_t cnst(uint64_t v, uint32_t width) { return cnst(c8_small(v, width), width); }
    int32_t bconst(bool v) { return add(K_BCONST, 1, {}, v ? 1u : 0u, true); }

    const C8* cval(int32_t i) const { return nodes[i].kind == K_CONST ? &nodes[i].cv : nullptr; }

    int32_t op(uint32_t opc, uint32_t w, std::initializer_list<int32_t> args, uint32_t aux = 0) {
        const int32_t r = simplify(opc, w, args.begin(), aux);
        if (r >= 0) return r;
        return add_n(opc, w, args.begin(), (uint32_t)args.size(), aux, opc >= PF_B_CONST);
    }

    // Dag._simplify: the word-slicing rewrites (lower.py)
    int32_t simplify(uint32_t opc, uint32_t w, const int32_t* args, uint32_t aux) {
        if (opc == PF_W_UDIV) {
            const C8* c = cval(args[1]);
            if (c) {
                const Big cb = big_of(*c);
                const uint32_t bl = bitlen(cb);
                if (bl && bitlen(mask_big(shr_big(cb, 0), bl - 1)) == 0) {  // power of two
                    const uint32_t k = bl - 1;
                    return k == 0 ? args[0] : op(PF_W_LSHR, w, {args[0], cnst(k, w)});
                }
            }
        } else if (opc == PF_W_LSHR) {
            const C8* c = cval(args[1]);
            const DNode x = nodes[args[0]];
            if (c && bitlen(big_of(*c)) <= 32 && c->l[0] < w) {
                const uint32_t k = c->l[0];
                if (k == 0) return args[0];
                if (x.kind == PF_W_MOV) {
                    const int32_t inner = x.args[0];
                    const uint32_t wi = nodes[inner].width;
                    if (k >= wi) return cnst(0, w);
                    return op(PF_W_MOV, w, {op(PF_W_EXTRACT, wi - k, {inner}, k)});
                }
                if (x.kind == PF_W_CONCAT) return op(PF_W_MOV, w, {op(PF_W_EXTRACT, w - k, {args[0]}, k)});
            }
        } else if (opc == PF_W_AND) {
            for (int xi = 0; xi < 2; xi++) {
                const int ci = 1 - xi;
                const C8* c = cval(args[ci]);
                if (!c) continue;
                const Big cb = big_of(*c);
                const uint32_t bl = bitlen(cb);
                if (bl == 0) continue;
                // c == 2^bl - 1
                bool ones = true;
                for (uint32_t i = 0; i < bl; i++)
                    if (!((cb[i / 32] >> (i % 32)) & 1u)) { ones = false; break; }
                if (ones && bl < w) return op(PF_W_MOV, w, {op(PF_W_EXTRACT, bl, {args[xi]}, 0)});
            }
        } else if (opc == PF_W_EXTRACT) {
            const DNode x = nodes[args[0]];
            if (aux == 0 && w == x.width) return args[0];
            if (x.kind == PF_W_CONCAT) {
                const int32_t hi = x.args[0], lo = x.args[1];
                const uint32_t wl = x.aux;
                if (aux >= wl) return op(PF_W_EXTRACT, w, {hi}, aux - wl);
                if (aux + w <= wl) return op(PF_W_EXTRACT, w, {lo}, aux);
                const int32_t top = op(PF_W_EXTRACT, aux + w - wl, {hi}, 0);
                const int32_t bot = op(PF_W_EXTRACT, wl - aux, {lo}, aux);
                return op(PF_W_CONCAT, w, {top, bot}, wl - aux);
            }
            if (x.kind == PF_W_MOV) {
                const int32_t inner = x.args[0];
                const uint32_t wi = nodes[inner].width;
                if (aux + w <= wi) return op(PF_W_EXTRACT, w, {inner}, aux);
                if (aux >= wi) return cnst(0, w);
            }
            if (x.kind == K_CONST) return cnst(c8_of(shr_big(big_of(x.cv), aux), w), w);
        } else if (opc == PF_W_MOV) {
            const DNode x = nodes[args[0]];
            if (x.width == w) return args[0];
            if (x.kind == PF_W_MOV) return op(PF_W_MOV, w, {x.args[0]});
            if (x.kind == K_CONST) return cnst(x.cv, w);
        } else if (opc == PF_B_EQ) {
            for (int xi = 0; xi < 2; xi++) {
                const int ci = 1 - xi;
                const C8* c = cval(args[ci]);
                const DNode x = nodes[args[xi]];
                if (c && x.kind == PF_W_MOV) {
                    const uint32_t wy = nodes[x.args[0]].width;
                    if (!big_zero(shr_big(big_of(*c), wy))) return bconst(false);
                    return op(PF_B_EQ, wy, {x.args[0], cnst(*c, wy)});
                }
            }
        }
        return -1;
    }

    // the calldata-byte arm's word constants (Dag.word_constants / finalize_word_hints)
    void finalize_word_hints() {
        bool any = false;
        for (const DVar& v : vars) any |= v.kind == PF_VK_CDBYTE;
        if (!any) return;
        std::vector<C8> words;
        for (const DNode& nd : nodes) {
            if (!(nd.kind == PF_B_EQ || nd.kind == PF_B_ULT || nd.kind == PF_B_ULE ||
                  nd.kind == PF_B_SLT || nd.kind == PF_B_SLE))
                continue;
            const DNode& a = nodes[nd.args[0]];
            const DNode& b = nodes[nd.args[1]];
            const DNode* pairs[2][2] = {{&a, &b}, {&b, &a}};
            for (auto& pr : pairs) {
                const DNode* c = pr[0];
                const DNode* other = pr[1];
                if (c->kind != K_CONST) continue;
                if (other->kind == K_VAR && vars[other->aux].kind == PF_VK_SMALL) continue;
                bool seen = false;
                for (const C8& x : words) seen |= x == c->cv;
                if (!seen) words.push_back(c->cv);
            }
        }
        if (words.size() > 0xFFF) words.resize(0xFFF);
        if (words.empty() || forced.size() >= 0xFFF) return;
        const uint32_t start = force_consts(words);
        for (DVar& v : vars)
            if (v.kind == PF_VK_CDBYTE) v.hint0 = (v.hint0 & 0xFFu) | ((uint32_t)words.size() << 8) | (start << 20);
    }
};

// ---- term lowering (to_dag.TermLowering) ---------------------------------------------------
enum TOp : uint32_t {
    T_BV = PFLT_BV, T_TRUE = PFLT_TRUE, T_FALSE = PFLT_FALSE, T_VAR = PFLT_VAR, T_BVAR = PFLT_BVAR,
    T_ARRAY = PFLT_ARRAY, T_K = PFLT_K, T_SELECT = PFLT_SELECT, T_STORE = PFLT_STORE,
    T_APPLY = PFLT_APPLY, T_EXTRACT = PFLT_EXTRACT, T_CONCAT = PFLT_CONCAT,
    T_ZEXT = PFLT_ZERO_EXTEND, T_ITE = PFLT_ITE, T_EQ = PFLT_EQ, T_IFF = PFLT_IFF,
    T_AND = PFLT_AND, T_OR = PFLT_OR, T_NOT = PFLT_NOT, T_XOR = PFLT_XOR, T_BVNOT = PFLT_BVNOT,
    T_BVNEG = PFLT_BVNEG,
};

uint32_t wbin_op(uint32_t op) {
    switch (op) {
        case PFLT_BVADD: return PF_W_ADD;
        case PFLT_BVSUB: return PF_W_SUB;
        case PFLT_BVMUL: return PF_W_MUL;
        case PFLT_BVUDIV: return PF_W_UDIV;
        case PFLT_BVUREM: return PF_W_UREM;
        case PFLT_BVSDIV: return PF_W_SDIV;
        case PFLT_BVSREM: return PF_W_SREM;
        case PFLT_BVSMOD: return PF_W_SMOD;
        case PFLT_BVAND: return PF_W_AND;
        case PFLT_BVOR: return PF_W_OR;
        case PFLT_BVXOR: return PF_W_XOR;
        case PFLT_BVSHL: return PF_W_SHL;
        case PFLT_BVLSHR: return PF_W_LSHR;
        case PFLT_BVASHR: return PF_W_ASHR;
        case PFLT_BVEXP: return PF_W_EXP;
        default: return 0;
    }
}

uint32_t bcmp_op(uint32_t op) {
    switch (op) {
        case PFLT_BVULT: return PF_B_ULT;
        case PFLT_BVULE: return PF_B_ULE;
        case PFLT_BVSLT: return PF_B_SLT;
        case PFLT_BVSLE: return PF_B_SLE;
        case PFLT_BVUADD_NOOVF: return PF_B_UADD_NOOVF;
        case PFLT_BVUMUL_NOOVF: return PF_B_UMUL_NOOVF;
        default: return 0;
    }
}

typedef std::vector<std::pair<int32_t, uint32_t>> Chunks;  // (node, width), LSB first

struct Val {  // TermLowering.w(): a node, or chunks for values wider than 256 bits
    bool wide;
    int32_t node;
    Chunks ch;
};

struct KSpec {
    bool has_lo;
    C8 base;
    std::vector<std::pair<Big, C8>> concrete;  // insertion order (dict order)
};

// var_terms descriptors handed back to the host (Lowered.var_terms)
struct VarTerm {
    uint32_t type;  // PFLT_VT_TERM / PFLT_VT_SELECT / PFLT_VT_EXTRACT
    uint32_t a, b;  // term id | (array id, index id) | (term id, lo)
    uint32_t c;     // extract hi
};

// term id -> Val memo of a lowering: open addressing over the term ids, values in a deque (a
// reference handed out stays valid while the table grows, as with the node-based map this
// replaces, without its per-entry allocation)
struct ValMemo {
    std::vector<uint32_t> key;   // term id + 1, 0 = empty
    std::vector<uint32_t> idx;
    std::deque<Val> vals;
    ValMemo() : key(64, 0u), idx(64, 0u) {}
    static size_t hsh(uint32_t t) { return (size_t)((t * 0x9E3779B1u) ^ (t >> 15)); }
    Val* find(uint32_t t) {
        const size_t mask = key.size() - 1;
        for (size_t h = hsh(t) & mask;; h = (h + 1) & mask) {
            if (key[h] == 0u) return nullptr;
            if (key[h] == t + 1u) return &vals[idx[h]];
        }
    }
    Val& put(uint32_t t, Val&& v) {
        if (2 * (vals.size() + 1) > key.size()) {
            std::vector<uint32_t> ok, oi;
            ok.swap(key);
            oi.swap(idx);
            key.assign(ok.size() * 2, 0u);
            idx.assign(ok.size() * 2, 0u);
            const size_t m2 = key.size() - 1;
            for (size_t i = 0; i < ok.size(); i++) {
                if (!ok[i]) continue;
                size_t h = hsh(ok[i] - 1u) & m2;
                while (key[h]) h = (h + 1) & m2;
                key[h] = ok[i];
                idx[h] = oi[i];
            }
        }
        const size_t mask = key.size() - 1;
        size_t h = hsh(t) & mask;
        while (key[h]) h = (h + 1) & mask;
        key[h] = t + 1u;
        idx[h] = (uint32_t)vals.size();
        vals.push_back(std::move(v));
        return vals.back();
    }
};

struct Lowering {
    const Store& S;
    Dag d;
    ValMemo memo;
    std::vector<VarTerm> var_terms;
    // base array name -> [(idx id, arr id, idx node, value node)]; names in insertion order
    std::vector<std::string> array_order;
    std::unordered_map<std::string, std::vector<std::array<int32_t, 4>>> arrays;
    std::map<uint32_t, std::vector<std::pair<uint32_t, int32_t>>> keccak_apps;  // n -> (arg id, f node)
    std::map<uint32_t, std::vector<std::pair<int32_t, int32_t>>> inv_apps;      // n -> (key node, value node)
    std::vector<uint32_t> uf_apps;   // app term ids, registration order
    std::vector<int32_t> side;
    bool actors_forced = false;
    // explicit-model lowering (PFLT_EXPLICIT): leaves by (array, index) / by UF-application term
    bool explicit_ = false;
    std::map<std::pair<uint32_t, uint32_t>, int32_t> leaf_reads;
    std::unordered_map<uint32_t, int32_t> leaf_apps;
    uint32_t n_leaves = 0;
    uint32_t actor_start = 0;
    std::vector<C8> actors;
    std::map<uint32_t, KSpec> kspecs;
    // Power: (b id, e id, value node, symbolic); concrete facts in discovery order
    std::vector<std::tuple<uint32_t, uint32_t, int32_t, bool>> power_apps;
    std::vector<std::pair<std::pair<C8, C8>, C8>> power_facts;
    // parents: by symbol name, by (array id, index id)
    const std::unordered_map<std::string, Big>& par_name;
    const std::map<std::pair<uint32_t, uint32_t>, C8>& par_read;

    Lowering(const Store& s, const Parents& p) : S(s), par_name(p.names), par_read(p.reads) {}

    const TermRec& T(uint32_t id) const { return S.t[id]; }
    uint32_t width(uint32_t id) const { return T(id).sortk == 1 ? T(id).w1 : 0; }

    // ---- leaves --------------------------------------------------------------------
    static bool cdbyte_name(const std::string& name, uint32_t* off) {
        // ^\d+_calldata\[(\d+)\]$
        size_t i = 0;
        while (i < name.size() && isdigit((unsigned char)name[i])) i++;
        if (i == 0) return false;
        static const char mid[] = "_calldata[";
        if (name.compare(i, sizeof(mid) - 1, mid) != 0) return false;
        i += sizeof(mid) - 1;
        size_t j = i;
        while (j < name.size() && isdigit((unsigned char)name[j])) j++;
        if (j == i || j + 1 != name.size() || name[j] != ']') return false;
        *off = (uint32_t)strtoul(name.c_str() + i, nullptr, 10);
        return true;
    }

    static uint32_t var_kind(const std::string& name, uint32_t w) {
        if (name.rfind("sender_", 0) == 0 && w == 256) return PF_VK_ACTOR;
        const std::string suf = "_calldatasize";
        if (name.size() >= suf.size() && name.compare(name.size() - suf.size(), suf.size(), suf) == 0)
            return PF_VK_SMALL;
        uint32_t off;
        if (w == 8 && cdbyte_name(name, &off)) return PF_VK_CDBYTE;
        if (w == 256 && (name.rfind("call_value", 0) == 0 || name.rfind("callvalue", 0) == 0))
            return PF_VK_VALUE;
        return PF_VK_GENERIC;
    }

    int32_t mkvar(const std::string& name, uint32_t w, const VarTerm& term, const C8* parent,
                  const std::pair<uint32_t, uint32_t>* read) {
        const uint32_t kind = var_kind(name, w);
        uint32_t h0 = 0, h1 = 0;
        if (kind == PF_VK_ACTOR) {
            if (!actors_forced) {
                actor_start = d.force_consts(actors);
                actors_forced = true;
            }
            h0 = actor_start;
            h1 = (uint32_t)actors.size();
        } else if (kind == PF_VK_SMALL) {
            h0 = 4 + 32 * 8;
        } else if (kind == PF_VK_CDBYTE) {
            uint32_t i;
            cdbyte_name(name, &i);
            if (i < 4) {
                h0 = 8 * (3 - i);
                h1 = 0xFFFFFFFFu;
            } else {
                h0 = 8 * (31 - (i - 4) % 32);
                h1 = (i - 4) / 32;
            }
        }
        C8 pv;
        bool hp = false;
        if (parent) {
            pv = *parent;
            hp = true;
        } else {
            auto it = par_name.find(name);
            if (it != par_name.end()) {
                pv = c8_of(it->second, 256);
                hp = true;
            } else if (read) {
                auto jt = par_read.find(*read);
                if (jt != par_read.end()) {
                    pv = jt->second;
                    hp = true;
                }
            }
        }
        if (hp) pv = c8_of(big_of(pv), w);  // Batch masks parents to the width
        bool created;
        const int32_t node = d.var(name, w, kind, h0, h1, hp, pv, &created);
        if (created) var_terms.push_back(term);
        return node;
    }

    // ---- generic lowering -----------------------------------------------------------
    const Val& w(uint32_t t) {
        if (const Val* hit = memo.find(t)) return *hit;
        Val v = lower_bv(t);
        // lower_bv may have put t itself (a recursive path to the same term): keep the first
        if (const Val* hit = memo.find(t)) return *hit;
        return memo.put(t, std::move(v));
    }

    int32_t node(uint32_t t) {
        const Val& v = w(t);
        if (v.wide) lerr("%u-bit value used where <= 256 bits are required", width(t));
        return v.node;
    }

    int32_t b(uint32_t t) {
        if (const Val* hit = memo.find(t)) return hit->node;
        const int32_t n = lower_bool(t);
        if (const Val* hit = memo.find(t)) return hit->node;
        memo.put(t, Val{false, n, {}});
        return n;
    }

    static Val V(int32_t n) { return Val{false, n, {}}; }
    static Val VW(Chunks c) { return Val{true, -1, std::move(c)}; }

    Chunks chunks(uint32_t t) { return rechunk(pieces(t)); }

    Chunks const_pieces(const Big& val, uint32_t wd) {
        Chunks out;
        Big v = val;
        uint32_t rest = wd;
        while (rest > 0) {
            const uint32_t k = std::min<uint32_t>(rest, 256);
            out.push_back({d.cnst(c8_of(v, k), k), k});
            v = shr_big(v, k);
            rest -= k;
        }
        return out;
    }

    Chunks pieces(uint32_t t) {
        const TermRec& r = T(t);
        const uint32_t wd = width(t);
        if (wd <= 256) return {{node(t), wd}};
        if (r.op == T_CONCAT) {
            Chunks out;
            for (size_t i = r.args.size(); i-- > 0;) {
                Chunks p = pieces(r.args[i]);
                out.insert(out.end(), p.begin(), p.end());
            }
            return out;
        }
        if (r.op == T_ZEXT) {
            Chunks out = pieces(r.args[0]);
            int64_t rest = r.i0;
            while (rest > 0) {
                const uint32_t k = (uint32_t)std::min<int64_t>(rest, 256);
                out.push_back({d.cnst(0, k), k});
                rest -= k;
            }
            return out;
        }
        if (r.op == T_BV) return const_pieces(r.val, wd);
        const Val& v = w(t);
        if (v.wide) return v.ch;
        lerr("wide op %u", r.op);
    }

    Chunks rechunk(const Chunks& ps) {
        Chunks out, cur;
        uint32_t fill = 0;
        for (const auto& pw : ps) {
            const int32_t nd = pw.first;
            const uint32_t wd = pw.second;
            uint32_t off = 0;
            while (off < wd) {
                const uint32_t take = std::min(256 - fill, wd - off);
                const int32_t part = (off == 0 && take == wd) ? nd : d.op(PF_W_EXTRACT, take, {nd}, off);
                cur.push_back({part, take});
                fill += take;
                off += take;
                if (fill == 256) {
                    out.push_back(join(cur));
                    cur.clear();
                    fill = 0;
                }
            }
        }
        if (!cur.empty()) out.push_back(join(cur));
        return out;
    }

    std::pair<int32_t, uint32_t> join(const Chunks& cur) {
        int32_t nd = cur.back().first;
        uint32_t wd = cur.back().second;
        for (size_t i = cur.size() - 1; i-- > 0;) {
            const int32_t part = cur[i].first;
            const uint32_t pw = cur[i].second;
            nd = d.op(PF_W_CONCAT, wd + pw, {nd, part}, pw);
            wd += pw;
        }
        return {nd, wd};
    }

    Chunks slice(const Chunks& ch, uint32_t lo, uint32_t wid) {
        Chunks ps;
        uint32_t base = 0;
        for (const auto& cw : ch) {
            const uint32_t a = std::max(lo, base), bb = std::min(lo + wid, base + cw.second);
            if (a < bb) {
                if (a == base && bb == base + cw.second)
                    ps.push_back(cw);
                else
                    ps.push_back({d.op(PF_W_EXTRACT, bb - a, {cw.first}, a - base), bb - a});
            }
            base += cw.second;
        }
        return rechunk(ps);
    }

    int32_t bit_to_w(int32_t bn, uint32_t wd) {
        return d.op(PF_W_ITE, wd, {bn, d.cnst(1, wd), d.cnst(0, wd)});
    }

    Chunks wide_addsub(const Chunks& A, const Chunks& B, bool sub) {
        const uint32_t opc = sub ? PF_W_SUB : PF_W_ADD;
        Chunks out;
        int32_t carry = -1;
        const size_t n = std::min(A.size(), B.size());
        for (size_t i = 0; i < n; i++) {
            const int32_t x = A[i].first, y = B[i].first;
            const uint32_t wx = A[i].second;
            const int32_t t = d.op(opc, wx, {x, y});
            int32_t s_ = t, cw = -1;
            if (carry >= 0) {
                cw = bit_to_w(carry, wx);
                s_ = d.op(opc, wx, {t, cw});
            }
            if (i + 1 < A.size()) {
                int32_t c1 = sub ? d.op(PF_B_ULT, wx, {x, y}) : d.op(PF_B_ULT, wx, {t, x});
                if (carry >= 0) {
                    const int32_t c2 = sub ? d.op(PF_B_ULT, wx, {t, cw}) : d.op(PF_B_ULT, wx, {s_, t});
                    c1 = d.op(PF_B_OR, 1, {c1, c2});
                }
                carry = c1;
            }
            out.push_back({s_, wx});
        }
        return out;
    }

    int32_t wide_cmp(uint32_t op, uint32_t a, uint32_t bt) {
        const Chunks A = chunks(a), B = chunks(bt);
        const bool signed_ = op == PFLT_BVSLT || op == PFLT_BVSLE;
        const bool strict = op == PFLT_BVULT || op == PFLT_BVSLT;
        int32_t lt = -1;
        const size_t n = std::min(A.size(), B.size());
        for (size_t i = 0; i < n; i++) {
            const bool top = i == A.size() - 1;
            const uint32_t c = (signed_ && top) ? PF_B_SLT : PF_B_ULT;
            const int32_t x = A[i].first, y = B[i].first;
            const uint32_t wx = A[i].second;
            int32_t li = d.op(c, wx, {x, y});
            if (lt >= 0) li = d.op(PF_B_OR, 1, {li, d.op(PF_B_AND, 1, {d.op(PF_B_EQ, wx, {x, y}), lt})});
            lt = li;
        }
        if (strict) return lt;
        return d.op(PF_B_NOT, 1, {wide_cmp(signed_ ? PFLT_BVSLT : PFLT_BVULT, bt, a)});
    }

    Val lower_wide(uint32_t t) {
        const TermRec& r = T(t);
        const uint32_t wd = width(t);
        if (r.op == T_CONCAT || r.op == T_ZEXT || r.op == T_BV) return VW(chunks(t));
        if (r.op == T_VAR) {
            Chunks out;
            uint32_t lo = 0;
            auto pit = par_name.find(r.name);
            const bool hp = pit != par_name.end();
            while (lo < wd) {
                const uint32_t cw = std::min<uint32_t>(256, wd - lo);
                C8 pv;
                if (hp) pv = c8_of(shr_big(pit->second, lo), cw);
                char nm[32];
                snprintf(nm, sizeof(nm), "#%u", lo / 256);
                VarTerm vt{PFLT_VT_EXTRACT, t, lo, lo + cw - 1};
                out.push_back({mkvar(r.name + nm, cw, vt, hp ? &pv : nullptr, nullptr), cw});
                lo += cw;
            }
            return VW(out);
        }
        if (r.op == T_APPLY) return apply(t);
        if (r.op == T_ITE) {
            const int32_t c = b(r.args[0]);
            const Chunks a = chunks(r.args[1]), bb = chunks(r.args[2]);
            Chunks out;
            for (size_t i = 0; i < std::min(a.size(), bb.size()); i++)
                out.push_back({d.op(PF_W_ITE, a[i].second, {c, a[i].first, bb[i].first}), a[i].second});
            return VW(out);
        }
        if (r.op == T_EXTRACT) return VW(slice(chunks(r.args[0]), (uint32_t)r.i1, wd));
        if (r.op == PFLT_BVADD || r.op == PFLT_BVSUB) {
            const Chunks A = chunks(r.args[0]);  // operands in order (node numbering)
            const Chunks B = chunks(r.args[1]);
            return VW(wide_addsub(A, B, r.op == PFLT_BVSUB));
        }
        if (r.op == T_BVNEG) {
            const Chunks A = chunks(r.args[0]);
            Chunks zero;
            for (const auto& c : A) zero.push_back({d.cnst(0, c.second), c.second});
            return VW(wide_addsub(zero, A, true));
        }
        if (r.op == PFLT_BVAND || r.op == PFLT_BVOR || r.op == PFLT_BVXOR) {
            const uint32_t opc = r.op == PFLT_BVAND ? PF_W_AND : (r.op == PFLT_BVOR ? PF_W_OR : PF_W_XOR);
            const Chunks A = chunks(r.args[0]), B = chunks(r.args[1]);
            Chunks out;
            for (size_t i = 0; i < std::min(A.size(), B.size()); i++)
                out.push_back({d.op(opc, A[i].second, {A[i].first, B[i].first}), A[i].second});
            return VW(out);
        }
        if (r.op == T_BVNOT) {
            Chunks out;
            for (const auto& c : chunks(r.args[0])) out.push_back({d.op(PF_W_NOT, c.second, {c.first}), c.second});
            return VW(out);
        }
        if ((r.op == PFLT_BVSHL || r.op == PFLT_BVLSHR) && T(r.args[1]).op == T_BV) {
            const Big& kb = T(r.args[1]).val;
            if (bitlen(kb) > 31 || limb(kb, 0) >= wd) return VW(rechunk(const_pieces(Big{}, wd)));
            const uint32_t k = limb(kb, 0);
            const Chunks A = chunks(r.args[0]);
            Chunks zeros;
            if (k) zeros = rechunk(const_pieces(Big{}, k));
            Chunks cat;
            if (r.op == PFLT_BVSHL) {
                cat = zeros;
                const Chunks s = slice(A, 0, wd - k);
                cat.insert(cat.end(), s.begin(), s.end());
            } else {
                cat = slice(A, k, wd - k);
                cat.insert(cat.end(), zeros.begin(), zeros.end());
            }
            return VW(rechunk(cat));
        }
        lerr("%u-bit %s", wd, r.name.empty() ? "op" : r.name.c_str());
    }

    // ExplicitLowering._lshr_concat: bvlshr(concat(p0 .. pn-1), k) without the low parts the
    // shift discards whole — concat(p0 .. pj) >> (k - their width), zero-extended to wd
    bool lshr_concat(const std::vector<uint32_t>& parts, const Big& kv, uint32_t wd, int32_t* out) {
        uint64_t k = (uint64_t)limb(kv, 0) | ((uint64_t)limb(kv, 1) << 32);
        for (size_t i = 2; i < kv.size(); i++)
            if (kv[i]) k = UINT64_MAX;  // past any width
        size_t j = parts.size();
        uint64_t drop = 0;
        while (j > 1 && drop + width(parts[j - 1]) <= k) {
            drop += width(parts[j - 1]);
            j--;
        }
        if (j == parts.size()) return false;
        int32_t hi = node(parts[0]);
        uint32_t hw = width(parts[0]);
        for (size_t i = 1; i < j; i++) {
            const uint32_t pw = width(parts[i]);
            hi = d.op(PF_W_CONCAT, hw + pw, {hi, node(parts[i])}, pw);
            hw += pw;
        }
        const uint64_t rem = k - drop;
        if (rem >= hw) {
            *out = d.cnst((uint64_t)0, wd);
            return true;
        }
        if (rem) hi = d.op(PF_W_LSHR, hw, {hi, d.cnst(rem, hw)});
        *out = d.op(PF_W_MOV, wd, {hi});
        return true;
    }

    Val lower_bv(uint32_t t) {
        const TermRec& r = T(t);
        const uint32_t wd = width(t);
        if (wd > 256) return lower_wide(t);
        if (r.op == T_BV) return V(d.cnst(c8_of(r.val, wd), wd));
        if (r.op == T_VAR) return V(mkvar(r.name, wd, VarTerm{PFLT_VT_TERM, t, 0, 0}, nullptr, nullptr));
        if (explicit_ && r.op == PFLT_BVLSHR && T(r.args[1]).op == T_BV && T(r.args[0]).op == T_CONCAT) {
            int32_t nd;
            if (lshr_concat(T(r.args[0]).args, T(r.args[1]).val, wd, &nd)) return V(nd);
        }
        if (const uint32_t opc = wbin_op(r.op)) return V(d.op(opc, wd, {node(r.args[0]), node(r.args[1])}));
        if (r.op == T_BVNOT) return V(d.op(PF_W_NOT, wd, {node(r.args[0])}));
        if (r.op == T_BVNEG) return V(d.op(PF_W_NEG, wd, {node(r.args[0])}));
        if (r.op == T_EXTRACT) {
            const uint32_t lo = (uint32_t)r.i1, src = r.args[0];
            if (width(src) <= 256) return V(d.op(PF_W_EXTRACT, wd, {node(src)}, lo));
            const Chunks s = slice(chunks(src), lo, wd);
            return V(s[0].first);
        }
        if (r.op == T_CONCAT) {
            int32_t nd = node(r.args[0]);
            uint32_t acc = width(r.args[0]);
            for (size_t i = 1; i < r.args.size(); i++) {
                const uint32_t pw = width(r.args[i]);
                nd = d.op(PF_W_CONCAT, acc + pw, {nd, node(r.args[i])}, pw);
                acc += pw;
            }
            return V(nd);
        }
        if (r.op == T_ZEXT) return V(d.op(PF_W_MOV, wd, {node(r.args[0])}));
        if (r.op == T_ITE) {
            const int32_t c = b(r.args[0]);
            const int32_t x = node(r.args[1]);
            const int32_t y = node(r.args[2]);
            return V(d.op(PF_W_ITE, wd, {c, x, y}));
        }
        if (r.op == T_SELECT) return V(select(r.args[0], r.args[1]));
        if (r.op == T_APPLY) return apply(t);
        lerr("unsupported bit-vector op %s", r.name.c_str());
    }

    int32_t lower_bool(uint32_t t) {
        const TermRec& r = T(t);
        switch (r.op) {
            case T_TRUE: return d.bconst(true);
            case T_FALSE: return d.bconst(false);
            case T_BVAR: {
                auto it = par_name.find(r.name);
                C8 pv;
                const bool hp = it != par_name.end();
                if (hp) pv = c8_of(it->second, 1);
                bool created;
                const int32_t nd = d.var(r.name, 1, PF_VK_BOOL, 0, 0, hp, pv, &created);
                if (created) var_terms.push_back(VarTerm{PFLT_VT_TERM, t, 0, 0});
                return nd;
            }
            case T_NOT: return d.op(PF_B_NOT, 1, {b(r.args[0])});
            case T_AND:
            case T_OR: {
                const uint32_t opc = r.op == T_AND ? PF_B_AND : PF_B_OR;
                int32_t acc = b(r.args[0]);
                for (size_t i = 1; i < r.args.size(); i++) acc = d.op(opc, 1, {acc, b(r.args[i])});
                return acc;
            }
            case T_XOR: {
                const int32_t x = b(r.args[0]);
                return d.op(PF_B_XOR, 1, {x, b(r.args[1])});
            }
            case T_IFF: {
                const int32_t x = b(r.args[0]);
                return d.op(PF_B_NOT, 1, {d.op(PF_B_XOR, 1, {x, b(r.args[1])})});
            }
            case T_ITE: {
                const int32_t c = b(r.args[0]);
                const int32_t x = b(r.args[1]);
                return d.op(PF_B_ITE, 1, {c, x, b(r.args[2])});
            }
            case T_EQ: {
                const uint32_t a = r.args[0], bt = r.args[1];
                if (width(a) > 256 || width(bt) > 256) {
                    const Chunks ca = chunks(a), cb = chunks(bt);
                    int32_t acc = -1;
                    for (size_t i = 0; i < std::min(ca.size(), cb.size()); i++) {
                        const int32_t e = d.op(PF_B_EQ, ca[i].second, {ca[i].first, cb[i].first});
                        acc = acc < 0 ? e : d.op(PF_B_AND, 1, {acc, e});
                    }
                    return acc;
                }
                const int32_t x = node(a);
                return d.op(PF_B_EQ, width(a), {x, node(bt)});
            }
            default: break;
        }
        if (const uint32_t opc = bcmp_op(r.op)) {
            const uint32_t a = r.args[0], bt = r.args[1];
            if (width(a) > 256 && (r.op == PFLT_BVULT || r.op == PFLT_BVULE || r.op == PFLT_BVSLT ||
                                   r.op == PFLT_BVSLE))
                return wide_cmp(r.op, a, bt);
            const int32_t x = node(a);
            return d.op(opc, width(a), {x, node(bt)});
        }
        lerr("unsupported bool op %s", r.name.c_str());
    }

    // ---- arrays -----------------------------------------------------------------------
    // (base, c) with t = base + c mod 2^w, constant additions / subtractions peeled off
    // (base NO_BASE for a constant): TermLowering._offset_form — indices with one base and
    // different offsets never alias
    static constexpr uint32_t NO_BASE = 0xffffffffu;
    // memoised per term: select() asks for every earlier entry's form on every read
    mutable std::unordered_map<uint32_t, std::pair<uint32_t, C8>> of_memo;
    std::pair<uint32_t, C8> offset_form(uint32_t t) const {
        auto it = of_memo.find(t);
        if (it != of_memo.end()) return it->second;
        return of_memo.emplace(t, offset_form_of(t)).first->second;
    }
    std::pair<uint32_t, C8> offset_form_of(uint32_t t) const {
        const uint32_t w = width(t);
        uint32_t c[8] = {0};
        auto addsub = [&](const Big& v, bool sub) {
            const C8 x = c8_of(v, 256);
            uint64_t carry = sub ? 1 : 0;
            for (int i = 0; i < 8; i++) {
                const uint64_t s = (uint64_t)c[i] + (sub ? (uint32_t)~x.l[i] : x.l[i]) + carry;
                c[i] = (uint32_t)s;
                carry = s >> 32;
            }
        };
        for (;;) {
            const TermRec& r = T(t);
            if (r.op == T_BV) {
                addsub(r.val, false);
                return {NO_BASE, c8_of(Big(c, c + 8), w)};
            }
            if (r.op == PFLT_BVADD && r.args.size() == 2) {
                if (T(r.args[1]).op == T_BV) {
                    addsub(T(r.args[1]).val, false);
                    t = r.args[0];
                    continue;
                }
                if (T(r.args[0]).op == T_BV) {
                    addsub(T(r.args[0]).val, false);
                    t = r.args[1];
                    continue;
                }
            } else if (r.op == PFLT_BVSUB && r.args.size() == 2 && T(r.args[1]).op == T_BV) {
                addsub(T(r.args[1]).val, true);
                t = r.args[0];
                continue;
            }
            return {t, c8_of(Big(c, c + 8), w)};
        }
    }

    int32_t select(uint32_t arr, uint32_t idx) {
        const TermRec& A = T(arr);
        if (A.op == T_STORE) {
            const uint32_t base = A.args[0], k = A.args[1], v = A.args[2];
            if (k == idx) return node(v);
            const auto kf = offset_form(k), xf = offset_form(idx);
            if (kf.first == xf.first)  // the same base: the offsets decide
                return kf.second == xf.second ? node(v) : select(base, idx);
            const int32_t rest = select(base, idx);
            const int32_t c = d.op(PF_B_EQ, width(idx), {node(idx), node(k)});
            return d.op(PF_W_ITE, A.w2, {c, node(v), rest});
        }
        if (A.op == T_K) return node(A.args[0]);
        if (A.op == T_ITE) {
            const int32_t c = b(A.args[0]);
            const int32_t x = select(A.args[1], idx);
            const int32_t y = select(A.args[2], idx);
            return d.op(PF_W_ITE, A.w2, {c, x, y});
        }
        if (A.op != T_ARRAY) lerr("select over %s", A.name.c_str());
        const std::string& name = A.name;
        const uint32_t rng = A.w2;
        if (width(idx) > 256) lerr("array index wider than 256 bits");
        if (explicit_) return leaf_read(arr, idx, rng);
        auto it = arrays.find(name);
        if (it == arrays.end()) {
            array_order.push_back(name);
            it = arrays.emplace(name, std::vector<std::array<int32_t, 4>>()).first;
        }
        for (const auto& e : it->second)
            if ((uint32_t)e[0] == idx) return e[3];
        const int32_t inode = node(idx);
        std::string vname;
        if (T(idx).op == T_BV) {
            // f"{name}[{idx.val}]": the index in decimal
            vname = name + "[" + big_decimal(T(idx).val) + "]";
        } else {
            vname = name + "@" + std::to_string(arrays[name].size());
        }
        const std::pair<uint32_t, uint32_t> rd{arr, idx};
        int32_t val = mkvar(vname, rng, VarTerm{PFLT_VT_SELECT, arr, idx, 0}, nullptr, &rd);
        auto& entries = arrays[name];
        const auto xf = offset_form(idx);
        // runs: entries next to each other in lookup order with one base other than idx's
        // (constants: NO_BASE) — distinct offsets, so at most one of them can match
        std::vector<RunEntry> run;
        uint32_t run_base = 0;
        for (size_t i = entries.size(); i-- > 0;) {
            const auto& e = entries[i];
            const auto ef = offset_form((uint32_t)e[0]);
            if (ef.first == xf.first && !(ef.second == xf.second)) continue;  // never aliases
            if (ef.first == xf.first) {
                val = index_run(run, run_base, idx, inode, rng, val);
                run.clear();
                val = d.op(PF_W_ITE, rng, {d.op(PF_B_EQ, width(idx), {inode, e[2]}), e[3], val});
                continue;
            }
            if (!run.empty() && ef.first != run_base) {
                val = index_run(run, run_base, idx, inode, rng, val);
                run.clear();
            }
            run_base = ef.first;
            run.push_back({ef.second, e[2], e[3]});
        }
        val = index_run(run, run_base, idx, inode, rng, val);
        entries.push_back({(int32_t)idx, (int32_t)arr, inode, val});
        return val;
    }

    // TermLowering._run / _window: a run of indices base + c of a byte array, contiguous in
    // 8..32-long pieces, read through one window lookup per piece; short runs and pieces
    // stay ite(idx == base + c, v_c, ...) chains in lookup order
    struct RunEntry {
        C8 c;
        int32_t inn, v;
    };
    static constexpr size_t WINDOW_MIN = 8;
    static bool c8_less(const C8& a, const C8& b) {
        for (int i = 7; i >= 0; i--)
            if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
        return false;
    }
    static bool c8_succ(const C8& a, const C8& b) {  // b == a + 1 (no wrap: b > a)
        C8 x = a;
        for (int i = 0; i < 8; i++)
            if (++x.l[i] != 0) break;
        return x == b && c8_less(a, b);
    }
    int32_t index_run(const std::vector<RunEntry>& run, uint32_t base, uint32_t idx, int32_t inode, uint32_t rng,
                      int32_t val) {
        auto chain = [&]() {
            for (const RunEntry& e : run)
                val = d.op(PF_W_ITE, rng, {d.op(PF_B_EQ, width(idx), {inode, e.inn}), e.v, val});
            return val;
        };
        if (run.size() < WINDOW_MIN || rng != 8 || width(idx) != 256) return chain();
        bool dup = false;
        std::vector<RunEntry> items(run);
        std::stable_sort(items.begin(), items.end(),
                         [](const RunEntry& a, const RunEntry& b) { return c8_less(a.c, b.c); });
        for (size_t i = 1; i < items.size(); i++) dup |= items[i].c == items[i - 1].c;
        if (dup) return chain();
        size_t i = 0;
        while (i < items.size()) {
            size_t j = i + 1;
            while (j < items.size() && c8_succ(items[j - 1].c, items[j].c) && j - i < 32) j++;
            if (j - i < WINDOW_MIN) {
                for (size_t k = i; k < j; k++)
                    val = d.op(PF_W_ITE, rng, {d.op(PF_B_EQ, width(idx), {inode, items[k].inn}), items[k].v, val});
            } else {
                val = window(items, i, j, base == NO_BASE, inode, val);
            }
            i = j;
        }
        return val;
    }
    int32_t window(const std::vector<RunEntry>& items, size_t i, size_t j, bool const_base, int32_t inode,
                   int32_t val) {
        const uint32_t n = (uint32_t)(j - i);
        int32_t acc = items[i].v;
        for (uint32_t k = 1; k < n; k++) acc = d.op(PF_W_CONCAT, 8 * (k + 1), {items[i + k].v, acc}, 8 * k);
        const C8& lo = items[i].c;
        bool lo_zero = true;
        for (int k = 0; k < 8; k++) lo_zero &= lo.l[k] == 0;
        // idx - (base + lo): the piece's lowest index node
        const int32_t t = const_base && lo_zero ? inode : d.op(PF_W_SUB, 256, {inode, items[i].inn});
        const int32_t hit = d.op(PF_B_ULT, 256, {t, d.cnst(n, 256)});
        const int32_t amt = d.op(PF_W_EXTRACT, 8 * n, {d.op(PF_W_SHL, 256, {t, d.cnst(3, 256)})}, 0);
        const int32_t byte = d.op(PF_W_EXTRACT, 8, {d.op(PF_W_LSHR, 8 * n, {acc, amt})}, 0);
        return d.op(PF_W_ITE, 8, {hit, byte, val});
    }

    static std::string big_decimal(const Big& v) {
        Big x = v;
        while (!x.empty() && x.back() == 0) x.pop_back();
        if (x.empty()) return "0";
        std::string s;
        while (!x.empty()) {
            uint64_t rem = 0;
            for (size_t i = x.size(); i-- > 0;) {
                const uint64_t cur = (rem << 32) | x[i];
                x[i] = (uint32_t)(cur / 10);
                rem = cur % 10;
            }
            s.push_back((char)('0' + rem));
            while (!x.empty() && x.back() == 0) x.pop_back();
        }
        std::reverse(s.begin(), s.end());
        return s;
    }

    // ---- uninterpreted functions ---------------------------------------------------------
    int32_t hash_args(const std::vector<uint32_t>& args, uint32_t salt) {
        int32_t h = -1;
        for (uint32_t a : args) {
            for (const auto& c : chunks(a)) {
                const int32_t x = c.second == 256 ? c.first : d.op(PF_W_MOV, 256, {c.first});
                h = d.op(PF_W_HASH, 256, {h < 0 ? x : d.op(PF_W_XOR, 256, {h, x})}, salt);
            }
        }
        return h;
    }

    static bool keccak_name(const std::string& f, uint32_t* n, bool* inv) {
        static const char pre[] = "keccak256_";
        if (f.compare(0, sizeof(pre) - 1, pre) != 0) return false;
        size_t i = sizeof(pre) - 1, j = i;
        while (j < f.size() && isdigit((unsigned char)f[j])) j++;
        if (j == i) return false;
        *n = (uint32_t)strtoul(f.c_str() + i, nullptr, 10);
        if (j == f.size()) {
            *inv = false;
            return true;
        }
        if (f.compare(j, std::string::npos, "-1") == 0) {
            *inv = true;
            return true;
        }
        return false;
    }

    // ---- explicit-model leaves (ExplicitLowering._leaf / _select / _apply) ----------------
    int32_t leaf_var(uint32_t w, const VarTerm& vt) {
        return mkvar("@leaf" + std::to_string(n_leaves++), w, vt, nullptr, nullptr);
    }

    int32_t leaf_read(uint32_t arr, uint32_t idx, uint32_t rng) {
        const auto key = std::make_pair(arr, idx);
        auto it = leaf_reads.find(key);
        if (it != leaf_reads.end()) return it->second;
        const int32_t n = leaf_var(rng, VarTerm{PFLT_VT_SELECT, arr, idx, 0});
        leaf_reads.emplace(key, n);
        return n;
    }

    Val leaf_apply(uint32_t t) {
        const uint32_t wd = width(t);
        if (wd <= 256) {
            auto it = leaf_apps.find(t);
            if (it != leaf_apps.end()) return V(it->second);
            const int32_t n = leaf_var(wd, VarTerm{PFLT_VT_TERM, t, 0, 0});
            leaf_apps.emplace(t, n);
            return V(n);
        }
        Chunks out;  // one leaf per 256-bit chunk, recorded as its extract term
        for (uint32_t lo = 0; lo < wd; lo += 256) {
            const uint32_t cw = std::min<uint32_t>(256, wd - lo);
            out.push_back({leaf_var(cw, VarTerm{PFLT_VT_EXTRACT, t, lo, lo + cw - 1}), cw});
        }
        return VW(out);
    }

    Val apply(uint32_t t) {
        if (explicit_) return leaf_apply(t);
        const TermRec& r = T(t);
        uint32_t n;
        bool inv;
        if (keccak_name(r.name, &n, &inv)) {
            if (!inv) return V(keccak(n, r.args[0], t));
            return keccak_inv(n, r.args[0], t);
        }
        if (r.name == "Power" && r.args.size() == 2 && width(t) == 256) return V(power(t));
        uf_apps.push_back(t);
        const int32_t h = hash_args(r.args, crc32_of(r.name));
        return V(width(t) == 256 ? h : d.op(PF_W_EXTRACT, width(t), {h}, 0));
    }

    int32_t eq_terms_const(uint32_t a, const Big& c) {  // _eq_value(a, c) = _eq_terms(a, const(c))
        const uint32_t wa = width(a);
        if (wa <= 256) {
            const int32_t x = node(a);
            return d.op(PF_B_EQ, wa, {x, d.cnst(c8_of(c, wa), wa)});
        }
        const Chunks A = chunks(a);
        const Chunks B = rechunk(const_pieces(mask_big(c, wa), wa));
        int32_t acc = -1;
        for (size_t i = 0; i < std::min(A.size(), B.size()); i++) {
            const int32_t e = d.op(PF_B_EQ, A[i].second, {A[i].first, B[i].first});
            acc = acc < 0 ? e : d.op(PF_B_AND, 1, {acc, e});
        }
        return acc;
    }

    int32_t eq_terms(uint32_t a, uint32_t bt) {
        if (width(a) != width(bt)) return d.bconst(false);
        if (width(a) <= 256) {
            const int32_t x = node(a);
            return d.op(PF_B_EQ, width(a), {x, node(bt)});
        }
        const Chunks A = chunks(a), B = chunks(bt);
        int32_t acc = -1;
        for (size_t i = 0; i < std::min(A.size(), B.size()); i++) {
            const int32_t e = d.op(PF_B_EQ, A[i].second, {A[i].first, B[i].first});
            acc = acc < 0 ? e : d.op(PF_B_AND, 1, {acc, e});
        }
        return acc;
    }

    int32_t keccak(uint32_t n, uint32_t arg, uint32_t t) {
        auto& apps = keccak_apps[n];
        for (const auto& a : apps)
            if (a.first == arg) return a.second;
        const int32_t h = hash_args({arg}, crc32_of("keccak256_" + std::to_string(n)));
        int32_t val = h;
        auto sit = kspecs.find(n);
        if (sit != kspecs.end()) {
            const KSpec& spec = sit->second;
            if (spec.has_lo) {
                Big m117;
                for (int i = 0; i < 4; i++) m117.push_back(i < 3 ? 0xffffffffu : (1u << 21) - 1u);
                const int32_t k = d.op(PF_W_AND, 256, {h, d.cnst(c8_of(m117, 256), 256)});
                val = d.op(PF_W_ADD, 256, {d.cnst(spec.base, 256), d.op(PF_W_SHL, 256, {k, d.cnst(6, 256)})});
            }
            for (const auto& ck : spec.concrete) {
                const int32_t eqs = eq_terms_const(arg, ck.first);
                val = d.op(PF_W_ITE, 256, {eqs, d.cnst(ck.second, 256), val});
            }
        }
        // injectivity on the set: f(a) = f(b) -> a = b
        for (const auto& a : apps) {
            const int32_t same_f = d.op(PF_B_EQ, 256, {val, a.second});
            const int32_t same_x = eq_terms(arg, a.first);
            side.push_back(d.op(PF_B_OR, 1, {d.op(PF_B_NOT, 1, {same_f}), same_x}));
        }
        keccak_apps[n].push_back({arg, val});
        uf_apps.push_back(t);
        return val;
    }

    Val keccak_inv(uint32_t n, uint32_t y, uint32_t t) {
        const TermRec& Y = T(y);
        uint32_t yn;
        bool yinv;
        if (Y.op == T_APPLY && keccak_name(Y.name, &yn, &yinv) && !yinv && yn == n) {
            w(y);  // make sure f(x) is registered (injectivity constraints)
            return w(Y.args[0]);
        }
        if (n > 256) lerr("inverse keccak of a wide input on a non-application");
        const int32_t ynode = node(y);
        const std::string vname = "keccak256_" + std::to_string(n) + "-1@" + std::to_string(inv_apps[n].size());
        int32_t val = mkvar(vname, n, VarTerm{PFLT_VT_TERM, t, 0, 0}, nullptr, nullptr);
        auto& entries = inv_apps[n];
        for (size_t i = entries.size(); i-- > 0;)
            val = d.op(PF_W_ITE, n, {d.op(PF_B_EQ, 256, {ynode, entries[i].first}), entries[i].second, val});
        auto kit = keccak_apps.find(n);
        if (kit != keccak_apps.end()) {
            const auto& ka = kit->second;
            for (size_t i = ka.size(); i-- > 0;) {
                const int32_t eq = d.op(PF_B_EQ, 256, {ynode, ka[i].second});
                val = d.op(PF_W_ITE, n, {eq, node(ka[i].first), val});
            }
        }
        inv_apps[n].push_back({ynode, val});
        uf_apps.push_back(t);
        return V(val);
    }

    int32_t power(uint32_t t) {
        const TermRec& r = T(t);
        const uint32_t bt = r.args[0], et = r.args[1];
        for (const auto& pa : power_apps)
            if (std::get<0>(pa) == bt && std::get<1>(pa) == et) return std::get<2>(pa);
        int32_t val;
        const bool sym = !(T(bt).op == T_BV && T(et).op == T_BV);
        if (!sym) {
            val = d.cnst(pow8(c8_of(T(bt).val, 256), c8_of(T(et).val, 256)), 256);
        } else {
            const int32_t bn = node(bt), en = node(et);
            size_t nsym = 0;
            for (const auto& pa : power_apps) nsym += std::get<3>(pa) ? 1 : 0;
            val = mkvar("Power@" + std::to_string(nsym), 256, VarTerm{PFLT_VT_TERM, t, 0, 0}, nullptr, nullptr);
            for (size_t i = power_apps.size(); i-- > 0;) {
                const auto& pa = power_apps[i];
                if (!std::get<3>(pa)) continue;
                const int32_t e1 = d.op(PF_B_EQ, 256, {bn, node(std::get<0>(pa))});
                const int32_t same = d.op(PF_B_AND, 1, {e1, d.op(PF_B_EQ, 256, {en, node(std::get<1>(pa))})});
                val = d.op(PF_W_ITE, 256, {same, std::get<2>(pa), val});
            }
            const int32_t one = d.cnst(1, 256);  // Python's argument order: 1 first
            const int32_t sh = d.op(PF_W_SHL, 256, {d.op(PF_W_AND, 256, {en, d.cnst(31, 256)}), d.cnst(3, 256)});
            const int32_t rule = d.op(PF_W_SHL, 256, {one, sh});
            val = d.op(PF_W_ITE, 256, {d.op(PF_B_EQ, 256, {bn, d.cnst(256, 256)}), rule, val});
            for (const auto& f : power_facts) {
                const int32_t e1 = d.op(PF_B_EQ, 256, {bn, d.cnst(f.first.first, 256)});
                const int32_t same = d.op(PF_B_AND, 1, {e1, d.op(PF_B_EQ, 256, {en, d.cnst(f.first.second, 256)})});
                val = d.op(PF_W_ITE, 256, {same, d.cnst(f.second, 256), val});
            }
        }
        power_apps.emplace_back(bt, et, val, sym);
        uf_apps.push_back(t);
        return val;
    }

    void collect_power_facts(const std::vector<uint32_t>& roots) {
        std::vector<uint32_t> stack(roots.begin(), roots.end());
        std::vector<char> seen(S.t.size(), 0);
        while (!stack.empty()) {
            const uint32_t x = stack.back();
            stack.pop_back();
            if (seen[x]) continue;
            seen[x] = 1;
            const TermRec& r = T(x);
            if (r.op == T_APPLY && r.name == "Power" && r.args.size() == 2 && T(r.args[0]).op == T_BV &&
                T(r.args[1]).op == T_BV) {
                const C8 c1 = c8_of(T(r.args[0]).val, 256), c2 = c8_of(T(r.args[1]).val, 256);
                const C8 pv = pow8(c1, c2);
                bool found = false;
                for (auto& f : power_facts)
                    if (f.first.first == c1 && f.first.second == c2) {
                        f.second = pv;
                        found = true;
                    }
                if (!found) power_facts.push_back({{c1, c2}, pv});
            }
            for (uint32_t a : r.args) stack.push_back(a);
        }
    }

    void lower(const std::vector<uint32_t>& roots) {
        if (!explicit_) collect_power_facts(roots);
        for (uint32_t c : roots) {
            if (T(c).sortk != 0) lerr("constraint is not a Bool");
            if (T(c).op == T_TRUE) continue;
            const int32_t r = b(c);
            if (!d.nodes[r].is_bool) lerr("root is not a Bool");
            d.roots.push_back(r);
        }
        for (int32_t s : side) d.roots.push_back(s);
    }
};

// ---- results ------------------------------------------------------------------------------
struct Result {
    Dag dag;
    std::vector<VarTerm> var_terms;
    std::vector<uint32_t> uf_apps;
    std::vector<uint32_t> reads;   // (array id, index id) pairs, arrays in insertion order
    std::vector<uint32_t> read_counts;  // entries per array, same order
    std::vector<uint32_t> code;    // n_ins x 4
    std::vector<uint32_t> consts;  // n_const x 8
    std::vector<uint32_t> packed_nodes, pool;  // pack_nodes of the DAG (tests)
    std::string names;             // variable names, '\0'-separated
    uint32_t n_wregs = 0;
    int n_sat = 0;
    int rc = 0;                    // 0, or the failure code (-2 LoweringError -> z3, -1 / -3 ...)
    std::string err;               // the failure message
    std::vector<uint32_t> in_roots;  // the bucket's conjuncts (the re-check's roots)
    bool parented = false;         // a parent model seeded some variable
};

void pack(const Dag& d, std::vector<uint32_t>* nodes, std::vector<uint32_t>* pool) {
    nodes->clear();
    pool->clear();
    uint32_t np = 0;
    for (const DNode& n : d.nodes) {
        uint32_t aux = n.aux;
        if (n.kind == K_CONST) {
            aux = np++;
            pool->insert(pool->end(), n.cv.l, n.cv.l + 8);
        }
        const uint32_t a0 = n.nargs > 0 ? (uint32_t)n.args[0] : 0u, a1 = n.nargs > 1 ? (uint32_t)n.args[1] : 0u,
                       a2 = n.nargs > 2 ? (uint32_t)n.args[2] : 0u;
        const uint32_t rec[8] = {n.kind, n.width, n.nargs, a0, a1, a2, aux, n.is_bool ? 1u : 0u};
        nodes->insert(nodes->end(), rec, rec + 8);
    }
    if (nodes->empty()) nodes->assign(8, 0u);
}

// parent values: per name its limb count then the limbs (any width); reads (array id,
// index id) with 8 limbs each
void fill_parents(Parents* P, const char* par_names, const uint32_t* par_name_vals, size_t n_par_names,
                  const uint32_t* par_reads, const uint32_t* par_read_vals, size_t n_par_reads) {
    const char* nm = par_names;
    const uint32_t* pv = par_name_vals;
    for (size_t i = 0; i < n_par_names; i++) {
        const uint32_t nl = *pv++;
        P->set_name(std::string(nm), Big(pv, pv + nl));
        pv += nl;
        nm += strlen(nm) + 1;
    }
    for (size_t i = 0; i < n_par_reads; i++) {
        C8 c;
        memcpy(c.l, par_read_vals + 8 * i, 32);
        P->set_read(std::make_pair(par_reads[2 * i], par_reads[2 * i + 1]), c);
    }
}

// Register allocation + emission of a finished DAG into R (lower.lower(dag): narrow register
// file first, wide when the narrow program is spill-heavy and the wide one at least halves
// its spill code).  Throws TermError like the lowering.
void emit_program(Dag& d, Result* R) {
    d.finalize_word_hints();
    pack(d, &R->packed_nodes, &R->pool);
    std::vector<uint32_t> forced;
    for (const C8& c : d.forced) forced.insert(forced.end(), c.l, c.l + 8);
    std::vector<uint32_t> roots2(d.roots.begin(), d.roots.end());
    if (roots2.empty()) roots2.push_back(0);
    const uint32_t tries[2] = {PF_NW_NARROW, PF_NW};
    int rc = -2;
    // the narrow program unless its spill code exceeds an eighth of it and the wide
    // register file at least halves that (lower.py lower(): the same policy)
    bool have_narrow = false;
    std::vector<uint32_t> n_code, n_consts;
    size_t n_spill_narrow = 0;
    // output scratch per thread, grown but never cleared (pfl_lower writes what it
    // reports); the result keeps only the words written
    thread_local std::vector<uint32_t> code_buf, const_buf;
    for (int ti = 0; ti < 2; ti++) {
        size_t cap_i = 16 * d.nodes.size() + 64 + 4 * d.roots.size();
        size_t cap_c = R->pool.size() / 8 + d.forced.size() + 1;
        size_t ni = 0, nc = 0;
        for (int attempt = 0; attempt < 4; attempt++) {
            if (code_buf.size() < 4 * cap_i) code_buf.resize(4 * cap_i);
            if (const_buf.size() < 8 * cap_c) const_buf.resize(8 * cap_c);
            rc = pfl_lower(R->packed_nodes.data(), d.nodes.size(), R->pool.data(), R->pool.size() / 8,
                           roots2.data(), d.roots.size(), forced.empty() ? nullptr : forced.data(),
                           d.forced.size(), tries[ti], code_buf.data(), cap_i, &ni, const_buf.data(),
                           cap_c, &nc);
            if (rc != -3) break;
            cap_i *= 4;
            cap_c *= 4;
        }
        if (rc == 0) {
            R->code.assign(code_buf.begin(), code_buf.begin() + 4 * ni);
            R->consts.assign(const_buf.begin(), const_buf.begin() + 8 * nc);
            size_t n_spill = 0;
            for (size_t i = 0; i < ni; i++) {
                const uint32_t op = R->code[4 * i] & 0xffu;
                n_spill += op == PF_W_SPILL || op == PF_W_FILL;
            }
            R->n_wregs = tries[ti];
            if (ti == 0 && 8 * n_spill > ni) {  // spill-heavy: try the wide register file
                have_narrow = true;
                n_code.swap(R->code);
                n_consts.swap(R->consts);
                n_spill_narrow = n_spill;
                continue;
            }
            if (ti == 1 && have_narrow && 2 * n_spill > n_spill_narrow) {
                R->code.swap(n_code);
                R->consts.swap(n_consts);
                R->n_wregs = tries[0];
            }
            break;
        }
        if (ti == 1 && have_narrow) {  // the wide lowering failed (any rc): keep the narrow one
            R->code.swap(n_code);
            R->consts.swap(n_consts);
            R->n_wregs = tries[0];
            rc = 0;
            break;
        }
        if (rc != -2) break;
    }
    if (rc != 0) {
        t_err = pfl_last_error();
        throw TermError{rc};
    }
}

// One bucket: terms -> DAG -> hints -> program (pflt_lower).  Reads the store only, so
// buckets lower concurrently (pflt_lower_many).  Never throws: a failure is R->rc / R->err.
#ifdef PFLT_PROFILE
// phase timers of lower_job (profiling builds only, tools/lower_profile.py): ns per phase,
// summed over every job, printed at exit
#include <atomic>
#include <chrono>
static std::atomic<uint64_t> g_prof_ns[6];
static const char* g_prof_names[6] = {"setup", "term->dag", "hints", "emit", "result", "jobs"};
struct ProfPrint {
    ~ProfPrint() {
        for (int i = 0; i < 6; i++) fprintf(stderr, "pflt_prof %s %llu\n", g_prof_names[i], (unsigned long long)g_prof_ns[i].load());
    }
} g_prof_print;
static inline uint64_t prof_now() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define PROF_LAP(k) do { const uint64_t t_ = prof_now(); g_prof_ns[k] += t_ - t_lap; t_lap = t_; } while (0)
#else
#define PROF_LAP(k) ((void)0)
#endif
Result* lower_job(const Store& S, const std::vector<uint32_t>& rs, const Parents& P, const uint32_t* registry,
                  size_t n_registry, uint32_t flags) {
#ifdef PFLT_PROFILE
    uint64_t t_lap = prof_now();
    g_prof_ns[5] += 1;
#endif
    Result* R = new Result();
    R->in_roots = rs;
    R->parented = !P.empty();
    try {
        Lowering L(S, P);
        L.explicit_ = (flags & PFLT_EXPLICIT) != 0;
        // registry: n_actors, actors x 8; n_specs; per spec: n, has_lo, base x 8, n_concrete,
        // per concrete: value limbs (ceil(n / 32)), digest x 8
        size_t p = 0;
        auto take = [&](void) -> uint32_t {
            if (p >= n_registry) lerr("registry blob truncated");
            return registry[p++];
        };
        const uint32_t na = take();
        for (uint32_t i = 0; i < na; i++) {
            C8 c;
            for (int k = 0; k < 8; k++) c.l[k] = take();
            L.actors.push_back(c);
        }
        const uint32_t ns = take();
        for (uint32_t s = 0; s < ns; s++) {
            const uint32_t n = take();
            KSpec sp;
            sp.has_lo = take() != 0;
            for (int k = 0; k < 8; k++) sp.base.l[k] = take();
            const uint32_t nc = take();
            for (uint32_t c = 0; c < nc; c++) {
                Big v;
                for (uint32_t k = 0; k < (n + 31) / 32; k++) v.push_back(take());
                C8 dg;
                for (int k = 0; k < 8; k++) dg.l[k] = take();
                sp.concrete.push_back({v, dg});
            }
            L.kspecs[n] = sp;
        }
        for (uint32_t r : rs) {
            if (r >= S.t.size()) lerr("root not in the store");
            // the term -> DAG -> program passes recurse over the nesting: past this depth a
            // host thread's 8 MiB stack could overflow (a 25,000-deep chain did), so such a
            // bucket is left to z3 like any other LoweringError
            if (S.t[r].depth > PF_MAX_TERM_DEPTH)
                lerr("term nested %u deep (more than %u): left to z3", S.t[r].depth, (unsigned)PF_MAX_TERM_DEPTH);
        }
        PROF_LAP(0);
        L.lower(rs);
        PROF_LAP(1);
        R->var_terms = L.var_terms;
        R->uf_apps = L.uf_apps;
        for (const std::string& name : L.array_order) {
            const auto& es = L.arrays[name];
            R->read_counts.push_back((uint32_t)es.size());
            for (const auto& e : es) {
                R->reads.push_back((uint32_t)e[1]);
                R->reads.push_back((uint32_t)e[0]);
            }
        }
        Dag& d = L.d;
        // hints (seed.apply_hints): the hint model becomes every variable's parent value
        if ((flags & PFLT_HINTS) && !d.vars.empty()) {
            pack(d, &R->packed_nodes, &R->pool);
            std::vector<uint32_t> widths, soft, out(8 * d.vars.size());
            for (const DVar& v : d.vars) {
                widths.push_back(v.width);
                for (int k = 0; k < 8; k++) soft.push_back(v.has_parent ? v.parent.l[k] : 0u);
            }
            std::vector<uint32_t> roots2(d.roots.begin(), d.roots.end());
            if (roots2.empty()) roots2.push_back(0);
            int n_sat = 0;
            const int rc = pfl_hints(R->packed_nodes.data(), d.nodes.size(), R->pool.data(), R->pool.size() / 8,
                                     roots2.data(), d.roots.size(), widths.data(), d.vars.size(), soft.data(),
                                     out.data(), &n_sat);
            if (rc != 0) {
                t_err = "pfl_hints failed";
                throw TermError{-1};
            }
            R->n_sat = n_sat;
            for (size_t i = 0; i < d.vars.size(); i++) {
                C8 c;
                memcpy(c.l, out.data() + 8 * i, 32);
                d.vars[i].parent = c8_of(big_of(c), d.vars[i].width);
                d.vars[i].has_parent = true;
            }
        }
        PROF_LAP(2);
        if (flags & PFLT_PROGRAM) {
            emit_program(d, R);
        } else {
            pack(d, &R->packed_nodes, &R->pool);
        }
        PROF_LAP(3);
        for (const DVar& v : d.vars) {
            R->names += v.name;
            R->names.push_back('\0');
        }
        R->dag = std::move(L.d);
        R->dag.memo.clear();  // the hash-consing table is done with
        // so is the variable index: freed here, on the lowering thread, rather than by the
        // caller's serial release after the upload (pflt_result_shrink: a node and a string
        // per variable were most of its ~7 us per result)
        decltype(R->dag.var_index)().swap(R->dag.var_index);
        PROF_LAP(4);
        return R;
    } catch (const TermError& e) {
        R->rc = e.rc;
        R->err = t_err;
    } catch (const std::exception& e) {
        R->rc = -1;
        R->err = std::string("pflt_lower: ") + e.what();
    }
    return R;
}

// ---- config-3 synthetic DAGs natively (synth.random_dag_set, bit for bit) ------------------
// numpy's Philox4x64-10 bit generator and the Generator draws random_dag_set makes: random()
// (53-bit double from next_uint64), integers(lo, hi) for int64 (Lemire on next_uint32, which
// uses both halves of a 64-bit output in turn) and integers(0, 2^32, size=8, dtype=uint64)
// (eight next_uint32).  Checked against numpy draw for draw (tests/test_synth_native.py).
struct NpPhilox {
    uint64_t ctr[4] = {0, 0, 0, 0}, key[2], buf[4] = {0, 0, 0, 0};
    int pos = 4;
    bool has32 = false;
    uint32_t u32 = 0;

    explicit NpPhilox(unsigned __int128 k) {
        key[0] = (uint64_t)k;
        key[1] = (uint64_t)(k >> 64);
    }
    static void mulhilo(uint64_t a, uint64_t b, uint64_t* hi, uint64_t* lo) {
        const unsigned __int128 p = (unsigned __int128)a * b;
        *hi = (uint64_t)(p >> 64);
        *lo = (uint64_t)p;
    }
    uint64_t next64() {
        if (pos < 4) return buf[pos++];
        if (++ctr[0] == 0 && ++ctr[1] == 0 && ++ctr[2] == 0) ++ctr[3];
        uint64_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]}, k0 = key[0], k1 = key[1];
        for (int r = 0; r < 10; r++) {
            uint64_t hi0, lo0, hi1, lo1;
            mulhilo(0xD2E7470EE14C6C93ull, c[0], &hi0, &lo0);
            mulhilo(0xCA5A826395121157ull, c[2], &hi1, &lo1);
            const uint64_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
            c[0] = n0;
            c[1] = lo1;
            c[2] = n2;
            c[3] = lo0;
            k0 += 0x9E3779B97F4A7C15ull;
            k1 += 0xBB67AE8584CAA73Bull;
        }
        for (int i = 0; i < 4; i++) buf[i] = c[i];
        pos = 1;
        return buf[0];
    }
    uint32_t next32() {
        if (has32) {
            has32 = false;
            return u32;
        }
        const uint64_t v = next64();
        has32 = true;
        u32 = (uint32_t)(v >> 32);
        return (uint32_t)v;
    }
    double random() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }
    int64_t integers(int64_t lo, int64_t hi) {  // [lo, hi), range < 2^32
        const uint64_t rng = (uint64_t)(hi - lo - 1);
        if (rng == 0) return lo;
        if (rng == 0xFFFFFFFFull) return lo + next32();
        const uint32_t rexcl = (uint32_t)rng + 1u;
        uint64_t m = (uint64_t)next32() * rexcl;
        uint32_t left = (uint32_t)m;
        if (left < rexcl) {
            const uint32_t thr = (uint32_t)((0xFFFFFFFFull - rng) % rexcl);
            while (left < thr) {
                m = (uint64_t)next32() * rexcl;
                left = (uint32_t)m;
            }
        }
        return lo + (int64_t)(m >> 32);
    }
};

// 256-bit values as C8 (little-endian u32 limbs): the planted-value arithmetic of synth._eval
bool c8_zero(const C8& a) {
    for (int i = 0; i < 8; i++)
        if (a.l[i]) return false;
    return true;
}
bool c8_ult(const C8& a, const C8& b) {
    for (int i = 7; i >= 0; i--)
        if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
    return false;
}
C8 c8_add(const C8& a, const C8& b) {
    C8 r;
    uint64_t c = 0;
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)a.l[i] + b.l[i];
        r.l[i] = (uint32_t)c;
        c >>= 32;
    }
    return r;
}
C8 c8_not(const C8& a) {
    C8 r;
    for (int i = 0; i < 8; i++) r.l[i] = ~a.l[i];
    return r;
}
C8 c8_neg(const C8& a) { return c8_add(c8_not(a), c8_small(1, 256)); }
C8 c8_sub(const C8& a, const C8& b) { return c8_add(a, c8_neg(b)); }
uint32_t c8_bitlen(const C8& a) {
    for (int i = 7; i >= 0; i--)
        if (a.l[i]) return 32u * (uint32_t)i + 32u - (uint32_t)__builtin_clz(a.l[i]);
    return 0;
}
C8 c8_shl(const C8& a, uint32_t k) {  // k < 256
    C8 r;
    const uint32_t q = k / 32, s = k % 32;
    for (int i = 7; i >= 0; i--) {
        const int j = i - (int)q;
        uint32_t v = j >= 0 ? a.l[j] << s : 0u;
        if (s && j - 1 >= 0) v |= a.l[j - 1] >> (32 - s);
        r.l[i] = v;
    }
    return r;
}
C8 c8_lshr(const C8& a, uint32_t k, uint32_t fill = 0u) {  // k < 256; fill: 0 or ~0u
    C8 r;
    const uint32_t q = k / 32, s = k % 32;
    for (int i = 0; i < 8; i++) {
        const uint32_t j = (uint32_t)i + q;
        const uint32_t lo = j < 8 ? a.l[j] : fill, hi = j + 1 < 8 ? a.l[j + 1] : fill;
        r.l[i] = s ? (lo >> s) | (hi << (32 - s)) : lo;
    }
    return r;
}
// a / b and a % b (b != 0): Knuth's algorithm D on 32-bit digits (Hacker's Delight divmnu)
void c8_divrem(const C8& a, const C8& b, C8* q, C8* r) {
    memset(q, 0, sizeof(C8));
    memset(r, 0, sizeof(C8));
    int m = 8, n = 8;
    while (m > 0 && a.l[m - 1] == 0) m--;
    while (n > 0 && b.l[n - 1] == 0) n--;
    if (m < n) {
        *r = a;
        return;
    }
    if (n == 1) {
        uint64_t k = 0;
        for (int j = m - 1; j >= 0; j--) {
            const uint64_t cur = (k << 32) | a.l[j];
            q->l[j] = (uint32_t)(cur / b.l[0]);
            k = cur - (uint64_t)q->l[j] * b.l[0];
        }
        r->l[0] = (uint32_t)k;
        return;
    }
    const int s = __builtin_clz(b.l[n - 1]);
    uint32_t vn[8], un[9];
    for (int i = n - 1; i > 0; i--) vn[i] = (b.l[i] << s) | (s ? (uint32_t)((uint64_t)b.l[i - 1] >> (32 - s)) : 0u);
    vn[0] = b.l[0] << s;
    un[m] = s ? (uint32_t)((uint64_t)a.l[m - 1] >> (32 - s)) : 0u;
    for (int i = m - 1; i > 0; i--) un[i] = (a.l[i] << s) | (s ? (uint32_t)((uint64_t)a.l[i - 1] >> (32 - s)) : 0u);
    un[0] = a.l[0] << s;
    const uint64_t base = 1ull << 32;
    for (int j = m - n; j >= 0; j--) {
        const uint64_t num = ((uint64_t)un[j + n] << 32) | un[j + n - 1];
        uint64_t qhat = num / vn[n - 1], rhat = num - qhat * vn[n - 1];
        while (qhat >= base || qhat * vn[n - 2] > ((rhat << 32) | un[j + n - 2])) {
            qhat--;
            rhat += vn[n - 1];
            if (rhat >= base) break;
        }
        int64_t borrow = 0;
        for (int i = 0; i < n; i++) {
            const uint64_t p = qhat * vn[i];
            const int64_t t = (int64_t)un[i + j] - borrow - (int64_t)(p & 0xFFFFFFFFull);
            un[i + j] = (uint32_t)t;
            borrow = (int64_t)(p >> 32) - (t >> 32);
        }
        const int64_t t = (int64_t)un[j + n] - borrow;
        un[j + n] = (uint32_t)t;
        q->l[j] = (uint32_t)qhat;
        if (t < 0) {
            q->l[j]--;
            uint64_t c = 0;
            for (int i = 0; i < n; i++) {
                c += (uint64_t)un[i + j] + vn[i];
                un[i + j] = (uint32_t)c;
                c >>= 32;
            }
            un[j + n] += (uint32_t)c;
        }
    }
    for (int i = 0; i < n; i++) r->l[i] = (un[i] >> s) | (s ? (uint32_t)((uint64_t)un[i + 1] << (32 - s)) : 0u);
}
// a * b mod 2^256 on 64-bit limbs (10 products)
C8 c8_mul64(const C8& a, const C8& b) {
    uint64_t x[4], y[4], r[4] = {0, 0, 0, 0};
    memcpy(x, a.l, 32);
    memcpy(y, b.l, 32);
    for (int i = 0; i < 4; i++) {
        unsigned __int128 c = 0;
        for (int j = 0; i + j < 4; j++) {
            c += (unsigned __int128)x[i] * y[j] + r[i + j];
            r[i + j] = (uint64_t)c;
            c >>= 64;
        }
    }
    C8 out;
    memcpy(out.l, r, 32);
    return out;
}
C8 c8_pow(const C8& b, const C8& e) {  // b^e mod 2^256 (pow(a, b, 1 << 256))
    const uint32_t n = c8_bitlen(e);
    if (!(b.l[0] & 1u) && n > 8) return c8_small(0, 256);   // even base, e >= 256: 2^256 | b^e
    C8 r = c8_small(1, 256), x = b;
    for (uint32_t i = 0; i < n; i++) {
        if ((e.l[i / 32] >> (i % 32)) & 1u) r = c8_mul64(r, x);
        if (i + 1 < n) x = c8_mul64(x, x);
    }
    return r;
}
bool c8_neg_sign(const C8& a) { return a.l[7] >> 31; }
C8 c8_abs(const C8& a) { return c8_neg_sign(a) ? c8_neg(a) : a; }
bool c8_slt(const C8& a, const C8& b) {
    const bool sa = c8_neg_sign(a), sb = c8_neg_sign(b);
    if (sa != sb) return sa;
    return c8_ult(a, b);
}

C8 synth_eval(uint32_t op, const C8& a, const C8& b) {  // synth._eval at w = 256
    C8 q, r;
    switch (op) {
        case PF_W_ADD: return c8_add(a, b);
        case PF_W_SUB: return c8_sub(a, b);
        case PF_W_MUL: return c8_mul64(a, b);
        case PF_W_UDIV:
            if (c8_zero(b)) return c8_not(c8_small(0, 256));
            c8_divrem(a, b, &q, &r);
            return q;
        case PF_W_UREM:
            if (c8_zero(b)) return a;
            c8_divrem(a, b, &q, &r);
            return r;
        case PF_W_SDIV:
        case PF_W_SREM: {
            const bool sa = c8_neg_sign(a), sb = c8_neg_sign(b);
            if (c8_zero(b)) return op == PF_W_SDIV ? (sa ? c8_small(1, 256) : c8_not(c8_small(0, 256))) : a;
            c8_divrem(c8_abs(a), c8_abs(b), &q, &r);
            if (op == PF_W_SDIV) return sa == sb ? q : c8_neg(q);
            return sa ? c8_neg(r) : r;
        }
        case PF_W_AND: { C8 z; for (int i = 0; i < 8; i++) z.l[i] = a.l[i] & b.l[i]; return z; }
        case PF_W_OR: { C8 z; for (int i = 0; i < 8; i++) z.l[i] = a.l[i] | b.l[i]; return z; }
        case PF_W_XOR: { C8 z; for (int i = 0; i < 8; i++) z.l[i] = a.l[i] ^ b.l[i]; return z; }
        case PF_W_NOT: return c8_not(a);
        case PF_W_SHL: return c8_bitlen(b) > 8 ? c8_small(0, 256) : c8_shl(a, b.l[0]);
        case PF_W_LSHR: return c8_bitlen(b) > 8 ? c8_small(0, 256) : c8_lshr(a, b.l[0]);
        case PF_W_ASHR: {
            const uint32_t fill = c8_neg_sign(a) ? ~0u : 0u;
            if (c8_bitlen(b) > 8) {
                C8 z;
                for (int i = 0; i < 8; i++) z.l[i] = fill;
                return z;
            }
            return c8_lshr(a, b.l[0], fill);
        }
        case PF_W_EXP: return c8_pow(a, b);
        default: return a;
    }
}

constexpr uint64_t kDagGenSeed = 20260101ull;
constexpr uint32_t kCandSeedBase = 0x4D595448u;
// synth._MIX in order (the op kinds) and its normalised cumulative probabilities, the doubles
// numpy's cumsum / cdf[-1] produces (tests/test_synth_native.py checks the table)
enum SynthKind { SK_MUL, SK_DIV, SK_REM, SK_EXP, SK_ADDSUB, SK_LOGIC, SK_SHIFT, SK_ITECMP };

C8 synth_leaf_value(NpPhilox& g) {  // synth._leaf_value
    if (g.random() < 0.5) {  // _rand256: eight u32 draws, the first the most significant
        C8 v;
        for (int i = 7; i >= 0; i--) v.l[i] = g.next32();
        return v;
    }
    const int64_t j = g.integers(0, 9);
    switch (j) {
        case 0: return c8_small(0, 256);
        case 1: return c8_small(1, 256);
        case 2: return c8_small(2, 256);
        case 3: return c8_not(c8_small(0, 256));
        case 4: { C8 v = c8_small(0, 256); v.l[7] = 0x80000000u; return v; }
        case 5: { C8 v = c8_small(0, 256); for (int i = 0; i < 5; i++) v.l[i] = ~0u; return v; }
        default: {
            const int64_t k = g.integers(0, 256);
            C8 p = c8_small(0, 256);
            p.l[k / 32] = 1u << (k % 32);
            if (j == 6) return c8_sub(p, c8_small(1, 256));
            if (j == 8) return c8_add(p, c8_small(1, 256));
            return p;
        }
    }
}

// One config-3 DAG into R (synth.random_dag_set(dag_id, plant)); the witness into *wit.
void synth_dag(uint32_t dag_id, bool plant, const double* cdf, Result* R, std::vector<C8>* wit) {
    NpPhilox g(((unsigned __int128)kDagGenSeed << 32) | dag_id);
    Dag d(256);
    const int64_t n_vars = g.integers(4, 9);
    wit->clear();
    for (int64_t v = 0; v < n_vars; v++) wit->push_back(synth_leaf_value(g));
    std::vector<std::pair<int32_t, C8>> leaves, interior;
    for (int64_t v = 0; v < n_vars; v++) {
        bool created;
        leaves.push_back({d.var("x" + std::to_string(v), 256, PF_VK_GENERIC, 0, 0, plant, (*wit)[v], &created),
                          (*wit)[v]});
    }
    for (int k = 0; k < 4; k++) {
        const C8 c = synth_leaf_value(g);
        leaves.push_back({d.cnst(c, 256), c});
    }
    const int depth = 32, window = 6;
    auto pick = [&](bool first) -> std::pair<int32_t, C8> {
        if (first && !interior.empty() && (int)interior.size() <= depth) return interior.back();
        const size_t np = std::min<size_t>(interior.size(), (size_t)window);
        if (np && g.random() < 0.6) return interior[interior.size() - np + (size_t)g.integers(0, (int64_t)np)];
        return leaves[(size_t)g.integers(0, (int64_t)leaves.size())];
    };
    for (int it = 0; it < 48; it++) {
        const double u = g.random();
        int kind = 0;
        while (kind < 7 && !(u < cdf[kind])) kind++;   // bisect_right
        auto A = pick(true);
        auto B = pick(false);
        uint32_t op = 0;
        switch (kind) {
            case SK_DIV: op = g.random() < 0.5 ? PF_W_UDIV : PF_W_SDIV; break;
            case SK_REM: op = g.random() < 0.5 ? PF_W_UREM : PF_W_SREM; break;
            case SK_ADDSUB: op = g.random() < 0.5 ? PF_W_ADD : PF_W_SUB; break;
            case SK_LOGIC: {
                static const uint32_t ops[4] = {PF_W_AND, PF_W_OR, PF_W_XOR, PF_W_NOT};
                op = ops[g.integers(0, 4)];
                break;
            }
            case SK_SHIFT: {
                static const uint32_t ops[3] = {PF_W_SHL, PF_W_LSHR, PF_W_ASHR};
                op = ops[g.integers(0, 3)];
                if (g.random() < 0.5) {
                    (void)g.integers(0, 256);   // drawn and unused, as in synth.py
                    B.first = d.op(PF_W_AND, 256, {B.first, d.cnst(0xFF, 256)});
                    C8 m = c8_small(0, 256);
                    m.l[0] = B.second.l[0] & 0xFFu;
                    B.second = m;
                }
                break;
            }
            case SK_ITECMP: {
                static const uint32_t ops[3] = {PF_B_ULT, PF_B_SLT, PF_B_EQ};
                const uint32_t c_op = ops[g.integers(0, 3)];
                auto C2 = pick(false);
                const int32_t cond = d.op(c_op, 256, {A.first, C2.first});
                const bool cv = c_op == PF_B_ULT ? c8_ult(A.second, C2.second)
                                : c_op == PF_B_EQ ? A.second == C2.second : c8_slt(A.second, C2.second);
                const int32_t node = d.op(PF_W_ITE, 256, {cond, A.first, B.first});
                interior.push_back({node, cv ? A.second : B.second});
                continue;
            }
            case SK_MUL: op = PF_W_MUL; break;
            default: op = PF_W_EXP; break;
        }
        int32_t node;
        C8 val;
        if (op == PF_W_NOT) {
            node = d.op(op, 256, {A.first});
            val = c8_not(A.second);
        } else {
            node = d.op(op, 256, {A.first, B.first});
            val = synth_eval(op, A.second, B.second);
        }
        interior.push_back({node, val});
    }
    const int64_t n_roots = g.integers(2, 5);
    const size_t nt = std::min<size_t>(interior.size(), (size_t)std::max<int64_t>(n_roots * 2, 8));
    const size_t t0 = interior.size() - nt;
    for (int64_t r = 0; r < n_roots; r++) {
        const auto& NV = interior[t0 + (size_t)g.integers(0, (int64_t)nt)];
        const int64_t cmp = g.integers(0, 3);
        int32_t root;
        if (cmp == 0) {
            root = d.op(PF_B_EQ, 256, {NV.first, d.cnst(NV.second, 256)});
        } else if (cmp == 1) {
            root = d.op(PF_B_ULE, 256, {NV.first, d.cnst(NV.second, 256)});
        } else {
            const int32_t c = d.cnst(NV.second, 256);
            root = d.op(PF_B_ULE, 256, {c, NV.first});
        }
        d.roots.push_back(root);
    }
    emit_program(d, R);
    for (const DVar& v : d.vars) {
        R->names += v.name;
        R->names.push_back('\0');
    }
    R->parented = plant;
    R->dag = std::move(d);
    R->dag.memo.clear();
}

}  // namespace

extern "C" {

void* pflt_store_new(void) {
    // The hint solver and the lowering report conflicts as C++ exceptions, and the first one
    // thrown in a process has libgcc's unwinder set up its frame tables for every library
    // loaded: ~80 ms once PyTorch's are (tools/slow_job_probe.py: the corpus's first bucket
    // whose hints hit a conflict took 80 ms, then 0.05 ms; 0.03 ms without torch loaded).
    // A store is made once per process (and per retired generation), before any lowering:
    // take that one-time cost here rather than inside the first query that conflicts.
    try {
        throw TermError{0};
    } catch (const TermError&) {
    }
    return new Store();
}

uint32_t pflt_features(void) { return PFLT_FEAT_EXPLICIT | PFLT_FEAT_SYNTH; }

int pflt_synth(uint32_t first_id, size_t n, uint32_t plant, const double* cdf, void** results,
               uint32_t* witness_limbs, uint32_t* n_vars_out) {
    try {
        std::vector<C8> wit;
        for (size_t i = 0; i < n; i++) {
            Result* R = new Result();
            results[i] = R;
            try {
                synth_dag(first_id + (uint32_t)i, plant != 0, cdf, R, &wit);
            } catch (const TermError& e) {
                R->rc = e.rc;
                R->err = t_err;
                return -1;
            }
            if (n_vars_out) n_vars_out[i] = (uint32_t)wit.size();
            if (witness_limbs)
                for (size_t v = 0; v < wit.size(); v++) memcpy(witness_limbs + 64 * i + 8 * v, wit[v].l, 32);
        }
    } catch (const std::exception& e) {
        t_err = std::string("pflt_synth: ") + e.what();
        return -1;
    }
    return 0;
}

void pflt_store_free(void* st) { delete (Store*)st; }

size_t pflt_store_size(void* st) { return ((Store*)st)->t.size(); }

int64_t pflt_add(void* st, uint32_t op, uint32_t sortk, uint32_t w1, uint32_t w2, const uint32_t* args,
                 uint32_t nargs, int64_t i0, int64_t i1, const uint32_t* limbs, uint32_t nlimbs,
                 const char* name) {
    Store* S = (Store*)st;
    TermRec r;
    r.op = op;
    r.sortk = sortk;
    r.w1 = w1;
    r.w2 = w2;
    for (uint32_t i = 0; i < nargs; i++) {
        if (args[i] >= S->t.size()) {
            t_err = "pflt_add: argument not in the store";
            return -1;
        }
        r.args.push_back(args[i]);
        r.depth = std::max(r.depth, S->t[args[i]].depth + 1u);
    }
    r.i0 = i0;
    r.i1 = i1;
    if (limbs) r.val.assign(limbs, limbs + nlimbs);
    if (name) r.name = name;
    S->t.push_back(std::move(r));
    return (int64_t)S->t.size() - 1;
}

void* pflt_lower(void* st, const uint32_t* roots, size_t n_roots, const uint32_t* registry,
                 size_t n_registry, const char* par_names, const uint32_t* par_name_vals, size_t n_par_names,
                 const uint32_t* par_reads, const uint32_t* par_read_vals, size_t n_par_reads,
                 uint32_t flags, uint32_t seed, int* rc_out) {
    (void)seed;
    Parents P;
    fill_parents(&P, par_names, par_name_vals, n_par_names, par_reads, par_read_vals, n_par_reads);
    Result* R = lower_job(*(const Store*)st, std::vector<uint32_t>(roots, roots + n_roots), P, registry,
                          n_registry, flags);
    *rc_out = R->rc;
    if (R->rc != 0) {
        t_err = R->err;
        delete R;
        return nullptr;
    }
    return R;
}

const char* pflt_last_error(void) { return t_err.c_str(); }

}  // extern "C"

namespace {

uint32_t key_id(Store* S, const std::string& k) {
    auto it = S->key_ids.find(k);
    if (it != S->key_ids.end()) return it->second;
    const uint32_t id = (uint32_t)S->key_names.size();
    S->key_names.push_back(k);
    S->key_ids.emplace(k, id);
    return id;
}

bool keccak_app(const std::string& f, std::string* n, bool* inv) {  // ^keccak256_(\d+)(-1)?$
    static const char pre[] = "keccak256_";
    if (f.compare(0, sizeof(pre) - 1, pre) != 0) return false;
    size_t i = sizeof(pre) - 1, j = i;
    while (j < f.size() && isdigit((unsigned char)f[j])) j++;
    if (j == i) return false;
    *n = f.substr(i, j - i);
    if (j == f.size()) { *inv = false; return true; }
    if (f.compare(j, std::string::npos, "-1") == 0) { *inv = true; return true; }
    return false;
}

void merge_sorted(std::vector<uint32_t>* into, const std::vector<uint32_t>& b) {
    std::vector<uint32_t> out;
    out.reserve(into->size() + b.size());
    std::set_union(into->begin(), into->end(), b.begin(), b.end(), std::back_inserter(out));
    into->swap(out);
}

// dependence_keys + free_inverse_widths of every term below root (iterative post-order)
int32_t dep_keys(Store* S, uint32_t root) {
    if (S->kmemo.size() < S->t.size()) S->kmemo.resize(S->t.size(), -1);
    if (S->kmemo[root] >= 0) return S->kmemo[root];
    std::vector<std::pair<uint32_t, bool>> stack{{root, false}};
    while (!stack.empty()) {
        const auto [x, expanded] = stack.back();
        stack.pop_back();
        if (S->kmemo[x] >= 0) continue;
        const TermRec& r = S->t[x];
        if (!expanded) {
            stack.push_back({x, true});
            for (uint32_t a : r.args)
                if (S->kmemo[a] < 0) stack.push_back({a, false});
            continue;
        }
        std::vector<uint32_t> own, finv;
        if (r.op == PFLT_VAR || r.op == PFLT_BVAR) own.push_back(key_id(S, "v:" + r.name));
        else if (r.op == PFLT_ARRAY) own.push_back(key_id(S, "a:" + r.name));
        else if (r.op == PFLT_APPLY) {
            std::string n;
            bool inv;
            if (keccak_app(r.name, &n, &inv)) {
                own.push_back(key_id(S, "k:" + n));
                if (inv) {
                    const TermRec& a = S->t[r.args[0]];
                    if (!(a.op == PFLT_APPLY && a.name == "keccak256_" + n)) finv.push_back(key_id(S, n));
                }
            } else if (r.name == "Power") {
                own.push_back(key_id(S, "f:Power"));
            }
        }
        std::sort(own.begin(), own.end());
        std::sort(finv.begin(), finv.end());
        for (uint32_t a : r.args) {
            merge_sorted(&own, S->keysets[S->kmemo[a]]);
            merge_sorted(&finv, S->finvs[S->kmemo[a]]);
        }
        S->kmemo[x] = (int32_t)S->keysets.size();
        S->keysets.push_back(std::move(own));
        S->finvs.push_back(std::move(finv));
    }
    return S->kmemo[root];
}

}  // namespace

extern "C" {

/* Independence buckets of one query (smt/independence.py:buckets, the same partition and
 * order): conjuncts = the roots with top-level ands flattened and true dropped; buckets
 * share no symbol, array, Power, or keccak family (a width with a free inverse lookup).
 * out_ids: the conjuncts bucket by bucket (capacity >= total conjuncts); out_sizes: each
 * bucket's size.  Returns the number of buckets, or -1 (capacity) / -2 (bad id). */
int64_t pflt_buckets(void* st, const uint32_t* roots, size_t n_roots, uint32_t* out_ids, size_t cap_ids,
                     uint32_t* out_sizes, size_t cap_sizes) {
    Store* S = (Store*)st;
    std::vector<uint32_t> cs;
    std::vector<uint32_t> stack;
    for (size_t i = n_roots; i-- > 0;) stack.push_back(roots[i]);
    while (!stack.empty()) {
        const uint32_t c = stack.back();
        stack.pop_back();
        if (c >= S->t.size()) return -2;
        const TermRec& r = S->t[c];
        if (r.op == PFLT_AND) {
            for (size_t i = r.args.size(); i-- > 0;) stack.push_back(r.args[i]);
        } else if (r.op != PFLT_TRUE) {
            cs.push_back(c);
        }
    }
    // flat arrays and key-indexed scratch instead of per-call maps and vectors of vectors (a
    // query's bucketing was ~20 us, mostly allocation and string lookups)
    std::vector<uint32_t> families;
    std::vector<int32_t> kidx(cs.size());
    for (size_t i = 0; i < cs.size(); i++) {
        kidx[i] = dep_keys(S, cs[i]);
        const auto& fv = S->finvs[kidx[i]];
        families.insert(families.end(), fv.begin(), fv.end());
    }
    std::sort(families.begin(), families.end());
    families.erase(std::unique(families.begin(), families.end()), families.end());
    const size_t nk = S->key_names.size();
    if (S->kfam.size() < nk) S->kfam.resize(nk, -3);
    if (S->uf.size() < nk) {
        S->uf.resize(nk, -1);
        S->ugrp.resize(nk, -1);
    }
    std::vector<int32_t>& uf = S->uf;
    std::vector<uint32_t> touched;
    auto find = [&](uint32_t k) {
        while ((uint32_t)uf[k] != k) {
            uf[k] = uf[uf[k]];
            k = (uint32_t)uf[k];
        }
        return k;
    };
    // kept keys of conjunct i: kept[off[i] .. off[i + 1])
    std::vector<uint32_t> kept, off(cs.size() + 1, 0);
    for (size_t i = 0; i < cs.size(); i++) {
        for (uint32_t k : S->keysets[kidx[i]]) {
            int32_t fam = S->kfam[k];
            if (fam == -3 || fam == -1) {
                const std::string& nm = S->key_names[k];
                if (nm.compare(0, 2, "k:") != 0) {
                    fam = -2;
                } else {
                    auto it = S->key_ids.find(nm.substr(2));
                    fam = it == S->key_ids.end() ? -1 : (int32_t)it->second;
                }
                S->kfam[k] = fam;
            }
            if (fam == -1 || (fam >= 0 && !std::binary_search(families.begin(), families.end(), (uint32_t)fam)))
                continue;
            kept.push_back(k);
        }
        off[i + 1] = (uint32_t)kept.size();
        bool have = false;
        uint32_t first = 0;
        for (uint32_t j = off[i]; j < off[i + 1]; j++) {
            const uint32_t k = kept[j];
            if (uf[k] < 0) {
                uf[k] = (int32_t)k;
                touched.push_back(k);
            }
            if (!have) {
                first = find(k);
                have = true;
            } else {
                const uint32_t rk = find(k);
                if (rk != first) uf[rk] = (int32_t)first;
            }
        }
    }
    // group of each conjunct, numbered in order of first appearance; the ground conjuncts
    // (no kept key) form the last group
    std::vector<int32_t>& ugrp = S->ugrp;
    std::vector<uint32_t> gi(cs.size()), gsize;
    uint32_t n_ground = 0;
    for (size_t i = 0; i < cs.size(); i++) {
        if (off[i] == off[i + 1]) {
            gi[i] = UINT32_MAX;
            n_ground++;
            continue;
        }
        const uint32_t rt = find(kept[off[i]]);
        if (ugrp[rt] < 0) {
            ugrp[rt] = (int32_t)gsize.size();
            gsize.push_back(0);
        }
        gi[i] = (uint32_t)ugrp[rt];
        gsize[gi[i]]++;
    }
    for (uint32_t k : touched) uf[k] = ugrp[k] = -1;
    const size_t ng = gsize.size() + (n_ground ? 1 : 0);
    if (cs.size() > cap_ids || ng > cap_sizes) return -1;
    // bucket by bucket, conjuncts in query order within each
    std::vector<uint32_t> pos(ng, 0);
    for (size_t g = 0; g < gsize.size(); g++) {
        out_sizes[g] = gsize[g];
        if (g + 1 < ng) pos[g + 1] = pos[g] + gsize[g];
    }
    if (n_ground) out_sizes[ng - 1] = n_ground;
    for (size_t i = 0; i < cs.size(); i++) out_ids[pos[gi[i] == UINT32_MAX ? ng - 1 : gi[i]]++] = cs[i];
    return (int64_t)ng;
}

int64_t pflt_buckets_many(void* st, const uint32_t* roots, const uint64_t* offsets, size_t n_queries,
                          uint32_t* out_ids, size_t cap_ids, uint32_t* out_sizes, size_t cap_sizes,
                          int64_t* out_counts) {
    size_t oi = 0, os = 0;
    for (size_t q = 0; q < n_queries; q++) {
        const int64_t nb = pflt_buckets(st, roots + offsets[q], (size_t)(offsets[q + 1] - offsets[q]), out_ids + oi,
                                        cap_ids - oi, out_sizes + os, cap_sizes - os);
        if (nb < 0) return nb;
        out_counts[q] = nb;
        for (int64_t g = 0; g < nb; g++) oi += out_sizes[os + (size_t)g];
        os += (size_t)nb;
    }
    return (int64_t)os;
}

int pflt_view(void* st, uint32_t id, pflt_term_view* out) {
    const Store* S = (const Store*)st;
    if (id >= S->t.size()) return -1;
    const TermRec& r = S->t[id];
    out->op = r.op;
    out->sortk = r.sortk;
    out->w1 = r.w1;
    out->w2 = r.w2;
    out->nargs = (uint32_t)r.args.size();
    out->args = r.args.data();
    out->i0 = r.i0;
    out->i1 = r.i1;
    out->limbs = r.val.data();
    out->nlimbs = (uint32_t)r.val.size();
    out->name = r.name.c_str();
    return 0;
}

void pflt_result_free(void* res) { delete (Result*)res; }

/* sizes: [0] n_vars, [1] names bytes, [2] n_var_terms, [3] n_uf_apps, [4] n_arrays,
 * [5] n_reads, [6] n_ins, [7] n_const, [8] n_nodes, [9] n_pool, [10] n_roots, [11] n_forced,
 * [12] n_wregs, [13] n_sat, [14] n_in_roots, [15] parented, [16] some variable has a parent value */
void pflt_result_info_many(void* const* results, size_t n, uint64_t* out) {
    for (size_t j = 0; j < n; j++) {
        uint64_t* row = out + 18 * j;
        const Result* R = (const Result*)results[j];
        row[0] = (uint64_t)(int64_t)R->rc;
        if (R->rc == 0)
            pflt_result_info(results[j], row + 1);
        else
            memset(row + 1, 0, 17 * sizeof(uint64_t));
    }
}

void pflt_result_info(void* res, uint64_t* info) {
    const Result* R = (const Result*)res;
    info[0] = R->dag.vars.size();
    info[1] = R->names.size();
    info[2] = R->var_terms.size();
    info[3] = R->uf_apps.size();
    info[4] = R->read_counts.size();
    info[5] = R->reads.size() / 2;
    info[6] = R->code.size() / 4;
    info[7] = R->consts.size() / 8;
    info[8] = R->dag.nodes.size();
    info[9] = R->pool.size() / 8;
    info[10] = R->dag.roots.size();
    info[11] = R->dag.forced.size();
    info[12] = R->n_wregs;
    info[13] = (uint64_t)R->n_sat;
    info[14] = R->in_roots.size();
    info[15] = R->parented ? 1u : 0u;
    bool hp = false;
    for (const DVar& v : R->dag.vars) hp |= v.has_parent;
    info[16] = hp ? 1u : 0u;
}

/* vars: n_vars x 12 u32 = width, kind, hint0, hint1, has_parent, parent x 8 ... (13 words)
 * var_terms: n x 4; uf_apps: n; reads: n x 2 (array id, index id) + counts per array;
 * code n_ins x 4; consts n_const x 8; nodes n_nodes x 8; pool n_pool x 8; roots; forced x 8 */
int pflt_result_candidate0(const void* res, uint32_t* out) {
    const Result* R = (const Result*)res;
    for (const DVar& v : R->dag.vars)
        if (!v.has_parent) return 0;
    for (const DVar& v : R->dag.vars) {
        const C8 c = c8_of(big_of(v.parent), v.width);
        memcpy(out, c.l, 32);
        out += 8;
    }
    return 1;
}

void pflt_result_get(void* res, uint32_t which, uint32_t* out, char* names_out) {
    const Result* R = (const Result*)res;
    switch (which) {
        case PFLT_GET_VARS:
            for (const DVar& v : R->dag.vars) {
                *out++ = v.width;
                *out++ = v.kind;
                *out++ = v.hint0;
                *out++ = v.hint1;
                *out++ = v.has_parent ? 1u : 0u;
                for (int k = 0; k < 8; k++) *out++ = v.parent.l[k];
            }
            if (names_out) memcpy(names_out, R->names.data(), R->names.size());
            break;
        case PFLT_GET_VAR_TERMS:
            for (const VarTerm& vt : R->var_terms) {
                *out++ = vt.type;
                *out++ = vt.a;
                *out++ = vt.b;
                *out++ = vt.c;
            }
            break;
        case PFLT_GET_UF_APPS: std::copy(R->uf_apps.begin(), R->uf_apps.end(), out); break;
        case PFLT_GET_READS:
            out = std::copy(R->read_counts.begin(), R->read_counts.end(), out);
            std::copy(R->reads.begin(), R->reads.end(), out);
            break;
        case PFLT_GET_CODE: std::copy(R->code.begin(), R->code.end(), out); break;
        case PFLT_GET_CONSTS: std::copy(R->consts.begin(), R->consts.end(), out); break;
        case PFLT_GET_NODES: std::copy(R->packed_nodes.begin(), R->packed_nodes.begin() + 8 * R->dag.nodes.size(), out); break;
        case PFLT_GET_POOL: std::copy(R->pool.begin(), R->pool.end(), out); break;
        case PFLT_GET_ROOTS:
            for (int32_t r : R->dag.roots) *out++ = (uint32_t)r;
            break;
        case PFLT_GET_FORCED:
            for (const C8& c : R->dag.forced) out = std::copy(c.l, c.l + 8, out);
            break;
        case PFLT_GET_IN_ROOTS: std::copy(R->in_roots.begin(), R->in_roots.end(), out); break;
        default: break;
    }
}

}  // extern "C"

// ---- batches: parent models, concurrent lowering, batch packing ---------------------------
namespace {

void note_read(Store* S, uint32_t arr, uint32_t idx, const C8& v) {
    auto& tab = S->recent.reads.touch(S->t[arr].name);
    tab.touch({arr, idx}) = v;
    tab.trim(256);
}

}  // namespace

extern "C" {

void* pflt_parent_new(const char* names, const uint32_t* name_vals, size_t n_names, const uint32_t* reads,
                      const uint32_t* read_vals, size_t n_reads) {
    Parents* P = new Parents();
    fill_parents(P, names, name_vals, n_names, reads, read_vals, n_reads);
    return P;
}

void pflt_parent_free(void* p) { delete (Parents*)p; }

void pflt_parent_info(const void* p, uint64_t* info) {
    const Parents* P = (const Parents*)p;
    uint64_t nb = 0, nw = 0;
    for (const std::string& n : P->name_order) {
        nb += n.size() + 1;
        nw += 1 + P->names.at(n).size();
    }
    info[0] = P->name_order.size();
    info[1] = nb;
    info[2] = nw;
    info[3] = P->read_order.size();
}

void pflt_parent_get(const void* p, char* names, uint32_t* name_vals, uint32_t* reads, uint32_t* read_vals) {
    const Parents* P = (const Parents*)p;
    for (const std::string& n : P->name_order) {
        memcpy(names, n.c_str(), n.size() + 1);
        names += n.size() + 1;
        const Big& v = P->names.at(n);
        *name_vals++ = (uint32_t)v.size();
        name_vals = std::copy(v.begin(), v.end(), name_vals);
    }
    for (const auto& k : P->read_order) {
        *reads++ = k.first;
        *reads++ = k.second;
        read_vals = std::copy(P->reads.at(k).l, P->reads.at(k).l + 8, read_vals);
    }
}

void pflt_recent_clear(void* st) {
    Store* S = (Store*)st;
    S->recent.vars.clear();
    S->recent.reads.clear();
}

void pflt_note_vars(void* st, const char* names, const uint32_t* vals, size_t n, size_t recent_size) {
    Store* S = (Store*)st;
    for (size_t i = 0; i < n; i++) {
        const uint32_t nl = *vals++;
        S->recent.vars.touch(std::string(names)) = Big(vals, vals + nl);
        vals += nl;
        names += strlen(names) + 1;
    }
    S->recent.vars.trim(recent_size);
}

void pflt_note_result(void* st, const void* res, const uint32_t* values, size_t recent_size) {
    Store* S = (Store*)st;
    const Result* R = (const Result*)res;
    const size_t n = std::min(R->var_terms.size(), R->dag.vars.size());
    for (size_t i = 0; i < n; i++) {
        const VarTerm& vt = R->var_terms[i];
        const uint32_t* v = values + 8 * i;
        if (vt.type == PFLT_VT_TERM) {
            const TermRec& r = S->t[vt.a];
            if (r.op == PFLT_VAR || r.op == PFLT_BVAR) S->recent.vars.touch(r.name) = Big(v, v + 8);
        } else if (vt.type == PFLT_VT_SELECT && S->t[vt.a].op == PFLT_ARRAY) {
            C8 c;
            memcpy(c.l, v, 32);
            note_read(S, vt.a, vt.b, c);
        }
    }
    S->recent.vars.trim(recent_size);
    S->recent.reads.trim(1024);
}

void* pflt_recent_parent(void* st, const uint32_t* roots, size_t n_roots) {
    Store* S = (Store*)st;
    std::vector<uint32_t> keys;
    for (size_t i = 0; i < n_roots; i++) {
        if (roots[i] >= S->t.size()) return nullptr;
        merge_sorted(&keys, S->keysets[dep_keys(S, roots[i])]);
    }
    Parents* P = new Parents();
    for (uint32_t k : keys) {
        const std::string& nm = S->key_names[k];
        if (nm.compare(0, 2, "v:") == 0) {
            if (const Big* v = S->recent.vars.get(nm.substr(2))) P->set_name(nm.substr(2), *v);
        } else if (nm.compare(0, 2, "a:") == 0) {
            if (const auto* tab = S->recent.reads.get(nm.substr(2)))
                for (const auto& rk : tab->order) P->set_read(rk, tab->m.at(rk).second);
        }
    }
    if (P->empty()) {
        delete P;
        return nullptr;
    }
    return P;
}

void pflt_lower_many(void* st, const pflt_job* jobs, size_t n, const uint32_t* registry, size_t n_registry,
                     uint32_t n_threads, void** results) {
    const Store& S = *(const Store*)st;
    static const Parents none;
    auto one = [&](size_t j) {
        const pflt_job& jb = jobs[j];
        results[j] = lower_job(S, std::vector<uint32_t>(jb.roots, jb.roots + jb.n_roots),
                               jb.parents ? *(const Parents*)jb.parents : none, registry, n_registry, jb.flags);
    };
    pfpool::parallel_for(n, n_threads, one);
}

int pflt_result_status(const void* res) { return ((const Result*)res)->rc; }

const char* pflt_result_error(const void* res) { return ((const Result*)res)->err.c_str(); }

int pflt_result_parented(const void* res) { return ((const Result*)res)->parented ? 1 : 0; }

void pflt_result_shrink(void* res) {
    Result* R = (Result*)res;
    std::vector<uint32_t>().swap(R->code);
    std::vector<uint32_t>().swap(R->consts);
    std::vector<uint32_t>().swap(R->packed_nodes);
    std::vector<uint32_t>().swap(R->pool);
    std::vector<DNode>().swap(R->dag.nodes);
    std::vector<int32_t>().swap(R->dag.roots);
    std::vector<C8>().swap(R->dag.forced);
    decltype(R->dag.var_index)().swap(R->dag.var_index);
}

void pflt_pack_sizes(void* const* results, size_t n, uint64_t* out) {
    uint64_t ni = 0, nc = 0, nv = 0, np = 0;
    for (size_t j = 0; j < n; j++) {
        const Result* R = (const Result*)results[j];
        ni += R->code.size() / 4;
        nc += R->consts.size() / 8;
        nv += R->dag.vars.size();
        for (const DVar& v : R->dag.vars) np += v.has_parent ? 1 : 0;
    }
    out[0] = ni;
    out[1] = nc;
    out[2] = nv;
    out[3] = np;
}

void pflt_pack_batch(void* const* results, size_t n, const uint32_t* seeds, const uint32_t* reach_lut,
                     uint32_t lut_w, uint32_t* code, uint32_t* consts, uint32_t* schema, uint32_t* parents,
                     uint32_t* descs) {
    uint32_t oc = 0, ok = 0, ov = 0, op = 0;
    for (size_t j = 0; j < n; j++) {
        const Result* R = (const Result*)results[j];
        const uint32_t ni = (uint32_t)(R->code.size() / 4), nk = (uint32_t)(R->consts.size() / 8),
                       nv = (uint32_t)R->dag.vars.size();
        bool has_par = false;
        for (const DVar& v : R->dag.vars) has_par |= v.has_parent;
        uint32_t* d = descs + 8 * j;
        d[0] = oc;
        d[1] = ni;
        d[2] = ok;
        d[3] = nk;
        d[4] = ov;
        d[5] = nv;
        d[6] = seeds[j];
        d[7] = has_par ? op : PF_NO_PARENT;
        for (uint32_t i = 0; i < ni; i++) {
            const uint32_t* w = R->code.data() + 4 * i;
            uint32_t* o = code + 4 * (size_t)(oc + i);
            o[0] = w[0];
            o[1] = w[1];
            o[2] = w[2];
            const uint32_t opc = w[0] & 0xffu, wd = (w[0] >> 8) & 0x3ffu;
            o[3] = wd < lut_w ? reach_lut[(size_t)opc * lut_w + wd] : 0u;
        }
        memcpy(consts + 8 * (size_t)ok, R->consts.data(), 4 * R->consts.size());
        for (uint32_t i = 0; i < nv; i++) {
            const DVar& v = R->dag.vars[i];
            uint32_t* s = schema + 4 * (size_t)(ov + i);
            s[0] = v.kind | (v.width << 8);
            s[1] = v.hint0;
            s[2] = v.hint1;
            s[3] = PF_NO_PARENT;
            if (has_par && v.has_parent) {
                s[3] = op;
                memcpy(parents + 8 * (size_t)op, v.parent.l, 32);
                op++;
            }
        }
        oc += ni;
        ok += nk;
        ov += nv;
    }
}

}  // extern "C"
