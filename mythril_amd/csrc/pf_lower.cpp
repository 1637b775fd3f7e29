// pf_lower.cpp — libpflower.so: register allocation + emission of one constraint DAG
// (include/pf_lower.h).  The native form of mythril_amd/lower.py:lower, instruction for
// instruction: the same emission order (post-order per root, operands largest-subtree first),
// the same linear-scan allocation over PF_NW W and PF_NB B registers with Belady eviction of
// rematerialisable values, the same spill-slot policy and the same constant-pool numbering —
// tests/test_native_lower.py checks the programs are identical.  Host code, no HIP.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pf_bytecode.h"
#include "../../include/pf_lower.h"

namespace {

thread_local std::string g_err;

int fail(int rc, const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return rc;
}

struct LowerError {
    int rc;
};

constexpr int INF = 1 << 30;
constexpr int NONE = -1;

struct Node {
    uint32_t kind, width, nargs, args[3], aux, is_bool;
};

bool is_leaf(uint32_t k) { return k >= PFL_K_VAR && k <= PFL_K_BVAR; }

// SURVEY.md §8(d) per-op int32 table scaled by width (mythril_amd/ir.py op_cost): the
// rematerialisation test only recomputes values whose op costs <= 16
int op_cost(uint32_t op, uint32_t w) {
    int c;
    switch (op) {
        case PF_W_ADD: case PF_W_SUB: case PF_W_NOT: case PF_W_AND: case PF_W_OR: case PF_W_XOR:
        case PF_W_NEG: case PF_W_ITE: case PF_W_EXTRACT: case PF_W_CONCAT: case PF_W_SEXT:
        case PF_B_EQ: case PF_B_ULT: case PF_B_ULE: case PF_B_SLT: case PF_B_SLE: case PF_B_UADD_NOOVF:
            c = 8; break;
        case PF_W_HASH: c = 0; break;
        case PF_W_SHL: case PF_W_LSHR: case PF_W_ASHR: c = 16; break;
        case PF_W_MUL: case PF_B_UMUL_NOOVF: c = 72; break;
        case PF_W_UDIV: case PF_W_UREM: c = 256; break;
        case PF_W_SDIV: case PF_W_SREM: case PF_W_SMOD: c = 280; break;
        case PF_W_EXP: c = 512 * 72; break;
        default: return 0;
    }
    const int nl = ((int)std::max<uint32_t>(1, w) + 31) / 32;
    return (c * nl + 7) / 8;
}

struct Const8 {
    uint32_t l[8];
    bool operator==(const Const8& o) const { return memcmp(l, o.l, sizeof(l)) == 0; }
};

struct RegFile {
    int n;
    std::vector<int> free_;     // stack: back() is taken first
    std::vector<int> holder;    // reg -> node or NONE
    std::vector<int>* where;    // node -> reg (shared array, NONE if not resident)
    explicit RegFile(int n_, std::vector<int>* w) : n(n_), holder(n_, NONE), where(w) {
        for (int r = n - 1; r >= 0; --r) free_.push_back(r);
    }
};

class Lowerer {
   public:
    Lowerer(const Node* nodes, size_t n_nodes, const Const8* pool, size_t n_pool, int n_wregs)
        : N(nodes), nn(n_nodes), pool(pool), n_pool(n_pool), where(n_nodes, NONE),
          slot_of(n_nodes, NONE), remat(n_nodes, -2), cost(n_nodes, -1), W(n_wregs, &where), B(PF_NB, &where) {
        for (int s = PF_MAX_SPILL - 1; s >= 0; --s) free_slots.push_back(s);
        // a variable is spilled (not regenerated) only when this many uses remain after its
        // eviction (lower.py _var_spill_uses: the same environment variable)
        const char* e = getenv("PF_VAR_SPILL_USES");
        spill_min_uses = e ? std::max(1, atoi(e)) : 1;
        // ... and at least this many when a W_EXP runs before its last use (the device
        // program's LDS spill slots are EXP's table entries, so that spill lands in scratch;
        // lower.py _var_spill_uses_exp: the same environment variable and default)
        const char* x = getenv("PF_VAR_SPILL_USES_EXP");
        spill_exp_uses = x ? std::max(0, atoi(x)) : 99;
    }

    std::vector<uint32_t> code;    // 4 words per instruction
    std::vector<Const8> consts;

    void run(const uint32_t* roots, size_t n_roots) {
        order(roots, n_roots);
        // use times per node, ascending (CSR: counted, then filled in event order)
        use_off.assign(nn + 1, 0);
        for (const auto& e : events) {
            if (!e.first) {
                const Node& n = N[e.second];
                for (uint32_t k = 0; k < n.nargs; ++k) use_off[n.args[k] + 1]++;
            } else {
                use_off[e.second + 1]++;
            }
        }
        for (size_t i = 0; i < nn; ++i) use_off[i + 1] += use_off[i];
        exp_at.clear();
        for (size_t t = 0; t < events.size(); ++t)
            if (!events[t].first && N[events[t].second].kind == PF_W_EXP) exp_at.push_back((int)t);
        use_at.assign(use_off[nn], 0);
        {
            std::vector<int> fill(use_off.begin(), use_off.end() - 1);
            for (size_t t = 0; t < events.size(); ++t) {
                const auto& e = events[t];
                if (!e.first) {
                    const Node& n = N[e.second];
                    for (uint32_t k = 0; k < n.nargs; ++k) use_at[fill[n.args[k]]++] = (int)t;
                } else {
                    use_at[fill[e.second]++] = (int)t;
                }
            }
        }
        for (size_t t = 0; t < events.size(); ++t) {
            const int i = events[t].second;
            if (events[t].first) {
                const int rb = materialize(i, (int)t, 0u, 0u);
                emit(PF_ASSERT, 1, 0, rb, 0, 0, 0);
                if (next_use(i, (int)t) >= INF) done(i);
                continue;
            }
            if (where[i] != NONE || slot_of[i] != NONE) continue;  // recomputed as an operand
            emit_node(i, (int)t, 0u, 0u);
            if (next_use(i, (int)t) >= INF) done(i);
        }
        if (code.empty() || (code[code.size() - 4] & 0xffu) != PF_END) emit(PF_END, 1, 0, 0, 0, 0, 0);
    }

   private:
    const Node* N;
    size_t nn;
    const Const8* pool;
    size_t n_pool;
    std::vector<std::pair<bool, int>> events;  // (is_assert, node)
    std::vector<int> use_off, use_at;  // uses of node i: use_at[use_off[i] .. use_off[i + 1])
    std::vector<int> where, slot_of, remat, cost, free_slots;
    int filling = NONE;  // the spilled node materialize() is restoring (not a steal candidate)
    int spill_min_uses = 1, spill_exp_uses = 99;
    std::vector<int> exp_at;  // event times of the W_EXP nodes, ascending
    RegFile W, B;

    // uses a variable evicted at t must still have to be spilled rather than regenerated
    int var_min_uses(int nd, int t) const {
        if (spill_exp_uses <= spill_min_uses || use_off[nd + 1] == use_off[nd]) return spill_min_uses;
        const int last = use_at[use_off[nd + 1] - 1];
        const auto it = std::upper_bound(exp_at.begin(), exp_at.end(), t);
        return (it != exp_at.end() && *it < last) ? spill_exp_uses : spill_min_uses;
    }

    void order(const uint32_t* roots, size_t n_roots) {
        std::vector<int> size(nn, 0);
        for (size_t i = 0; i < nn; ++i) {
            const Node& n = N[i];
            if (is_leaf(n.kind)) continue;
            long long s = 1;
            for (uint32_t k = 0; k < n.nargs; ++k) s += size[n.args[k]];
            size[i] = (int)std::min<long long>(s, 1 << 20);
        }
        std::vector<char> seen(nn, 0);
        for (size_t ri = 0; ri < n_roots; ++ri) {
            std::vector<std::pair<int, bool>> stack{{(int)roots[ri], false}};
            while (!stack.empty()) {
                auto [i, fin] = stack.back();
                stack.pop_back();
                const Node& n = N[i];
                if (is_leaf(n.kind)) continue;
                if (fin) {
                    if (!seen[i]) {
                        seen[i] = 1;
                        events.push_back({false, i});
                    }
                    continue;
                }
                if (seen[i]) continue;
                stack.push_back({i, true});
                // operands by subtree size, stable (insertion sort over <= 3)
                int args[3];
                const uint32_t na = n.nargs;
                for (uint32_t k = 0; k < na; ++k) {
                    const int a = (int)n.args[k];
                    uint32_t j = k;
                    while (j > 0 && size[args[j - 1]] > size[a]) {
                        args[j] = args[j - 1];
                        --j;
                    }
                    args[j] = a;
                }
                for (uint32_t k = 0; k < na; ++k) {
                    const int a = args[k];
                    if (!is_leaf(N[a].kind) && !seen[a]) stack.push_back({a, false});
                }
            }
            events.push_back({true, (int)roots[ri]});
        }
    }

    int uses_after(int nd, int now) const {
        const int* b = use_at.data() + use_off[nd];
        const int* e = use_at.data() + use_off[nd + 1];
        return (int)(e - std::upper_bound(b, e, now));
    }

    int next_use(int nd, int now) const {
        const int* b = use_at.data() + use_off[nd];
        const int* e = use_at.data() + use_off[nd + 1];
        const int* it = std::upper_bound(b, e, now);
        return it == e ? INF : *it;
    }

    int remat_size(int nd) {  // NONE = must stay resident
        if (remat[nd] != -2) return remat[nd];
        const Node& n = N[nd];
        int res;
        if (is_leaf(n.kind)) {
            res = 1;
        } else if (op_cost(n.kind, n.width) > 16 || n.kind == PF_W_EXP) {
            res = NONE;
        } else {
            int tot = 1;
            for (uint32_t k = 0; k < n.nargs && tot != NONE; ++k) {
                const int s = remat_size(n.args[k]);
                tot = s == NONE ? NONE : tot + s;
            }
            res = (tot != NONE && tot <= 6) ? tot : NONE;
        }
        remat[nd] = res;
        return res;
    }

    // GPU price of re-emitting nd in cheap instructions (only for rematerialisable nd): a
    // variable is a generator run, ~6 cheap ops (lower.py _VAR_REMAT_COST)
    int remat_cost(int nd) {
        if (cost[nd] >= 0) return cost[nd];
        const Node& n = N[nd];
        int c;
        if (n.kind == PFL_K_VAR || n.kind == PFL_K_BVAR) {
            c = 6;
        } else if (is_leaf(n.kind)) {
            c = 1;
        } else {
            c = 1;
            for (uint32_t k = 0; k < n.nargs; ++k) c += remat_cost(n.args[k]);
        }
        cost[nd] = c;
        return c;
    }

    RegFile& rf_of(int nd) { return N[nd].is_bool ? B : W; }

    void emit(uint32_t op, uint32_t width, uint32_t dst, uint32_t a, uint32_t b, uint32_t c, uint32_t aux0) {
        code.push_back((op & 0xffu) | ((width & 0x3ffu) << 8));
        code.push_back((dst & 0xffu) | ((a & 0xffu) << 8) | ((b & 0xffu) << 16) | ((c & 0xffu) << 24));
        code.push_back(aux0);
        code.push_back(0u);
    }

    uint32_t const_index(const Const8& v) {
        for (size_t i = 0; i < consts.size(); ++i)
            if (consts[i] == v) return (uint32_t)i;
        consts.push_back(v);
        return (uint32_t)(consts.size() - 1);
    }

    bool spill(int rg, int nd, int t, bool steal = true) {
        if (free_slots.empty()) {
            // a value that cannot be recomputed takes the slot of a spilled variable, the
            // one used farthest in the future (lower.py spill: the same choice)
            if (!steal) return false;
            int far_v = NONE, far_nu = -1;
            for (size_t v = 0; v < slot_of.size(); ++v) {
                // never the variable materialize() is filling right now (its slot is read
                // after the register is allocated)
                if (slot_of[v] == NONE || N[v].kind != PFL_K_VAR || (int)v == filling) continue;
                const int nu = next_use((int)v, t);
                if (far_v == NONE || nu >= far_nu) {
                    far_v = (int)v;
                    far_nu = nu;
                }
            }
            if (far_v == NONE) return false;
            free_slots.push_back(slot_of[far_v]);
            slot_of[far_v] = NONE;
        }
        const int s = free_slots.back();
        free_slots.pop_back();
        if (N[nd].is_bool)
            emit(PF_B_SPILL, 1, 0, rg, 0, 0, s);
        else
            emit(PF_W_SPILL, N[nd].width, 0, rg, 0, 0, s);
        slot_of[nd] = s;
        return true;
    }

    int alloc(RegFile& rf, int node, int t, uint32_t pinned) {
        int r;
        if (!rf.free_.empty()) {  // the lowest free register (lower.py _RegFile.alloc)
            auto it = std::min_element(rf.free_.begin(), rf.free_.end());
            r = *it;
            rf.free_.erase(it);
        } else {
            // evict the cheapest-to-restore value, farthest next use first (Belady)
            bool have = false;
            long long best_sz = 0, best_nu = 0;
            int best_r = -1;
            for (int rg = 0; rg < rf.n; ++rg) {
                const int nd = rf.holder[rg];
                if (nd == NONE || ((pinned >> rg) & 1u)) continue;
                if (slot_of[nd] == NONE && remat_size(nd) == NONE) continue;
                // a variable used again is spilled while a slot is free (lower.py
                // _VAR_SPILL_COST): one spill now, fills later, no generator re-run
                const int sz = slot_of[nd] != NONE ? 1
                             : (N[nd].kind == PFL_K_VAR && !free_slots.empty() &&
                                uses_after(nd, t) >= var_min_uses(nd, t)) ? 2
                                                                                : remat_cost(nd);
                const long long nu = -(long long)next_use(nd, t);
                if (!have || sz < best_sz || (sz == best_sz && (nu < best_nu || (nu == best_nu && rg < best_r)))) {
                    have = true;
                    best_sz = sz;
                    best_nu = nu;
                    best_r = rg;
                }
            }
            if (have) {
                r = best_r;
                const int old = rf.holder[r];
                if (N[old].kind == PFL_K_VAR && slot_of[old] == NONE && !free_slots.empty() &&
                    uses_after(old, t) >= var_min_uses(old, t))
                    spill(r, old, t, false);
            } else {  // spill the value used farthest in the future
                int vr = -1, vfar = -1;
                for (int rg = 0; rg < rf.n; ++rg) {
                    const int nd = rf.holder[rg];
                    if (nd == NONE || ((pinned >> rg) & 1u)) continue;
                    const int far = next_use(nd, t);
                    if (far > vfar || (far == vfar && rg > vr)) {
                        vfar = far;
                        vr = rg;
                    }
                }
                if (vr < 0 || !spill(vr, rf.holder[vr], t))
                    throw LowerError{fail(-2, "more than %d live %s values", rf.n, &rf == &W ? "W" : "B")};
                r = vr;
            }
            const int old = rf.holder[r];
            rf.holder[r] = NONE;
            where[old] = NONE;
        }
        rf.holder[r] = node;
        where[node] = r;
        return r;
    }

    void release(int nd) {
        RegFile& rf = rf_of(nd);
        const int r = where[nd];
        if (r != NONE) {
            where[nd] = NONE;
            rf.holder[r] = NONE;
            rf.free_.push_back(r);
        }
    }

    void done(int nd) {
        release(nd);
        if (slot_of[nd] != NONE) {
            free_slots.push_back(slot_of[nd]);
            slot_of[nd] = NONE;
        }
    }

    int emit_node(int i, int t, uint32_t pinned_w, uint32_t pinned_b) {
        const Node& n = N[i];
        RegFile& rf = rf_of(i);
        if (is_leaf(n.kind)) {
            const int r = alloc(rf, i, t, n.is_bool ? pinned_b : pinned_w);
            switch (n.kind) {
                case PFL_K_VAR: emit(PF_W_VAR, n.width, r, 0, 0, 0, n.aux); break;
                case PFL_K_CONST: {
                    if (n.aux >= n_pool) throw LowerError{fail(-1, "constant %u outside the pool", n.aux)};
                    emit(PF_W_CONST, n.width, r, 0, 0, 0, const_index(pool[n.aux]));
                    break;
                }
                case PFL_K_BCONST: emit(PF_B_CONST, 1, r, 0, 0, 0, n.aux); break;
                default: emit(PF_B_VAR, 1, r, 0, 0, 0, n.aux); break;
            }
            return r;
        }
        uint32_t pw = pinned_w, pb = pinned_b;
        int regs[3] = {0, 0, 0};
        for (uint32_t k = 0; k < n.nargs; ++k) {
            const int a = n.args[k];
            const int r = materialize(a, t, pw, pb);
            (N[a].is_bool ? pb : pw) |= 1u << r;
            regs[k] = r;
        }
        // operands whose last use is this node may be reused as the destination (distinct
        // operands in argument order, mythril_amd/lower.py)
        for (uint32_t k = 0; k < n.nargs; ++k) {
            const int a = n.args[k];
            bool dup = false;
            for (uint32_t j = 0; j < k; ++j) dup |= (int)n.args[j] == a;
            if (dup) continue;
            // not an operand the caller pinned (a remat inside an enclosing node's operand
            // list shares its event time: mythril_amd/lower.py)
            if (next_use(a, t) >= INF && !(((N[a].is_bool ? pinned_b : pinned_w) >> regs[k]) & 1u)) {
                done(a);
                (N[a].is_bool ? pb : pw) &= ~(1u << regs[k]);
            }
        }
        const int dst = alloc(rf, i, t, n.is_bool ? pb : pw);
        if (n.kind == PF_W_ITE || n.kind == PF_B_ITE)
            emit(n.kind, n.kind == PF_W_ITE ? n.width : 1, dst, regs[1], regs[2], regs[0], 0);
        else
            emit(n.kind, n.width, dst, regs[0], regs[1], 0, n.aux);
        return dst;
    }

    int materialize(int nd, int t, uint32_t pinned_w, uint32_t pinned_b) {
        RegFile& rf = rf_of(nd);
        if (where[nd] != NONE) return where[nd];
        if (slot_of[nd] != NONE) {
            const Node& n = N[nd];
            const int slot = slot_of[nd];
            const int outer = filling;
            filling = nd;
            const int r = alloc(rf, nd, t, n.is_bool ? pinned_b : pinned_w);
            filling = outer;
            if (n.is_bool)
                emit(PF_B_FILL, 1, r, 0, 0, 0, slot);
            else
                emit(PF_W_FILL, n.width, r, 0, 0, 0, slot);
            return r;
        }
        if (!is_leaf(N[nd].kind) && remat_size(nd) == NONE)
            throw LowerError{fail(-2, "non-rematerialisable value was evicted")};
        return emit_node(nd, t, pinned_w, pinned_b);
    }
};

}  // namespace

extern "C" {

int pfl_version(void) { return 2; }

const char* pfl_last_error(void) { return g_err.c_str(); }

int pfl_lower(const uint32_t* nodes, size_t n_nodes, const uint32_t* const_pool, size_t n_pool,
              const uint32_t* roots, size_t n_roots, const uint32_t* forced, size_t n_forced,
              uint32_t n_wregs, uint32_t* code_out, size_t cap_ins, size_t* n_ins_out,
              uint32_t* consts_out, size_t cap_const, size_t* n_const_out) {
    const Node* N = reinterpret_cast<const Node*>(nodes);
    if (n_wregs == 0) n_wregs = PF_NW;
    if (n_wregs < 3 || n_wregs > PF_NW) return fail(-1, "n_wregs %u outside [3, %d]", n_wregs, PF_NW);
    for (size_t i = 0; i < n_nodes; ++i) {  // shape checks: indices the lowering follows
        const Node& n = N[i];
        if (n.nargs > 3) return fail(-1, "node %zu: %u operands", i, n.nargs);
        for (uint32_t k = 0; k < n.nargs; ++k)
            if (n.args[k] >= i) return fail(-1, "node %zu: operand %u not before it", i, n.args[k]);
    }
    for (size_t r = 0; r < n_roots; ++r)
        if (roots[r] >= n_nodes || !N[roots[r]].is_bool) return fail(-1, "root %zu is not a Bool node", r);
    try {
        Lowerer L(N, n_nodes, reinterpret_cast<const Const8*>(const_pool), n_pool, (int)n_wregs);
        for (size_t f = 0; f < n_forced; ++f) {
            Const8 c;
            memcpy(c.l, forced + 8 * f, 32);
            L.consts.push_back(c);  // pinned at 0.. (no de-duplication, like Program.consts.extend)
        }
        L.run(roots, n_roots);
        const size_t ni = L.code.size() / 4;
        if (ni > cap_ins || L.consts.size() > cap_const) return fail(-3, "output capacity");
        memcpy(code_out, L.code.data(), L.code.size() * 4);
        if (!L.consts.empty()) memcpy(consts_out, L.consts.data(), L.consts.size() * 32);
        *n_ins_out = ni;
        *n_const_out = L.consts.size();
        return 0;
    } catch (const LowerError& e) {
        return e.rc;
    }
}

}  // extern "C"
