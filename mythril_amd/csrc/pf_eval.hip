// pf_eval.hip — gfx950 kernels of the batched path-feasibility engine.
//
// Execution model:
//   * one wavefront lane = one candidate assignment; a wave evaluates one constraint set's
//     bytecode for 64 candidates at a time.  The instruction stream is wave-uniform, so it
//     is fetched with scalar loads (s_load_dwordx4) and dispatched with scalar branches.
//   * the W register file is limb-sliced: bank k (an ext_vector of 16 dwords) holds limb k
//     of all 16 registers, so reading register r is one s_set_gpr_idx_on + 8 v_mov (the
//     index is an SGPR) — no scratch, no LDS.  Bool registers live in one 32-dword bank.
//   * candidates are generated in-register from Philox4x32-10 (include/pf_bytecode.h
//     contract); only (set, candidate index) ever leaves the kernel.
//   * ballot early exit: a wave records the smallest satisfying candidate with atomicMin
//     and stops; other waves of the set stop once a witness below their candidates exists.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pf_bytecode.h"
#include "u256.h"

using pf::u256;

// profiling buckets: the 8 datapath units, EXP (8), W_CONST (9), waiting for the next
// instruction's scalar fetch (10); slot = u64 index in the launch's counter scratch; bucket
// PF_PROF_BUCKETS = whole-wave time
#define PF_PROF_BUCKETS 18  // + DIV by udivrem256 path: 11 zero, 12 short, 13 one-digit, 14 general;
                            // EXP parts: 15 window, 16 t recurrence, 17 Horner + product
#define PF_PROF_SLOT 16

// Register file: NREG wide registers (NREG - 1 usable + the write sink), limb-sliced into
// 16-dword vectors.  NREG 16: vector k holds limb k of every register (8 vectors).  NREG 8:
// vector j holds limbs 2j and 2j+1 (element 2r + (k & 1)), 4 vectors — 64 VGPRs instead of
// 128, which is what lets that build run 3 waves per SIMD.  The vectors stay 16 wide either
// way: hipcc expands a dynamic index into a vector of 8 or fewer dwords into a v_cndmask
// tree (56 VALU per operand read) but indexes a 16-dword vector with s_set_gpr_idx (one
// v_mov per limb).
typedef uint32_t vbank __attribute__((ext_vector_type(16)));
// the instruction stream in the constant address space (scalar loads), as a clang vector
// (HIP's uint4 struct cannot be copied out of a non-generic address space)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) u32x4 pf_code_t;
PF_INL uint4 fetch_ins(const pf_code_t* p) {
    const u32x4 v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
typedef uint32_t v32u __attribute__((ext_vector_type(32)));

namespace {

// These are macros, not functions: taking the vector array by reference defeats
// AMDGPUPromoteAlloca (the banks land in scratch), while direct element accesses become one
// s_set_gpr_idx_on + 8 v_mov per operand.
#define RD_W(dst, W, r, LPB)                                                                  \
    do {                                                                                      \
        _Pragma("unroll") for (int k_ = 0; k_ < 8; k_++)                                    \
            (dst).l[k_] = (W)[k_ / (LPB)][(r) * (LPB) + (k_ % (LPB))];                         \
    } while (0)
// The 8-register kernels read and write registers through a uniform switch over the
// register number instead: static VGPR indices, no indexing mode (config 3 +0.8 %, and 8
// VGPRs fewer: 155).  The 16-register kernels keep s_set_gpr_idx (a 16-way switch per
// operand is a lot of code for the 0.4 % of sets that run them).
#define RD_CASE(dst, W, R, LPB)                                                            \
    case R:                                                                               \
        _Pragma("unroll") for (int k_ = 0; k_ < 8; k_++)                                  \
            (dst).l[k_] = (W)[k_ / (LPB)][(R) * (LPB) + (k_ % (LPB))];                     \
        break;
#define RD_SW(dst, W, r, LPB)                                                              \
    do {                                                                                  \
        switch (r) {                                                                      \
            RD_CASE(dst, W, 0, LPB) RD_CASE(dst, W, 1, LPB) RD_CASE(dst, W, 2, LPB)       \
            RD_CASE(dst, W, 3, LPB) RD_CASE(dst, W, 4, LPB) RD_CASE(dst, W, 5, LPB)       \
            default: RD_CASE(dst, W, 6, LPB)                                              \
        }                                                                                 \
    } while (0)
#define WR_CASE(W, R, src, LPB)                                                            \
    case R:                                                                               \
        _Pragma("unroll") for (int k_ = 0; k_ < 8; k_++)                                  \
            (W)[k_ / (LPB)][(R) * (LPB) + (k_ % (LPB))] = (src).l[k_];                     \
        break;
#define WR_SW(W, r, src, LPB)                                                              \
    do {                                                                                  \
        switch (r) {                                                                      \
            WR_CASE(W, 0, src, LPB) WR_CASE(W, 1, src, LPB) WR_CASE(W, 2, src, LPB)       \
            WR_CASE(W, 3, src, LPB) WR_CASE(W, 4, src, LPB) WR_CASE(W, 5, src, LPB)       \
            WR_CASE(W, 6, src, LPB) default: WR_CASE(W, 7, src, LPB)                      \
        }                                                                                 \
    } while (0)
// Narrow kernels: the register file is PF_NW_NARROW x 8 plain scalars, every access a
// static index under a uniform switch over the register number, so each limb is its own
// VGPR (no 16-dword vector tuples, no write sink): 56 VGPRs for 7 registers.
// The operand copy is one asm block per case: as plain assignments, the phi copies of a
// case were placed before the compare that leaves it (critical edges are not split), so a
// read of register 2 executed the copies of registers 0, 1 and 2 (24 v_mov, ~14 on average
// over the register mix instead of 8).  Early-clobber outputs: the moves run in order.
#ifndef PF_RD_PLAIN
#define PF_MOV8(d, s)                                                                        \
    asm("v_mov_b32 %0, %8\n\tv_mov_b32 %1, %9\n\tv_mov_b32 %2, %10\n\tv_mov_b32 %3, %11\n\t"     \
        "v_mov_b32 %4, %12\n\tv_mov_b32 %5, %13\n\tv_mov_b32 %6, %14\n\tv_mov_b32 %7, %15"          \
        : "=&v"((d).l[0]), "=&v"((d).l[1]), "=&v"((d).l[2]), "=&v"((d).l[3]), "=&v"((d).l[4]),     \
          "=&v"((d).l[5]), "=&v"((d).l[6]), "=&v"((d).l[7])                                      \
        : "v"((s)[0]), "v"((s)[1]), "v"((s)[2]), "v"((s)[3]), "v"((s)[4]), "v"((s)[5]),           \
          "v"((s)[6]), "v"((s)[7]))
#define RDN_CASE(dst, W, R)                                                                \
    case R:                                                                               \
        PF_MOV8(dst, (W)[R]);                                                             \
        break;
#else
#define RDN_CASE(dst, W, R)                                                                \
    case R:                                                                               \
        _Pragma("unroll") for (int k_ = 0; k_ < 8; k_++)(dst).l[k_] = (W)[R][k_];          \
        break;
#endif
#define WRN_CASE(W, R, src)                                                                \
    case R:                                                                               \
        _Pragma("unroll") for (int k_ = 0; k_ < 8; k_++)(W)[R][k_] = (src).l[k_];          \
        break;
// Where the next instruction's fetch is issued.  Default: right after this instruction's
// decode, before its operand reads.  PF_FETCH_LATE issues it after the operand reads, with an
// explicit lgkmcnt(0) after each LDS operand read: LDS reads and scalar loads share lgkmcnt
// and scalar loads return out of order, so with the early fetch the compiler's wait at the
// join of the operand switch also waits for the fetch in flight.  Measured on config 3
// (round 4, two A/B pairs on one box): the late fetch is 1.9 % SLOWER (14.54 vs 14.26 ms) —
// the fetch latency the early issue exposes at that join is smaller than what it hides.
#ifndef PF_FETCH_LATE
#define PF_FETCH_EARLY
#endif
#ifndef PF_FETCH_EARLY
#define PF_WAIT_LDS() __builtin_amdgcn_s_waitcnt(0xC07F)  // lgkmcnt(0)
#else
#define PF_WAIT_LDS() ((void)0)
#endif
#if PF_NW_NARROW == 7
// Registers 5 and 6 live in LDS, one 32-byte slot per lane each: entry 0 of EXP's window
// table (which keeps base^0 = 1 out of it) and one entry past it (PF_LDS_WREG6).  40 VGPRs of
// register file is what lets the kernel run 4 waves per SIMD without spilling; the lowering
// hands out the lowest free register, so 5 and 6 are the least used (15 % of the operand
// traffic on config 3).
#define RDN_SW(dst, W, r, LT)                                                              \
    do {                                                                                  \
        switch (r) {                                                                      \
            RDN_CASE(dst, W, 0) RDN_CASE(dst, W, 1) RDN_CASE(dst, W, 2) RDN_CASE(dst, W, 3) \
            RDN_CASE(dst, W, 4)                                                           \
            case 5: (dst) = pf::tbl_get(LT, 64u, PF_LDS_WREG5); PF_WAIT_LDS(); break;       \
            default: (dst) = pf::tbl_get(LT, 64u, PF_LDS_WREG6); PF_WAIT_LDS(); break;      \
        }                                                                                 \
    } while (0)
#define WRN_SW(W, r, src, LT)                                                              \
    do {                                                                                  \
        switch (r) {                                                                      \
            WRN_CASE(W, 0, src) WRN_CASE(W, 1, src) WRN_CASE(W, 2, src) WRN_CASE(W, 3, src) \
            WRN_CASE(W, 4, src)                                                           \
            case 5: pf::tbl_put(LT, 64u, PF_LDS_WREG5, src); break;                         \
            default: pf::tbl_put(LT, 64u, PF_LDS_WREG6, src); break;                        \
        }                                                                                 \
    } while (0)
#if PF_EXP_SPLIT > 32
#error "the narrow kernels' LDS registers need exp256_w32 (PF_EXP_SPLIT <= 32)"
#endif
#elif PF_NW_NARROW == 6
#define RDN_SW(dst, W, r, LT)                                                                  \
    do {                                                                                  \
        switch (r) {                                                                      \
            RDN_CASE(dst, W, 0) RDN_CASE(dst, W, 1) RDN_CASE(dst, W, 2) RDN_CASE(dst, W, 3) \
            RDN_CASE(dst, W, 4) default: RDN_CASE(dst, W, 5)                              \
        }                                                                                 \
    } while (0)
#define WRN_SW(W, r, src, LT)                                                              \
    do {                                                                                  \
        switch (r) {                                                                      \
            WRN_CASE(W, 0, src) WRN_CASE(W, 1, src) WRN_CASE(W, 2, src) WRN_CASE(W, 3, src) \
            WRN_CASE(W, 4, src) default: WRN_CASE(W, 5, src)                              \
        }                                                                                 \
    } while (0)
#else
#error "PF_NW_NARROW must be 6 or 7"
#endif
#define WR_W(W, r, src, LPB)                                                                  \
    do {                                                                                      \
        _Pragma("unroll") for (int k_ = 0; k_ < 8; k_++)                                    \
            (W)[k_ / (LPB)][(r) * (LPB) + (k_ % (LPB))] = (src).l[k_];                         \
    } while (0)

// Explicit waits at the end of the datapath arms that load (constants, generator, spill
// fills, EXP's LDS table): the arms join at the write-back, and a load still pending there on
// ANY incoming path makes the compiler put `s_waitcnt vmcnt(0) lgkmcnt(0)` in the shared
// write-back, where lgkmcnt(0) also waits for the next instruction's scalar fetch issued at
// the top of this one — every bytecode instruction then paid the fetch latency.
#define PF_WAIT_ALL() __builtin_amdgcn_s_waitcnt(0)
// vector-memory loads only (vmcnt(0) expcnt(7) lgkmcnt(15)): the generator's loads are
// vector gathers, and lgkmcnt would also wait for the next instruction's scalar fetch
#ifdef PF_GEN_WAIT_VM
#define PF_WAIT_GEN() __builtin_amdgcn_s_waitcnt(0x0F70)
#else
#define PF_WAIT_GEN() PF_WAIT_ALL()
#endif

// per-limb mask for width w.  w is wave-uniform (it comes from the scalar-loaded
// instruction); the mask is formed from the top limb index and its partial mask with
// scalar selects, and readfirstlane pins the result to an SGPR — the plain expression was
// compiled to ~6 VALU instructions per limb (~56 per masked op: as much as a cheap op
// itself, on every op narrower than 256 bits — LASER's bytes and addresses).
PF_INL uint32_t limb_mask(uint32_t w, int i) {
    const uint32_t li = (w - 1u) >> 5, r = w & 31u;
    const uint32_t top = r ? ((1u << r) - 1u) : 0xffffffffu;
    const uint32_t m = (uint32_t)i < li ? 0xffffffffu : ((uint32_t)i == li ? top : 0u);
    return __builtin_amdgcn_readfirstlane(m);
}

// Re-mask a W result to width w (wave-uniform).  A switch on the top limb: the limbs
// above it are zeroed and only the top limb is and-ed — per-limb masks formed with scalar
// selects cost ~35 SALU per narrow op.
PF_INL void maskw(u256& x, uint32_t w) {
    if (__builtin_expect(w < 256u, 0)) {
        const uint32_t r = w & 31u;
        const uint32_t top = r ? ((1u << r) - 1u) : 0xffffffffu;
#define PF_MASK_CASE(K)                                                   \
    case K:                                                               \
        x.l[K] &= top;                                                    \
        _Pragma("unroll") for (int i_ = K + 1; i_ < 8; i_++) x.l[i_] = 0u; \
        break;
        switch ((w - 1u) >> 5) {
            PF_MASK_CASE(0)
            PF_MASK_CASE(1)
            PF_MASK_CASE(2)
            PF_MASK_CASE(3)
            PF_MASK_CASE(4)
            PF_MASK_CASE(5)
            PF_MASK_CASE(6)
            default: x.l[7] &= top; break;
        }
#undef PF_MASK_CASE
    }
}

// sign-extend a w-bit value (bits >= w zero) to 256 bits
PF_INL u256 sextw(const u256& x, uint32_t w) {
    if (w >= 256u) return x;
    uint32_t li = (w - 1u) >> 5, bi = (w - 1u) & 31u;
    uint32_t word = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) word = ((uint32_t)i == li) ? x.l[i] : word;
    uint32_t fill = 0u - ((word >> bi) & 1u);
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = x.l[i] | (fill & ~limb_mask(w, i));
    return r;
}

// value >= w (shift amounts)
PF_INL uint32_t ge_width(const u256& b, uint32_t w) {
    uint32_t hi = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) hi |= b.l[i];
    return (uint32_t)(hi != 0u) | (uint32_t)(b.l[0] >= w);
}

PF_INL u256 pow2(uint32_t k) {  // 2^k, k < 256 (per lane)
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.l[i] = ((k >> 5) == (uint32_t)i) ? (1u << (k & 31u)) : 0u;
    return r;
}

PF_INL u256 pow2m1(uint32_t k) {  // 2^k - 1
    u256 r;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t li = k >> 5;
        r.l[i] = ((uint32_t)i < li) ? 0xffffffffu : (((uint32_t)i == li) ? ((1u << (k & 31u)) - 1u) : 0u);
    }
    return r;
}

#if defined(PF_PROBE_2X_GEN) || defined(PF_PROBE_2X_DIV) || defined(PF_PROBE_2X_EXP) || \
    defined(PF_PROBE_2X_MUL) || defined(PF_PROBE_2X_PHILOX)
// Doubling probes (timing only, tools/gpu_probe2x.sh): a unit runs twice on operands that
// differ by a per-lane zero the compiler cannot see through, and the second result is folded
// in under that zero — same values, same branches, twice the unit's issue.  The time added is
// the unit's marginal cost in the running kernel, without the value shift of a removal probe.
PF_INL uint32_t hidden_zero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
#endif

// boundary-arm deltas (gen_var): entry j in bits 3j..3j+2, biased by 2
#define PF_BND_DELTA 0x2ca281b1aull

// ---- Philox4x32-10 -------------------------------------------------------------------
// 32 x 32 -> 64 product as ONE v_mad_u64_u32 (addend 0): the backend otherwise emits a
// v_mul_lo_u32 + v_mul_hi_u32 pair, two quarter-rate instructions for the same product.
PF_INL uint64_t mul_wide(uint32_t a, uint32_t m) {
    uint64_t r, c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(c) : "v"(a), "s"(m));
    return r;
}

// rounds FIRST..9 of Philox4x32-10 (k0, k1 already advanced FIRST times)
template <int FIRST>
PF_INL uint4 philox_tail(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = FIRST; i < 10; i++) {
        const uint64_t p0 = mul_wide(c.x, PF_PHILOX_M0), p1 = mul_wide(c.z, PF_PHILOX_M1);
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        // the two 3-input xors as one v_bitop3_b32 each (truth table 0x96)
        c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, (unsigned char)0x96), lo1,
                       __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, (unsigned char)0x96), lo0);
        k0 += PF_PHILOX_W0;
        k1 += PF_PHILOX_W1;
    }
    return c;
}

PF_INL uint4 philox(uint4 c, uint32_t k0, uint32_t k1) { return philox_tail<0>(c, k0, k1); }

// philox(make_uint4(cand, v, z, 0), k0, k1), bit for bit, for the generator's counters:
// only cand varies per lane, so round 1's second product (z * M1) is a constant, its first
// (cand * M0, passed in as p0) is shared by the three blocks of a variable, and round 2's
// first product has a wave-uniform operand and runs on the scalar unit — 17 per-lane
// v_mad_u64_u32 per block instead of 20
PF_INL uint4 philox_gen(uint64_t p0, uint32_t v, uint32_t z, uint32_t k0, uint32_t k1) {
    const uint64_t p1 = (uint64_t)z * PF_PHILOX_M1;
    const uint32_t x1 = (uint32_t)(p1 >> 32) ^ v ^ k0;  // uniform
    const uint32_t y1 = (uint32_t)p1;                   // constant
    const uint32_t z1 = (uint32_t)(p0 >> 32) ^ k1;      // per lane (counter word 3 is 0)
    const uint32_t w1 = (uint32_t)p0;                   // per lane
    k0 += PF_PHILOX_W0;
    k1 += PF_PHILOX_W1;
    const uint64_t q0 = (uint64_t)x1 * PF_PHILOX_M0;    // uniform: scalar multiply
    const uint64_t q1 = mul_wide(z1, PF_PHILOX_M1);
    const uint4 c = make_uint4((uint32_t)(q1 >> 32) ^ (y1 ^ k0), (uint32_t)q1,
                               ((uint32_t)(q0 >> 32) ^ k1) ^ w1, (uint32_t)q0);
    return philox_tail<2>(c, k0 + PF_PHILOX_W0, k1 + PF_PHILOX_W1);
}

struct SetCtx {
    const uint4* code;    // instruction stream of this set
    const uint32_t* consts;   // this set's constants (8 u32 each)
    const uint4* schema;  // this set's variable schema
    const uint32_t* parents;  // parent values base (global) or null
    uint32_t n_ins, n_const, n_vars, seed;
    uint32_t k0, k1;      // Philox key
    uint32_t nc_rcp;      // urcp32(n_const) (0 without constants): gen_var's x % n_const
};

// x % d for 32-bit unsigned x, d >= 1, split so the reciprocal of a divisor that stays
// fixed (a set's constant count) is formed once per set instead of in every generator call:
// the backend's own expansion of a 32-bit udiv/urem (an f32 reciprocal estimate, one
// Newton-Raphson step, a quotient estimate low by at most two, two corrections) — exact
// for every x and d >= 1, the same values as the `%` it replaces
PF_INL uint32_t urcp32(uint32_t d) {
    uint32_t z = (uint32_t)(__builtin_amdgcn_rcpf((float)d) * 4294966784.0f);  // 0x4f7ffffe
    return z + __umulhi(z, (0u - d) * z);
}
PF_INL uint32_t umod_rcp(uint32_t x, uint32_t d, uint32_t z) {
    uint32_t r = x - __umulhi(x, z) * d;
    r = r >= d ? r - d : r;
    return r >= d ? r - d : r;
}

// candidate value of variable v (include/pf_bytecode.h generator contract).
// Laid out for latency, not branches: the three Philox blocks depend only on (cand, v, key)
// and are formed before anything waits on the schema, parent or constant loads; the
// strategy arms (random / boundary / constant +-1 / parent mutation / small) are each
// computed for every lane and selected, so the wave runs one straight sequence instead of
// walking a lane-divergent if-chain; the per-variable kind stays a (uniform) branch.
PF_INL u256 gen_var(const SetCtx& S, uint32_t v, uint32_t cand) {
    const uint4 sc = S.schema[v];  // uniform -> scalar load
    const uint64_t p0 = mul_wide(cand, PF_PHILOX_M0);  // round 1 of all three blocks
#ifdef PF_PROBE_2X_PHILOX
    uint4 m = philox_gen(p0, v, 2u, S.k0, S.k1);
    const uint32_t hzp = hidden_zero();
    {
        const uint64_t p0b = mul_wide(cand ^ hzp, PF_PHILOX_M0);
        const uint4 mb = philox_gen(p0b, v, 2u, S.k0, S.k1);
        const uint4 r0b = philox_gen(p0b, v, 0u, S.k0, S.k1);
        const uint4 r1b = philox_gen(p0b, v, 1u, S.k0, S.k1);
        m.w ^= (mb.w ^ r0b.x ^ r1b.y) & hzp;
    }
#else
    const uint4 m = philox_gen(p0, v, 2u, S.k0, S.k1);
#endif
    const uint32_t kind = sc.x & 0xffu, w = (sc.x >> 8) & 0x3ffu;
    const uint32_t hint0 = sc.y, hint1 = sc.z, pslot = sc.w;
    // The one per-lane gather (a constant of the set for the +-1 arm, or the actor table
    // entry) is issued here, in the entry block, so the two Philox blocks below cover its
    // latency; inside the strategy branches it was waited for a dozen instructions after
    // issue.  Its address is always in bounds: the pool carries one zero entry past its end
    // (pathfeas.hip), so a set without constants reads that.
    const uint32_t ai = m.y & 3u;
    const uint32_t act = (uint32_t)(kind == PF_VK_ACTOR) & (uint32_t)(ai < hint1);
    const uint32_t ci = S.n_const ? umod_rcp(m.y, S.n_const, S.nc_rcp) : 0u;
    const uint32_t* gp = S.consts + (size_t)(act ? hint0 + ai : ci) * 8u;
    u256 g;
#ifdef PF_DIAG_NO_GATHER  // timing probe only: the per-lane gather's cost
    g = pf::zero256(); g.l[0] = (uint32_t)(size_t)gp;
#else
#pragma unroll
    for (int i = 0; i < 8; i++) g.l[i] = gp[i];
#endif
    const uint4 r0 = philox_gen(p0, v, 0u, S.k0, S.k1);
    // r1 only feeds limbs 4..7 of the random arm, which the final mask clears for w <= 128
    // (bytes, selectors, small counters): skipped there under a wave-uniform branch
    uint4 r1 = make_uint4(0u, 0u, 0u, 0u);
#ifdef PF_DIAG_R1_CHEAP  // timing probe only (wrong values): limbs 4..7 from a cheap mix of r0
    if (w > 128u) {
        r1.x = __umulhi(r0.x ^ 0x9E3779B9u, 0xD2511F53u) ^ r0.w;
        r1.y = __umulhi(r0.y ^ 0x7F4A7C15u, 0xCD9E8D57u) ^ r0.x;
        r1.z = __umulhi(r0.z ^ 0x85EBCA6Bu, 0xD2511F53u) ^ r0.y;
        r1.w = __umulhi(r0.w ^ 0xC2B2AE35u, 0xCD9E8D57u) ^ r0.z;
    }
#else
    if (w > 128u) r1 = philox_gen(p0, v, 1u, S.k0, S.k1);
#endif
    const bool has_parent = pslot != PF_NO_PARENT;
    u256 par = pf::zero256();
    if (has_parent) {
        const uint32_t* pp = S.parents + (size_t)pslot * 8u;
#pragma unroll
        for (int i = 0; i < 8; i++) par.l[i] = pp[i];
    }
    u256 rv;
    rv.l[0] = r0.x; rv.l[1] = r0.y; rv.l[2] = r0.z; rv.l[3] = r0.w;
    rv.l[4] = r1.x; rv.l[5] = r1.y; rv.l[6] = r1.z; rv.l[7] = r1.w;
    u256 out = pf::zero256();
    if (kind == PF_VK_KECCAK) {
        const uint32_t* lo = S.consts + (size_t)hint0 * 8u;
        u256 k = pf::zero256();
        k.l[0] = r0.x << 6;
        k.l[1] = (r0.y << 6) | (r0.x >> 26);
        k.l[2] = (r0.z << 6) | (r0.y >> 26);
        k.l[3] = ((r0.w & 0x1fffffu) << 6) | (r0.z >> 26);
        u256 base;
#pragma unroll
        for (int i = 0; i < 8; i++) base.l[i] = lo[i];
        out = pf::add256(base, k);
    } else if (kind == PF_VK_SMALL) {
        out.l[0] = (hint0 == 0xffffffffu) ? r0.x : (r0.x % (hint0 + 1u));
#ifndef PF_DIAG_NO_LASER_ARMS
        if (hint0 >= 4u && hint0 != 0xffffffffu) {  // uniform: ABI-aligned sizes in half the lanes
            const uint32_t al = 4u + 32u * (r0.y % ((hint0 - 4u) / 32u + 1u));
            out.l[0] = (m.x & 16u) ? al : out.l[0];
        }
#endif
    } else if (kind == PF_VK_BOOL) {
        out.l[0] = r0.x & 1u;
    } else {
        const uint32_t sel = m.x & 15u;
        // constant +-1 arm (sel 9..11)
        u256 cst = rv;
        if (S.n_const > 0u) {
            const uint32_t dsel = m.z % 3u;  // +0, +1, -1
            u256 dl;
            dl.l[0] = dsel == 0u ? 0u : (dsel == 1u ? 1u : 0xffffffffu);
#pragma unroll
            for (int i = 1; i < 8; i++) dl.l[i] = dsel == 2u ? 0xffffffffu : 0u;
            cst = pf::add256(g, dl);
        }
        // boundary arm (sel 5..8): {0, 1, 2, 3, 2^w-1, 2^w-2, 2^(w-1), 2^(w-1)-1, 2^k, 2^k-1,
        // 2^k+1, 2^160-1}[j] mod 2^w as one formula, (j >= 6 ? 2^p : 0) + delta
        // one power of two serves both the boundary arm (2^p) and the parent-mutation arm
        // (2^k, k = m[2] % w): a lane takes one arm, so the exponent is selected per lane
        // (w is uniform; a power of two — every 256-bit variable — needs no division)
        const uint32_t j = m.y % 12u, k = (w & (w - 1u)) == 0u ? (m.z & (w - 1u)) : m.z % w;
        const uint32_t p = j <= 7u ? w - 1u : (j <= 10u ? k : 160u);
        const u256 pw = pow2(sel <= 8u ? p : k);
        u256 bnd;
        {
            // delta by j, 3 bits per entry biased by 2 (a ternary chain here became a
            // divergent if-chain): j 0..11 -> 0 1 2 3 -1 -2 0 -1 0 -1 1 -1
            const int32_t delta = (int32_t)((PF_BND_DELTA >> (3u * j)) & 7ull) - 2;
            u256 base = pw;
            const uint32_t usepow = j >= 6u ? 0xffffffffu : 0u;
            u256 dl;
            dl.l[0] = (uint32_t)delta;
#pragma unroll
            for (int i = 1; i < 8; i++) dl.l[i] = delta < 0 ? 0xffffffffu : 0u;
#pragma unroll
            for (int i = 0; i < 8; i++) base.l[i] &= usepow;
            bnd = pf::add256(base, dl);
        }
        // parent-mutation arm (sel 12..13): one bit of the parent flipped in a quarter of
        // the lanes; without a parent, a random byte
        u256 mut = pf::zero256();
        if (has_parent) {
            const uint32_t flip = (m.y & 3u) == 0u ? 0xffffffffu : 0u;
#pragma unroll
            for (int i = 0; i < 8; i++) mut.l[i] = par.l[i] ^ (pw.l[i] & flip);
        } else {
            mut.l[0] = r0.x & 0xffu;
        }
        // small arm (sel 14..15): 1..16 random low bits
        const uint32_t nb = 1u + (m.y & 15u);
        const uint32_t small = r0.x & ((nb >= 32u) ? 0xffffffffu : ((1u << nb) - 1u));
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t sm = i == 0 ? small : 0u;
            out.l[i] = sel <= 4u ? rv.l[i]
                     : (sel <= 8u ? bnd.l[i] : (sel <= 11u ? cst.l[i] : (sel <= 13u ? mut.l[i] : sm)));
            // the actor set (transaction/symbolic.py:215) in most lanes
            out.l[i] = act ? g.l[i] : out.l[i];
        }
#ifndef PF_DIAG_NO_LASER_ARMS  // timing probe only: the LASER-aware arms compiled out
        if (kind == PF_VK_VALUE) {  // uniform: call values are 0 in half the lanes
#pragma unroll
            for (int i = 0; i < 8; i++) out.l[i] = (m.x & 16u) ? 0u : out.l[i];
        }
        if (kind == PF_VK_CDBYTE) {
            // calldata bytes (uniform branch, after the generic arms so nothing of it lives
            // across the Philox blocks): one hash per (candidate, ABI word) decides whether
            // the word is spelled from one of the set's word constants const[ws .. ws + wk)
            // (+-1), which every byte of the word then agrees on
            uint32_t wk = (hint0 >> 8) & 0xfffu, ws = hint0 >> 20;
            if (wk == 0u) { wk = S.n_const; ws = 0u; }
            if (wk) {
                uint32_t u = cand ^ S.k0 ^ (hint1 * PF_CDWORD_MUL);
                u ^= u >> 16; u *= PF_MIX_M1; u ^= u >> 15; u *= PF_MIX_M2; u ^= u >> 16;
                const uint32_t cdd = u >> 30;  // the word's neighbour: +0, +1, -1, +0
                const uint32_t* wp = S.consts + (size_t)(ws + (u >> 1) % wk) * 8u;
                u256 cw, dl;
#pragma unroll
                for (int i = 0; i < 8; i++) cw.l[i] = wp[i];
                dl.l[0] = cdd == 1u ? 1u : (cdd == 2u ? 0xffffffffu : 0u);
#pragma unroll
                for (int i = 1; i < 8; i++) dl.l[i] = cdd == 2u ? 0xffffffffu : 0u;
                cw = pf::add256(cw, dl);
                const uint32_t li = (hint0 >> 5) & 7u;
                uint32_t word = cw.l[0];
#pragma unroll
                for (int i = 1; i < 8; i++) word = li == (uint32_t)i ? cw.l[i] : word;
                const uint32_t byte = (word >> (hint0 & 24u)) & 0xffu;
                out.l[0] = (u & 1u) ? byte : out.l[0];
            }
        }
#endif
    }
    // the parent model itself (candidate 0) and its neighbourhood (odd candidates keep the
    // parent value of most variables)
    if (has_parent) {
        const uint32_t keep = (uint32_t)(cand == 0u) |
                              ((cand & 1u) & (uint32_t)((m.w & ((4u << ((cand >> 1) & 3u)) - 1u)) != 0u));
        out = pf::sel256(keep, par, out);
    }
    maskw(out, w);
    return out;
}

enum Mode { MODE_GEN = 0, MODE_SOA = 1 };



// Per-unit cycle accounting (profiling builds only, tools/unitprof.py): s_memtime deltas of
// every bytecode instruction, bucketed by datapath unit (EXP separately), kept in SGPRs.
struct UnitProf {
    uint64_t c[PF_PROF_BUCKETS];
};
#ifdef PF_PROFILE_UNITS
PF_INL void prof_add(UnitProf* P, uint32_t b, uint64_t dt) {
#pragma unroll
    for (int i = 0; i < PF_PROF_BUCKETS; i++)
        if (b == (uint32_t)i) P->c[i] += dt;
}
#endif

// LDS for EXP's window table (pf::exp256): 2^WB entries x 4 limb pairs per lane, 64 lanes,
// 4 waves per 256-thread workgroup (2-bit window: 32 KiB, so PF_WG_PER_CU workgroups fit
// in the CU's 160 KiB).
// One more 32-byte entry per lane after the table: the narrow kernels' LDS registers are
// that entry and the table's entry 0 (PF_LDS_WREG5/6).  40 KiB per 256-thread workgroup: 4 workgroups fill the CU's 160 KiB.
#define PF_LDS_WREG5 0u
#define PF_LDS_WREG6 PF_EXP_TBL_ENTRIES
#define PF_LDS_ENTRIES (PF_EXP_TBL_ENTRIES + 1)
#define PF_EXP_LDS_U2 (4 * PF_LDS_ENTRIES * 4 * 64)
// search kernels: PF_SEARCH_WG_WAVES waves per workgroup (pathfeas.hip launches with the
// same constant from include/pathfeas.h)
#define PF_SEARCH_LDS_U2 (PF_SEARCH_WG_WAVES * PF_LDS_ENTRIES * 4 * 64)
PF_INL uint2* exp_tbl_of(uint2* lds) {
    return lds + (threadIdx.x >> 6) * (PF_LDS_ENTRIES * 4 * 64) + (threadIdx.x & 63u);
}
#ifndef PF_WG_PER_CU_NARROW
#define PF_WG_PER_CU_NARROW 4
#endif
#ifndef PF_WG_PER_CU
#define PF_WG_PER_CU 2
#endif

// Run one set's program for this lane's candidate.  Returns the lane's root (0/1);
// *complete = 1 if the program ran to END (not short-circuited).  `ops` accumulates
// aux1 (per-lane algorithmic cost) of every executed instruction.
template <int MODE, int NREG>
PF_INL uint32_t run_program(const SetCtx& S, uint32_t cand, bool active, uint32_t flags,
                            const uint32_t* __restrict__ soa, uint32_t soa_n,
                            uint2* exp_tbl, uint32_t* complete, uint64_t* ops, UnitProf* prof) {
    // No initialisation: pf_batch_create rejects programs that read a register before
    // writing it, so the banks never leak values between candidates.
    constexpr int LPB = 16 / NREG;  // limbs per vector
    vbank W[8 / LPB];               // wide kernels (NREG 16)
    uint32_t Wn[PF_NW_NARROW][8];   // narrow kernels (NREG 8)
    // the 32 bool registers are the bits of one VGPR (bit r = B register r)
    uint32_t Bk = 0u;
    // spill slots (lowering under register pressure): dynamically indexed, so the compiler
    // keeps them in private scratch memory, never in the VGPR banks
    // physical spill slot of bytecode slot k (PF_SPILL_ROT: rotated by the wave's hardware
    // slot, a probe of how the scratch lines of the 4096 waves share the L2)
#ifdef PF_SPILL_ROT
    const uint32_t spill_rot = __builtin_amdgcn_readfirstlane(blockIdx.x);
#define PF_SLOT(k) (((k) + spill_rot) & (PF_MAX_SPILL - 1u))
#else
#define PF_SLOT(k) ((k) & (PF_MAX_SPILL - 1u))
#endif
// Extra private dwords per lane.  The spill slots live in each wave's scratch window, and
// with 2,064 B per lane the windows are 0x20400 bytes apart, so the slot-0 lines of the 4,096
// resident waves collided in the L2 and were evicted to memory: WRITE_SIZE 115 MB per
// config-3 launch, of which 11 MB without any spill (PF_VAR_SPILL_USES=99).  A 256-byte pad
// per lane (window 0x24400) halves it, 53 MB, at the same speed (profiles/r04e_*, r04f_*:
// pads of 32 B .. 1 KB and a per-wave slot rotation all land at 53–64 MB); the rest is the
// spill stores themselves (PF_VAR_SPILL_USES=3: 31 MB at -0.4 %, =99: 11 MB at -0.9 %).
#ifndef PF_SPILL_PAD
#define PF_SPILL_PAD 64
#endif
    uint32_t spill[PF_MAX_SPILL * 8 + PF_SPILL_PAD];
#if PF_SPILL_PAD
    if (__builtin_expect(cand == 0xFFFFFFFFu, 0)) spill[PF_MAX_SPILL * 8 + PF_SPILL_PAD - 1] = 0u;  // keep the pad
#endif
#define BGET(r) ((Bk >> ((r) & 31u)) & 1u)
#define BSET(r, v) (Bk = (Bk & ~(1u << ((r) & 31u))) | (((v) & 1u) << ((r) & 31u)))
    // Ops with a B result (compares, bool logic, B_VAR, UMUL_NOOVF) set their bit and skip
    // the W write-back: a uniform branch to the loop latch.
    // PF_ASSERT (or a PF_I_ASSERT-flagged B op): and the lane's bit into the root; with
    // PF_FLAG_SHORTCIRCUIT a wave whose every lane is decided leaves the program (the next
    // instruction becomes END; the fetch in flight is dropped)
#define PF_DO_ASSERT(v)                                                                       \
    do {                                                                                      \
        root &= (v);                                                                          \
        if ((flags & PF_FLAG_SHORTCIRCUIT) && __ballot(root & (uint32_t)active) == 0ull) {   \
            In = make_uint4(PF_U_END << 21, 0u, 0u, 0u);                                      \
            sc = 1u;                                                                          \
        }                                                                                     \
    } while (0)
#ifdef PF_PROFILE_UNITS
#define PF_NEXT()                                                                      \
    {                                                                                  \
        prof_add(prof, pbucket, __builtin_amdgcn_s_memtime() - t_ins);                 \
        continue;                                                                      \
    }
#else
#define PF_NEXT() continue
#endif
    uint32_t root = 1u, sc = 0u;
    uint64_t cost = 0;
    // Software-pipelined fetch: the scalar load of instruction i+1 is issued while
    // instruction i executes.  The loop ends at PF_END (pf_batch_create checks that every
    // program ends with it), which is decoded before the next fetch, so no load reads past
    // the program and the loop needs no instruction counter.
    // The stream is read through the constant address space: the kernel's LDS and scratch
    // stores made hipcc treat the code as possibly clobbered, and it then fetched every
    // instruction with a vector load waited on at once (plus 4 readfirstlanes) instead of
    // the pipelined scalar load
    const pf_code_t* ip = (const pf_code_t*)S.code;
    uint4 In = fetch_ins(ip);
    // z, the W result, lives across iterations: at the top of an instruction it still holds
    // the last W result, which PF_I_FA / PF_I_FB operands read (pf_batch_create's forwarding
    // peephole sets them only on the instruction right after a W write; nothing writes z in
    // between — B ops and the narrow W_SPILL leave before the write-back)
    u256 z;
#ifndef PF_NO_FORWARD
#define PF_FWD_A() else if (I.x & PF_I_FA) x = z
#define PF_FWD_B() else if (I.x & PF_I_FB) y = z
#define PF_FWD_WB(tr) __builtin_expect(((tr) & PF_TR_WW) != 0u, 1)
#else
#define PF_FWD_A() else {}
#define PF_FWD_B() else {}
#define PF_FWD_WB(tr) true
#endif
    for (;;) {
#ifdef PF_PROFILE_UNITS
        {
            const uint64_t t_f = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the fetch of this instruction
            prof_add(prof, 10u, __builtin_amdgcn_s_memtime() - t_f);
        }
#endif
        const uint4 I = In;
        const uint32_t op = I.x & 0xffu;
        const uint32_t w = (I.x >> 8) & 0x3ffu;
        const uint32_t tr = (I.x >> 18) & 7u;
        const uint32_t unit = (I.x >> 21) & 7u;
        const uint32_t d = I.y & 0xffu, a = (I.y >> 8) & 0xffu, b = (I.y >> 16) & 0xffu,
                       c = (I.y >> 24) & 0xffu;
        const uint32_t aux = I.z;
        cost += I.w;
#ifdef PF_PROFILE_UNITS
        const uint64_t t_ins = __builtin_amdgcn_s_memtime();
        uint32_t pbucket = op == PF_W_EXP ? 8u : (op == PF_W_CONST ? 9u : unit);
#endif
        // branch hints: every taken scalar branch refetches the wave's instruction buffer, so
        // the common path (operands read) is laid out as the fall-through.  END is a case
        // of the unit dispatch below, not a test of its own on every instruction: it reads
        // no operand (traffic bits 0) and its fetch of the slot after it stays inside the
        // batch (pf_batch_create pads the code region by one instruction)
#ifdef PF_END_TEST
        if (__builtin_expect(unit == PF_U_END, 0)) break;
#endif
        // Issue the next fetch only after this instruction's words are decoded: scalar
        // loads return out of order, so a fetch issued before the decode would be waited
        // for together with the one being consumed (lgkmcnt(0)).  And after the operand
        // reads (PF_WAIT_LDS): see there.
#ifdef PF_FETCH_EARLY
        __builtin_amdgcn_sched_barrier(0);
        In = fetch_ins(++ip);
#endif
        u256 x, y;
        // register indices are trusted: pf_batch_create checks every read and write
        // against the register file of the kernel that runs the set
        if (NREG == 8) {
            if (__builtin_expect((tr & PF_TR_RA) != 0u, 1)) RDN_SW(x, Wn, a, exp_tbl);
            PF_FWD_A();
            if (__builtin_expect((tr & PF_TR_RB) != 0u, 1)) RDN_SW(y, Wn, b, exp_tbl);
            PF_FWD_B();
        } else {
            if (__builtin_expect((tr & PF_TR_RA) != 0u, 1)) RD_W(x, W, a, LPB);
            PF_FWD_A();
            if (__builtin_expect((tr & PF_TR_RB) != 0u, 1)) RD_W(y, W, b, LPB);
            PF_FWD_B();
        }
        // constant operands (pf_batch_create's peephole deleted their W_CONST): one scalar
        // load of const[a] / const[b] each
        if (__builtin_expect((I.x & (PF_I_KA | PF_I_KB)) != 0u, 0)) {
            if (I.x & PF_I_KA) {
                const uint32_t* cp = S.consts + (size_t)a * 8u;
#pragma unroll
                for (int i = 0; i < 8; i++) x.l[i] = cp[i];
            }
            if (I.x & PF_I_KB) {
                const uint32_t* cp = S.consts + (size_t)b * 8u;
#pragma unroll
                for (int i = 0; i < 8; i++) y.l[i] = cp[i];
            }
        }
#ifndef PF_FETCH_EARLY
        __builtin_amdgcn_sched_barrier(0);
        In = fetch_ins(++ip);
#endif
        // Dispatch on the datapath unit (w0 bits 21..23) first.  The heavy datapaths exist
        // once each (multiplier, divider, shifter, generator) and are shared by every
        // opcode that needs them: the kernel's code must stay small enough for the
        // instruction cache, since consecutive bytecode instructions jump between units.
        switch (unit) {
#ifndef PF_END_TEST
            case PF_U_END:
                goto program_end;
#endif
            case PF_U_MUL:
                // ---- multiplier: MUL = one product; EXP = windowed square-and-multiply over
                // the low 84 exponent bits + the 2-adic closed form for bits 84..253
                // (pf::exp256_split)
                if (op == PF_W_MUL) {
                    z = pf::mul256(x, y);
#ifdef PF_PROBE_2X_MUL
                    {
                        const uint32_t hz = hidden_zero();
                        u256 x2 = x;
                        x2.l[0] ^= hz;
                        const u256 z2 = pf::mul256(x2, y);
                        z.l[7] ^= z2.l[7] & hz;
                    }
#endif
                } else {
#ifdef PF_DIAG_NO_EXP
                    z = pf::add256(x, y);
#else
#ifdef PF_PROFILE_UNITS
                    z = pf::exp256_split(x, y, exp_tbl, 64u, &prof->c[15]);
#else
#ifdef PF_PROBE_2X_EXP
                    {
                        const uint32_t hz = hidden_zero();
                        u256 x2 = x;
                        x2.l[1] ^= hz;
                        const u256 z2 = pf::exp256_split(x2, y, exp_tbl, 64u);
                        z = pf::exp256_split(x, y, exp_tbl, 64u);
                        z.l[7] ^= z2.l[7] & hz;
                    }
#else
                    z = pf::exp256_split(x, y, exp_tbl, 64u);
#endif
#endif
#endif
                    PF_WAIT_ALL();
                }
                break;
            case PF_U_DIV: {
                // ---- divider: bvudiv/bvurem/bvsdiv/bvsrem/bvsmod (SMT-LIB2 definitions on
                // magnitudes) and bvumul_noovfl (a*b < 2^w  <=>  b == 0 || a <= (2^w-1)/b)
                // The signed / overflow pre- and post-processing sit under wave-uniform branches
                // on the opcode: computed for every division and selected away, the
                // negations, the SMOD fix-up and the overflow compare cost ~70 VALU per
                // unsigned division (config 3: 10.7 divisions per set).
                const bool sgn = op >= PF_W_SDIV && op <= PF_W_SMOD;
                u256 ua = x, ub = y;
                uint32_t sa = 0u, sb = 0u;
                if (sgn) {
                    const u256 xs = sextw(x, w), ys = sextw(y, w);
                    sa = xs.l[7] >> 31;
                    sb = ys.l[7] >> 31;
                    ua = pf::sel256(sa, pf::neg256(xs), xs);
                    ub = pf::sel256(sb, pf::neg256(ys), ys);
                } else if (op == PF_B_UMUL_NOOVF) {
                    ua = pf::ones256();
                    maskw(ua, w);
                    // a waits in LDS table entry 1 (free outside EXP) across the division
                    pf::tbl_put(exp_tbl, 64u, 1u, x);
                }
                u256 q, rr;
#ifdef PF_PROFILE_UNITS
                {
                    const uint32_t bz = pf::iszero256(ub);
                    pbucket = !pf::wave_any((bz ^ 1u) & (pf::ult256(ua, ub) ^ 1u)) ? 11u
                            : !pf::wave_any((ub.l[1] | ub.l[2] | ub.l[3] | ub.l[4] | ub.l[5] | ub.l[6] | ub.l[7]) != 0u) ? 12u
                            : !pf::wave_any((bz ^ 1u) & (uint32_t)(pf::clz256(ub) > pf::clz256(ua) + 31u)) ? 13u : 14u;
                }
#endif
#ifdef PF_DIAG_NO_DIV
                q = ua; rr = ub;
#else
                pf::udivrem256(ua, ub, &q, &rr);
#ifdef PF_PROBE_2X_DIV
                {
                    const uint32_t hz = hidden_zero();
                    u256 ua2 = ua, q2, r2;
                    ua2.l[0] ^= hz;
                    pf::udivrem256(ua2, ub, &q2, &r2);
                    q.l[0] ^= q2.l[0] & hz;
                    rr.l[0] ^= r2.l[7] & hz;
                }
#endif
#endif
                // x and y are not read past the division (their registers are free in it):
                // UMUL_NOOVF's a comes back from LDS, SMOD's signed divisor is rebuilt from |b|
                if (op == PF_B_UMUL_NOOVF) {
                    BSET(d, pf::iszero256(ub) | (pf::ult256(q, pf::tbl_get(exp_tbl, 64u, 1u)) ^ 1u));
                    PF_NEXT();
                } else if (!sgn) {
                    z = op == PF_W_UDIV ? q : rr;
                } else if (op == PF_W_SDIV) {
                    z = pf::sel256(sa ^ sb, pf::neg256(q), q);
                } else {
                    z = pf::sel256(sa, pf::neg256(rr), rr);
                    if (op == PF_W_SMOD)  // uniform; the fix-up itself is a per-lane select
                        z = pf::sel256((pf::iszero256(rr) ^ 1u) & (sa ^ sb),
                                       pf::add256(z, pf::sel256(sb, pf::neg256(ub), ub)), z);
                }
                break;
            }
            case PF_U_SHIFT: {
#ifdef PF_DIAG_NO_SHIFT
                z = pf::add256(x, y); break;
#endif
                const bool by_reg = op <= PF_W_ASHR;
                const uint32_t big = by_reg ? ge_width(y, w) : (aux >= 256u);
                const uint32_t amt = by_reg ? y.l[0] : aux;
                if (op == PF_W_SHL || op == PF_W_CONCAT) {
                    z = pf::shl256(x, big ? 0u : amt, big);
                    if (op == PF_W_CONCAT) {
#pragma unroll
                        for (int i = 0; i < 8; i++) z.l[i] |= y.l[i];
                    }
                } else {
                    const bool ar = op == PF_W_ASHR;
                    const u256 src = ar ? sextw(x, w) : x;
                    const uint32_t f = ar ? 0u - (src.l[7] >> 31) : 0u;
                    z = pf::shr256(src, big ? (ar ? 255u : 0u) : (amt & 255u), f);
                    if (!ar) z = pf::sel256(big, pf::zero256(), z);
                }
                break;
            }
            case PF_U_GEN:
                // ---- candidate generator (one site for W and B variables)
                if (MODE == MODE_GEN) {
#ifdef PF_DIAG_NO_GEN
                    z = pf::zero256(); z.l[0] = cand ^ aux;
#else
                    z = gen_var(S, aux, cand);
#ifdef PF_PROBE_2X_GEN
                    {
                        const uint32_t hz = hidden_zero();
                        const u256 z2 = gen_var(S, aux, cand ^ hz);
                        z.l[0] ^= z2.l[0] & (hz - 1u) & hz;
                        z.l[1] ^= z2.l[7] & hz;
                    }
#endif
#endif
                } else {
#pragma unroll
                    for (int i = 0; i < 8; i++)
                        z.l[i] = active ? soa[((size_t)aux * 8u + i) * soa_n + cand] : 0u;
                }
                PF_WAIT_GEN();
                if (op == PF_B_VAR) {
                    BSET(d, z.l[0]);
                    PF_NEXT();
                }
                break;
            case PF_U_CMP: {
                uint32_t bres;
                switch (op) {
                    case PF_B_EQ: bres = pf::eq256(x, y); break;
                    case PF_B_ULT: bres = pf::ult256(x, y); break;
                    case PF_B_ULE: bres = pf::ult256(y, x) ^ 1u; break;
                    case PF_B_SLT:
                    case PF_B_SLE: {
                        u256 sx = sextw(x, w), sy = sextw(y, w);
                        sx.l[7] ^= 0x80000000u;
                        sy.l[7] ^= 0x80000000u;
                        bres = (op == PF_B_SLT) ? pf::ult256(sx, sy) : (pf::ult256(sy, sx) ^ 1u);
                        break;
                    }
                    default: {  // PF_B_UADD_NOOVF
                        uint32_t co;
                        u256 sm = pf::add256c(x, y, &co);
                        u256 s2 = sm;
                        maskw(s2, w);  // no overflow iff the sum fits in w bits
                        bres = (uint32_t)(co == 0u) & pf::eq256(sm, s2);
                        break;
                    }
                }
                BSET(d, bres);
                if (I.x & PF_I_ASSERT) PF_DO_ASSERT(bres);
                PF_NEXT();
            }
            case PF_U_BOOL:
                switch (op) {
                    case PF_B_CONST: BSET(d, aux); break;
                    case PF_B_AND: BSET(d, BGET(a) & BGET(b)); break;
                    case PF_B_OR: BSET(d, BGET(a) | BGET(b)); break;
                    case PF_B_XOR: BSET(d, BGET(a) ^ BGET(b)); break;
                    case PF_B_NOT: BSET(d, BGET(a) ^ 1u); break;
                    case PF_B_ITE: BSET(d, BGET(c) ? BGET(a) : BGET(b)); break;
                    case PF_B_FILL:
                        if (aux & PF_SPILL_LDS) {  // uniform: pf_batch_create's LDS slots
                            BSET(d, exp_tbl[(aux & 3u) * 4u * 64u].x);
                        } else {
                            BSET(d, spill[PF_SLOT(aux) * 8u]);
                        }
                        PF_WAIT_ALL();
                        break;
                    case PF_B_SPILL:
                        if (aux & PF_SPILL_LDS)
                            exp_tbl[(aux & 3u) * 4u * 64u] = make_uint2(BGET(a), 0u);
                        else
                            spill[PF_SLOT(aux) * 8u] = BGET(a);
                        break;
                    default:  // PF_ASSERT
                        PF_DO_ASSERT(BGET(a));
                        PF_NEXT();
                }
                if (I.x & PF_I_ASSERT) PF_DO_ASSERT(BGET(d));
                PF_NEXT();
            default:  // PF_U_ALU
                switch (op) {
                    case PF_W_ADD: z = pf::add256(x, y); break;
                    case PF_W_SUB: z = pf::sub256(x, y); break;
                    case PF_W_AND:
#pragma unroll
                        for (int i = 0; i < 8; i++) z.l[i] = x.l[i] & y.l[i];
                        break;
                    case PF_W_OR:
#pragma unroll
                        for (int i = 0; i < 8; i++) z.l[i] = x.l[i] | y.l[i];
                        break;
                    case PF_W_XOR:
#pragma unroll
                        for (int i = 0; i < 8; i++) z.l[i] = x.l[i] ^ y.l[i];
                        break;
                    case PF_W_CONST: {
                        const uint32_t* cp = S.consts + (size_t)aux * 8u;
#pragma unroll
                        for (int i = 0; i < 8; i++) z.l[i] = cp[i];
                        PF_WAIT_ALL();
                        break;
                    }
                    case PF_W_MOV: z = x; break;
                    case PF_W_SPILL:
                        if (aux & PF_SPILL_LDS) {  // uniform: pf_batch_create's LDS slots
                            pf::tbl_put(exp_tbl, 64u, aux & 3u, x);
                        } else {
#pragma unroll
                            for (int i = 0; i < 8; i++) spill[PF_SLOT(aux) * 8u + i] = x.l[i];
                        }
                        if (NREG == 8) PF_NEXT();  // no W result (the wide kernels write the sink)
                        z = x;
                        break;
                    case PF_W_FILL:
                        if (aux & PF_SPILL_LDS) {
                            z = pf::tbl_get(exp_tbl, 64u, aux & 3u);
                        } else {
#pragma unroll
                            for (int i = 0; i < 8; i++) z.l[i] = spill[PF_SLOT(aux) * 8u + i];
                        }
                        PF_WAIT_ALL();
                        break;
                    case PF_W_NOT: z = pf::not256(x); break;
                    case PF_W_NEG: z = pf::neg256(x); break;
                    case PF_W_SEXT: z = sextw(x, aux); break;
                    case PF_W_ITE: z = pf::sel256(BGET(c), x, y); break;
                    case PF_W_HASH: {
#ifdef PF_DIAG_NO_HASH
                        z = pf::sub256(x, y); break;
#endif
                        uint4 h = philox(make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]), aux, PF_HASH_K1A);
                        uint4 g = philox(make_uint4(x.l[4] ^ h.x, x.l[5] ^ h.y, x.l[6] ^ h.z, x.l[7] ^ h.w),
                                         aux, PF_HASH_K1B);
                        z.l[0] = h.x; z.l[1] = h.y; z.l[2] = h.z; z.l[3] = h.w;
                        z.l[4] = g.x; z.l[5] = g.y; z.l[6] = g.z; z.l[7] = g.w;
                        break;
                    }
                    default: break;
                }
                break;
        }
        {
            // W write-back of every op that reaches here (ops without a W result other than
            // the B ops above — W_SPILL — write the sink register PF_W_SINK)
            maskw(z, w);
            const uint32_t dd = (tr & PF_TR_WW) ? d : (uint32_t)(NREG - 1);
            // keep the 8 indexed moves one s_set_gpr_idx block: the scheduler otherwise
            // interleaves the B update into it and re-enters indexing mode per move
            if (NREG == 8) {
                // only W results reach here (W_SPILL leaves above); PF_TR_WW clear = a result
                // only the next instruction reads (forwarded), no write-back
                if (PF_FWD_WB(tr)) WRN_SW(Wn, d, z, exp_tbl);
            } else {
                __builtin_amdgcn_sched_barrier(0);
                WR_W(W, dd, z, LPB);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#ifdef PF_PROFILE_UNITS
        prof_add(prof, pbucket, __builtin_amdgcn_s_memtime() - t_ins);
#else
        (void)prof;
#endif
    }
#ifndef PF_END_TEST
program_end:
#endif
    *complete = sc ^ 1u;
    *ops += cost;
    return root;
#undef PF_FWD_A
#undef PF_FWD_B
#undef PF_FWD_WB
#undef BGET
}

PF_INL SetCtx make_ctx(const pf_set_desc* __restrict__ descs, uint32_t set,
                       const uint4* __restrict__ code, const uint32_t* __restrict__ consts,
                       const uint4* __restrict__ schema, const uint32_t* __restrict__ parents,
                       uint64_t gseed) {
    pf_set_desc D = descs[set];
    SetCtx S;
    S.code = code + D.code_off;
    S.consts = consts + (size_t)D.const_off * 8u;
    S.schema = schema + D.var_off;
    S.parents = parents;
    S.n_ins = D.n_ins;
    S.n_const = D.n_const;
    S.n_vars = D.n_vars;
    S.seed = D.seed;
    S.k0 = (uint32_t)gseed ^ D.seed;
    S.k1 = (uint32_t)(gseed >> 32);
    S.nc_rcp = __builtin_amdgcn_readfirstlane(D.n_const ? urcp32(D.n_const) : 0u);  // set is uniform
    return S;
}

}  // namespace

// candidates [begin, end) of one set: 64-candidate groups, ballot, smallest witness by
// atomicMin; with EARLY the walk stops at the first witness or once a witness below the
// next group exists
template <bool EARLY, int NREG>
PF_INL void search_item(const SetCtx& S, uint32_t set, uint32_t begin, uint32_t end, uint32_t flags,
                        uint64_t deadline_ticks, uint64_t t0, uint32_t* __restrict__ found,
                        uint2* exp_tbl, uint64_t& evals_full, uint64_t& decided, uint64_t& ops,
                        uint32_t& cut, UnitProf& prof) {
    const uint32_t lane = threadIdx.x & 63u;
    // the item's groups run in increasing candidate order, so its first witness is its
    // smallest: one found[] atomic per item.  (Device-scope atomics are performed beyond the
    // per-XCD L2s, so each is an HBM-side write request: one per witnessed group made the
    // round-2 full sweep's 30 MB of WRITE_SIZE per launch.)
    bool posted = false;
    for (uint32_t base = begin; base < end; base += 64u) {
        if (EARLY) {
            uint32_t f = __hip_atomic_load(found + set, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane(f) <= base) break;
        }
        if (deadline_ticks) {
            uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (now - t0 > deadline_ticks) {
                cut = 1u;  // this item is not fully searched: no complete verdict
                break;
            }
        }
        const uint32_t cand = base + lane;
        const bool active = cand < end;
        uint32_t complete = 0;
        uint64_t lane_ops = 0;
        uint32_t sat = run_program<MODE_GEN, NREG>(S, cand, active, flags, nullptr, 0u, exp_tbl, &complete,
                                             &lane_ops, &prof);
        const uint64_t m_act = __ballot(active);
        const uint64_t m_sat = __ballot((uint32_t)active & sat);
        const uint64_t m_full = __ballot((uint32_t)active & complete);
        decided += __popcll(m_act);
        evals_full += __popcll(m_full);
        ops += lane_ops * (uint64_t)__popcll(m_act);
#ifdef PF_DIAG_ALL_ATOMICS  // timing probe only: one found[] atomic per witnessed group
        posted = false;
#endif
        if (m_sat && !posted) {
            uint32_t first = base + (uint32_t)__builtin_ctzll(m_sat);
            if (lane == 0) atomicMin(found + set, first);
            posted = true;
            if (EARLY) break;
        }
    }
}

// PF_FULL_QUEUE (default 1): the full sweep also runs as the persistent work queue (items
// set-major, sets longest first; +2 % on config 3 against one wave per item, which
// PF_FULL_QUEUE=0 restores)
#ifndef PF_FULL_QUEUE
#define PF_FULL_QUEUE 1
#endif
// ---- search kernel: generate + evaluate + ballot early exit ---------------------------
// grid: one wave per (set, slice); a slice is `per_wave` consecutive candidates.
// Two entry points over one body: the full sweep (pf_check_kernel) and the production
// early-exit search (pf_check_early_kernel).  EARLY is a template constant so the full sweep
// carries no found[] polling, and the two launches are separate rows in a rocprof trace.
template <bool EARLY, int NREG>
PF_INL void check_body(const pf_set_desc* __restrict__ descs, const uint32_t* __restrict__ order,
                       uint32_t n_sets,
                       const uint4* __restrict__ code, const uint32_t* __restrict__ consts,
                       const uint4* __restrict__ schema, const uint32_t* __restrict__ parents,
                       uint64_t gseed, uint32_t budget, uint32_t per_wave, uint32_t slices,
                       uint32_t flags, uint64_t deadline_ticks, uint64_t* __restrict__ t0_slot,
                       uint32_t* __restrict__ found, unsigned long long* __restrict__ counters,
                       uint32_t* __restrict__ queue, uint32_t cand_begin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t n_items = n_sets * slices;
    if (!EARLY && !PF_FULL_QUEUE && wave >= n_items) return;
    __shared__ uint2 pf_exp_lds[PF_SEARCH_LDS_U2];
    uint2* exp_tbl = exp_tbl_of(pf_exp_lds);

    uint64_t t0 = 0;
    if (deadline_ticks) {
        // the first wave stamps the launch's start; later waves only read it (a CAS from
        // every one of ~10^5 waves on one address serialises in L2: ~100 ms per launch)
        uint64_t now = __builtin_amdgcn_s_memrealtime();
        uint64_t prev = __hip_atomic_load(t0_slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == 0) prev = atomicCAS((unsigned long long*)t0_slot, 0ull, (unsigned long long)now);
        // wave-uniform (both halves read from lane 0): the deadline exit stays a scalar branch
        const uint64_t t = prev ? prev : now;
        // (readfirstlane returns int: go through uint32_t, or the low half sign-extends)
        t0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)t) |
             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(t >> 32)) << 32);
    }
    UnitProf prof;
#pragma unroll
    for (int i = 0; i < PF_PROF_BUCKETS; i++) prof.c[i] = 0;
#ifdef PF_PROFILE_UNITS
    const uint64_t t_wave = __builtin_amdgcn_s_memtime();
#endif
    uint64_t evals_full = 0, decided = 0, ops = 0;
    uint32_t cut = 0u;
    // Full sweep: one wave per (set, slice), set-major (a set's slices side by side, sets
    // longest first).  Early exit: a work queue of (set, chunk) items in chunk-major order —
    // chunk 0 of every set first, then chunk 1, ... — taken one at a time by a chip-filling
    // grid of waves.  A witness found in a low chunk makes the set's later chunks cost one
    // found[] read each, instead of every concurrently launched slice of the set evaluating
    // at least one group, and no wave idles while items remain (dynamic balance).  The
    // smallest-witness result does not depend on the order: a chunk stops only once a witness
    // below its own range exists.  Every wave leaves the loop: the queue head only grows.
    if (!EARLY && !PF_FULL_QUEUE) {
        const uint32_t set = __builtin_amdgcn_readfirstlane(order[wave / slices]);
        const uint32_t slice = wave % slices;
        search_item<EARLY, NREG>(make_ctx(descs, set, code, consts, schema, parents, gseed), set,
                                 cand_begin + slice * per_wave, min(budget, cand_begin + slice * per_wave + per_wave), flags,
                                 deadline_ticks, t0, found, exp_tbl, evals_full, decided, ops, cut, prof);
    } else {
        // PF_EARLY_QUEUES heads, 128 B apart: queue q hands out items q, q + Q, q + 2Q, ...
        // (so the claims stay close to chunk-major order overall); a wave starts at queue
        // wave % Q and moves on to the next queue when one runs dry.  One head serialised the
        // claims at ~14 ns each in L2 — the whole cost of a planted batch, whose items after
        // the first chunk are all skips.  Each inner loop ends because its head only grows.
        for (uint32_t qi = 0; qi < PF_EARLY_QUEUES; ++qi) {
            const uint32_t q = (wave + qi) % PF_EARLY_QUEUES;
            const uint32_t nq = n_items > q ? (n_items - q + PF_EARLY_QUEUES - 1u) / PF_EARLY_QUEUES : 0u;
#ifndef PF_QUEUE_NO_PEEK
            // another wave's queue is read before it is claimed from: once the items run out,
            // every wave passes every queue on its way out, and as atomics those probes
            // serialise on the 16 heads (~14 ns each: ~60 us for a 4,096-wave grid, the
            // larger part of a small batch's search); a plain load of a drained head does not
            if (qi > 0u) {
                uint32_t h = 0u;
                if (lane == 0u) h = __hip_atomic_load(queue + q * PF_EARLY_QUEUE_STRIDE, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                if (__builtin_amdgcn_readfirstlane(h) >= nq) continue;
            }
#endif
            for (;;) {
                uint32_t v = 0u;
                if (lane == 0u) v = atomicAdd(queue + q * PF_EARLY_QUEUE_STRIDE, 1u);
                const uint32_t k = __builtin_amdgcn_readfirstlane(v);
                if (k >= nq) break;
                const uint32_t item = k * PF_EARLY_QUEUES + q;
                // early exit: chunk-major; full sweep: set-major, sets longest first
                const uint32_t set = __builtin_amdgcn_readfirstlane(order[EARLY ? item % n_sets : item / slices]);
                const uint32_t slice = EARLY ? item / n_sets : item % slices;
                search_item<EARLY, NREG>(make_ctx(descs, set, code, consts, schema, parents, gseed), set,
                                         cand_begin + slice * per_wave, min(budget, cand_begin + slice * per_wave + per_wave), flags,
                                         deadline_ticks, t0, found, exp_tbl, evals_full, decided, ops, cut, prof);
                if (cut) break;
            }
            if (cut) break;
        }
    }
    if (lane == 0) {
        unsigned long long* cs = counters + PF_COUNTER_OFF / 8 + (wave % PF_COUNTER_STRIPES) * 16u;
        if (evals_full) atomicAdd(cs + 0, (unsigned long long)evals_full);
        if (decided) atomicAdd(cs + 1, (unsigned long long)decided);
        if ((flags & PF_FLAG_COUNT_OPS) && ops) atomicAdd(cs + 2, (unsigned long long)ops);
        if (cut) atomicAdd(cs + 3, 1ull);
#ifdef PF_PROFILE_UNITS
#pragma unroll
        for (int i = 0; i < PF_PROF_BUCKETS; i++)
            atomicAdd(counters + PF_PROF_SLOT + i, (unsigned long long)prof.c[i]);
        atomicAdd(counters + PF_PROF_SLOT + PF_PROF_BUCKETS,
                  (unsigned long long)(__builtin_amdgcn_s_memtime() - t_wave));
#endif
    }
}

#define PF_CHECK_PARAMS                                                                      \
    const pf_set_desc *__restrict__ descs, const uint32_t *__restrict__ order, uint32_t n_sets, \
        const uint4 *__restrict__ code, const uint32_t *__restrict__ consts,                   \
        const uint4 *__restrict__ schema, const uint32_t *__restrict__ parents, uint64_t gseed, \
        uint32_t budget, uint32_t per_wave, uint32_t slices, uint32_t flags,                   \
        uint64_t deadline_ticks, uint64_t *__restrict__ t0_slot, uint32_t *__restrict__ found, \
        unsigned long long *__restrict__ counters, uint32_t *__restrict__ queue, uint32_t cand_begin
#define PF_CHECK_ARGS                                                                         \
    descs, order, n_sets, code, consts, schema, parents, gseed, budget, per_wave, slices, flags, \
        deadline_ticks, t0_slot, found, counters, queue, cand_begin

// The search kernels exist twice: over 8 registers at 3 waves per SIMD (programs whose
// lowering fits PF_NW_NARROW registers — the host picks per batch, pathfeas.hip) and over 16
// at 2 waves.  Occupancy is the lever: config 3 runs +22 % faster on the 8-register build
// (DESIGN.md §3), the interpreter's scalar dispatch and memory latency being what a third
// wave hides.
// Per-search reset of a batch: the scratch words (t0, queue heads, counter lines) to 0 and
// the verdicts to "none" (0xFFFFFFFF) — one launch where two runtime fills were two enqueues
extern "C" __global__ void __launch_bounds__(256) pf_reset_kernel(uint32_t* __restrict__ scratch, uint32_t n_scratch,
                                                                  uint32_t* __restrict__ found, uint32_t n_found) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_scratch + n_found; i += stride) {
        if (i < n_scratch)
            scratch[i] = 0u;
        else
            found[i - n_scratch] = 0xFFFFFFFFu;
    }
}

extern "C" __global__ void __launch_bounds__(64 * PF_SEARCH_WG_WAVES, PF_WG_PER_CU_NARROW) pf_check_kernel(PF_CHECK_PARAMS) {
    check_body<false, PF_NW_NARROW + 1>(PF_CHECK_ARGS);
}
extern "C" __global__ void __launch_bounds__(64 * PF_SEARCH_WG_WAVES, PF_WG_PER_CU_NARROW) pf_check_early_kernel(PF_CHECK_PARAMS) {
    check_body<true, PF_NW_NARROW + 1>(PF_CHECK_ARGS);
}
extern "C" __global__ void __launch_bounds__(64 * PF_SEARCH_WG_WAVES, PF_WG_PER_CU) pf_check_r16_kernel(PF_CHECK_PARAMS) {
    check_body<false, 16>(PF_CHECK_ARGS);
}
extern "C" __global__ void __launch_bounds__(64 * PF_SEARCH_WG_WAVES, PF_WG_PER_CU) pf_check_early_r16_kernel(PF_CHECK_PARAMS) {
    check_body<true, 16>(PF_CHECK_ARGS);
}

// ---- explicit-assignment evaluation (SoA [var][limb][cand]) --------------------------
extern "C" __global__ void __launch_bounds__(256, PF_WG_PER_CU)
pf_eval_soa_kernel(const pf_set_desc* __restrict__ descs, uint32_t set,
                   const uint4* __restrict__ code, const uint32_t* __restrict__ consts,
                   const uint4* __restrict__ schema, const uint32_t* __restrict__ parents,
                   const uint32_t* __restrict__ soa, uint32_t n_cand, uint8_t* __restrict__ out) {
    const uint32_t cand = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = cand < n_cand;
    const SetCtx S = make_ctx(descs, __builtin_amdgcn_readfirstlane(set), code, consts, schema, parents, 0ull);
    __shared__ uint2 pf_exp_lds[PF_EXP_LDS_U2];
    uint32_t complete = 0;
    uint64_t ops = 0;
    UnitProf prof;
    uint32_t sat = run_program<MODE_SOA, 16>(S, active ? cand : 0u, active, 0u, soa, n_cand,
                                         exp_tbl_of(pf_exp_lds), &complete, &ops, &prof);
    if (active) out[cand] = (uint8_t)sat;
}

// ---- several programs over one set of explicit assignments ----------------------------
// grid (ceil(n_cand / 64), n_sets), one wave per block: block (x, s) runs set s's program on
// candidates 64x .. 64x + 63, its variables at rows descs[s].var_off.. of the SoA; verdicts
// out[s * n_cand + cand].  The GPU-resident ModelCache splits a query's conjuncts into groups
// lowered as separate sets, so the groups run side by side instead of one lone wave walking
// the whole conjunction (mythril_amd/model_cache.py).
extern "C" __global__ void __launch_bounds__(64)
pf_eval_soa_sets_kernel(const pf_set_desc* __restrict__ descs, const uint4* __restrict__ code,
                        const uint32_t* __restrict__ consts, const uint4* __restrict__ schema,
                        const uint32_t* __restrict__ soa, uint32_t n_cand, uint8_t* __restrict__ out) {
    const uint32_t set = blockIdx.y;
    const uint32_t cand = blockIdx.x * 64u + threadIdx.x;
    const bool active = cand < n_cand;
    const SetCtx S = make_ctx(descs, set, code, consts, schema, nullptr, 0ull);
    const uint32_t* soa_s = soa + (size_t)__builtin_amdgcn_readfirstlane(descs[set].var_off) * 8u * n_cand;
    __shared__ uint2 pf_exp_lds[PF_LDS_ENTRIES * 4 * 64];
    uint32_t complete = 0;
    uint64_t ops = 0;
    UnitProf prof;
    uint32_t sat = run_program<MODE_SOA, 16>(S, active ? cand : 0u, active, 0u, soa_s, n_cand,
                                         exp_tbl_of(pf_exp_lds), &complete, &ops, &prof);
    if (active) out[(size_t)set * n_cand + cand] = (uint8_t)sat;
}

// ---- materialise witness assignments --------------------------------------------------
// one thread per (request, variable); out offset per request given by req_off (in vars)
extern "C" __global__ void __launch_bounds__(256)
pf_materialize_kernel(const pf_set_desc* __restrict__ descs, const uint4* __restrict__ code,
                      const uint32_t* __restrict__ consts, const uint4* __restrict__ schema,
                      const uint32_t* __restrict__ parents, uint64_t gseed,
                      const uint32_t* __restrict__ set_ids, const uint32_t* __restrict__ cand_ids,
                      const uint32_t* __restrict__ req_off, uint32_t n_req, uint32_t max_vars,
                      uint32_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t req = t / max_vars, v = t % max_vars;
    if (req >= n_req) return;
    const uint32_t set = set_ids[req];
    pf_set_desc D = descs[set];
    if (v >= D.n_vars) return;
    SetCtx S;
    S.code = code + D.code_off;
    S.consts = consts + (size_t)D.const_off * 8u;
    S.schema = schema + D.var_off;
    S.parents = parents;
    S.n_ins = D.n_ins;
    S.n_const = D.n_const;
    S.n_vars = D.n_vars;
    S.seed = D.seed;
    S.k0 = (uint32_t)gseed ^ D.seed;
    S.k1 = (uint32_t)(gseed >> 32);
    S.nc_rcp = D.n_const ? urcp32(D.n_const) : 0u;
    u256 x = gen_var(S, v, cand_ids[req]);
    uint32_t* o = out + ((size_t)req_off[req] + v) * 8u;
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = x.l[i];
}
