// Micro-benchmark (diagnostic): issue cost on gfx950 of the data-movement and arithmetic
// instructions the interpreter spends its non-algorithmic VALU cycles on — 32- vs 64-bit
// register copies (operand reads / write-backs), per-limb selects, 32-bit multiplies (the
// EXP Horner chain's Hensel divisions) and the f64 ops of the division estimates.
// Each lane runs `iters` rounds of 16 independent instructions (inline asm, so the compiler
// cannot fold or reorder them); grid = 4 waves per SIMD, the search kernels' occupancy.
// Prints SIMD cycles per wave-instruction: latency-limited rates at the given occupancy (16
// independent instructions per wave), not throughput — the VALU issues a wave64 instruction
// every 2 cycles at best (MI355X_MICROARCH.md).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

#define R16(T, init)                                                                          \
    T a0 = init + 0, a1 = init + 1, a2 = init + 2, a3 = init + 3, a4 = init + 4, a5 = init + 5, \
      a6 = init + 6, a7 = init + 7, b0 = init + 8, b1 = init + 9, b2 = init + 10, b3 = init + 11, \
      b4 = init + 12, b5 = init + 13, b6 = init + 14, b7 = init + 15
#define SINK16 (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7)
// 16 instructions: a_i <- op(b_i), then b_i <- op(a_i)
#define BODY(OP)                                                                               \
    asm volatile(OP " %0, %8\n\t" OP " %1, %9\n\t" OP " %2, %10\n\t" OP " %3, %11\n\t"         \
                 OP " %4, %12\n\t" OP " %5, %13\n\t" OP " %6, %14\n\t" OP " %7, %15"           \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));     \
    asm volatile(OP " %0, %8\n\t" OP " %1, %9\n\t" OP " %2, %10\n\t" OP " %3, %11\n\t"         \
                 OP " %4, %12\n\t" OP " %5, %13\n\t" OP " %6, %14\n\t" OP " %7, %15"           \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7))

#define KERN(NAME, T, OP)                                                                      \
    extern "C" __global__ void __launch_bounds__(256) NAME(uint32_t iters, uint64_t* out) {     \
        R16(T, (T)threadIdx.x);                                                                \
        for (uint32_t i = 0; i < iters; i++) { BODY(OP); }                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;                                   \
    }

KERN(k_mov32, uint32_t, "v_mov_b32")
KERN(k_mov64, uint64_t, "v_mov_b64")
KERN(k_not32, uint32_t, "v_not_b32")
KERN(k_rcp64, double, "v_rcp_f64")

// two-source forms: a_i <- op(b_i, b_i)
#define BODY2(OP)                                                                              \
    asm volatile(OP " %0, %8, %8\n\t" OP " %1, %9, %9\n\t" OP " %2, %10, %10\n\t" OP " %3, %11, %11\n\t" \
                 OP " %4, %12, %12\n\t" OP " %5, %13, %13\n\t" OP " %6, %14, %14\n\t" OP " %7, %15, %15" \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));     \
    asm volatile(OP " %0, %8, %8\n\t" OP " %1, %9, %9\n\t" OP " %2, %10, %10\n\t" OP " %3, %11, %11\n\t" \
                 OP " %4, %12, %12\n\t" OP " %5, %13, %13\n\t" OP " %6, %14, %14\n\t" OP " %7, %15, %15" \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7))
#define KERN2(NAME, T, OP)                                                                     \
    extern "C" __global__ void __launch_bounds__(256) NAME(uint32_t iters, uint64_t* out) {     \
        R16(T, (T)threadIdx.x);                                                                \
        for (uint32_t i = 0; i < iters; i++) { BODY2(OP); }                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;                                   \
    }
KERN2(k_add32, uint32_t, "v_add_u32")
KERN2(k_mullo, uint32_t, "v_mul_lo_u32")
KERN2(k_mulhi, uint32_t, "v_mul_hi_u32")
KERN2(k_pkmov, uint64_t, "v_pk_mov_b32")
KERN2(k_fma64m, double, "v_mul_f64")

// three-source forms: a_i <- op(b_i, b_i, b_i) (FMA-shaped)
#define BODY3(OP)                                                                              \
    asm volatile(OP " %0, %8, %8, %8\n\t" OP " %1, %9, %9, %9\n\t" OP " %2, %10, %10, %10\n\t" OP " %3, %11, %11, %11\n\t" \
                 OP " %4, %12, %12, %12\n\t" OP " %5, %13, %13, %13\n\t" OP " %6, %14, %14, %14\n\t" OP " %7, %15, %15, %15" \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));     \
    asm volatile(OP " %0, %8, %8, %8\n\t" OP " %1, %9, %9, %9\n\t" OP " %2, %10, %10, %10\n\t" OP " %3, %11, %11, %11\n\t" \
                 OP " %4, %12, %12, %12\n\t" OP " %5, %13, %13, %13\n\t" OP " %6, %14, %14, %14\n\t" OP " %7, %15, %15, %15" \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7))
#define KERN3(NAME, T, OP)                                                                     \
    extern "C" __global__ void __launch_bounds__(256) NAME(uint32_t iters, uint64_t* out) {     \
        R16(T, (T)threadIdx.x);                                                                \
        for (uint32_t i = 0; i < iters; i++) { BODY3(OP); }                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;                                   \
    }
// three sources in three different registers (the operand banks differ)
#define BODY3D(OP)                                                                             \
    asm volatile(OP " %0, %8, %9, %10\n\t" OP " %1, %9, %10, %11\n\t" OP " %2, %10, %11, %12\n\t" OP " %3, %11, %12, %13\n\t" \
                 OP " %4, %12, %13, %14\n\t" OP " %5, %13, %14, %15\n\t" OP " %6, %14, %15, %8\n\t" OP " %7, %15, %8, %9" \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));     \
    asm volatile(OP " %0, %8, %9, %10\n\t" OP " %1, %9, %10, %11\n\t" OP " %2, %10, %11, %12\n\t" OP " %3, %11, %12, %13\n\t" \
                 OP " %4, %12, %13, %14\n\t" OP " %5, %13, %14, %15\n\t" OP " %6, %14, %15, %8\n\t" OP " %7, %15, %8, %9" \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7))
#define KERN3D(NAME, T, OP)                                                                    \
    extern "C" __global__ void __launch_bounds__(256) NAME(uint32_t iters, uint64_t* out) {     \
        R16(T, (T)threadIdx.x);                                                                \
        for (uint32_t i = 0; i < iters; i++) { BODY3D(OP); }                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;                                   \
    }
KERN3D(k_bfi_d, uint32_t, "v_bfi_b32")
KERN3D(k_add3_d, uint32_t, "v_add3_u32")
KERN3D(k_fma_d, float, "v_fma_f32")
// a per-lane select from a lane mask in VCC (v_cndmask_b32 e32), the alternative to v_bfi
#define BODYC                                                                                  \
    asm volatile("v_cndmask_b32 %0, %8, %9, vcc\n\tv_cndmask_b32 %1, %9, %10, vcc\n\tv_cndmask_b32 %2, %10, %11, vcc\n\t" \
                 "v_cndmask_b32 %3, %11, %12, vcc\n\tv_cndmask_b32 %4, %12, %13, vcc\n\tv_cndmask_b32 %5, %13, %14, vcc\n\t" \
                 "v_cndmask_b32 %6, %14, %15, vcc\n\tv_cndmask_b32 %7, %15, %8, vcc"          \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));     \
    asm volatile("v_cndmask_b32 %0, %8, %9, vcc\n\tv_cndmask_b32 %1, %9, %10, vcc\n\tv_cndmask_b32 %2, %10, %11, vcc\n\t" \
                 "v_cndmask_b32 %3, %11, %12, vcc\n\tv_cndmask_b32 %4, %12, %13, vcc\n\tv_cndmask_b32 %5, %13, %14, vcc\n\t" \
                 "v_cndmask_b32 %6, %14, %15, vcc\n\tv_cndmask_b32 %7, %15, %8, vcc"          \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7))
#define BODYCS                                                                                 \
    asm volatile("v_cndmask_b32_e64 %0, %8, %9, %16\n\tv_cndmask_b32_e64 %1, %9, %10, %16\n\tv_cndmask_b32_e64 %2, %10, %11, %16\n\t" \
                 "v_cndmask_b32_e64 %3, %11, %12, %16\n\tv_cndmask_b32_e64 %4, %12, %13, %16\n\tv_cndmask_b32_e64 %5, %13, %14, %16\n\t" \
                 "v_cndmask_b32_e64 %6, %14, %15, %16\n\tv_cndmask_b32_e64 %7, %15, %8, %16"  \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %8, %9, %16\n\tv_cndmask_b32_e64 %1, %9, %10, %16\n\tv_cndmask_b32_e64 %2, %10, %11, %16\n\t" \
                 "v_cndmask_b32_e64 %3, %11, %12, %16\n\tv_cndmask_b32_e64 %4, %12, %13, %16\n\tv_cndmask_b32_e64 %5, %13, %14, %16\n\t" \
                 "v_cndmask_b32_e64 %6, %14, %15, %16\n\tv_cndmask_b32_e64 %7, %15, %8, %16"  \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7), "s"(msk))
// the mask in an SGPR pair written by the scalar unit (a uniform select)
extern "C" __global__ void __launch_bounds__(256) k_cndmask_s(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    const uint64_t msk = __builtin_amdgcn_readfirstlane(iters) & 1u ? ~0ull : 0ull;
    for (uint32_t i = 0; i < iters; i++) { BODYCS; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
// VOP3 encoding, mask = VCC
extern "C" __global__ void __launch_bounds__(256) k_cndmask_e64vcc(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    asm volatile("v_cmp_ne_u32 vcc, 0, %0" :: "v"(threadIdx.x & 1u) : "vcc");
    for (uint32_t i = 0; i < iters; i++) {
        asm volatile("v_cndmask_b32_e64 %0, %8, %9, vcc\n\tv_cndmask_b32_e64 %1, %9, %10, vcc\n\tv_cndmask_b32_e64 %2, %10, %11, vcc\n\t"
                     "v_cndmask_b32_e64 %3, %11, %12, vcc\n\tv_cndmask_b32_e64 %4, %12, %13, vcc\n\tv_cndmask_b32_e64 %5, %13, %14, vcc\n\t"
                     "v_cndmask_b32_e64 %6, %14, %15, vcc\n\tv_cndmask_b32_e64 %7, %15, %8, vcc"
                     : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
                     : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));
        asm volatile("v_cndmask_b32_e64 %0, %8, %9, vcc\n\tv_cndmask_b32_e64 %1, %9, %10, vcc\n\tv_cndmask_b32_e64 %2, %10, %11, vcc\n\t"
                     "v_cndmask_b32_e64 %3, %11, %12, vcc\n\tv_cndmask_b32_e64 %4, %12, %13, vcc\n\tv_cndmask_b32_e64 %5, %13, %14, vcc\n\t"
                     "v_cndmask_b32_e64 %6, %14, %15, vcc\n\tv_cndmask_b32_e64 %7, %15, %8, vcc"
                     : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7)
                     : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
// VOP2 with VCC written by the scalar unit each iteration (the compiler's uniform selects:
// s_cselect_b64 vcc, -1, 0 then v_cndmask_b32_e32 ... vcc)
extern "C" __global__ void __launch_bounds__(256) k_cndmask_svcc(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    for (uint32_t i = 0; i < iters; i++) {
        asm volatile("s_cmp_eq_u32 %0, 0\n\ts_cselect_b64 vcc, -1, 0" :: "s"(i & 1u) : "vcc", "scc");
        BODYC;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
// 256-bit add carry chains as the compiler emits them (VOP2, carry through VCC) and as VOP3
// with the carry in an SGPR pair: a <- a + b, 8 limbs, one chain per iteration
extern "C" __global__ void __launch_bounds__(256) k_add256_e32(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    for (uint32_t i = 0; i < iters; i++) {
        asm volatile("v_add_co_u32_e32 %0, vcc, %0, %8\n\tv_addc_co_u32_e32 %1, vcc, %1, %9, vcc\n\t"
                     "v_addc_co_u32_e32 %2, vcc, %2, %10, vcc\n\tv_addc_co_u32_e32 %3, vcc, %3, %11, vcc\n\t"
                     "v_addc_co_u32_e32 %4, vcc, %4, %12, vcc\n\tv_addc_co_u32_e32 %5, vcc, %5, %13, vcc\n\t"
                     "v_addc_co_u32_e32 %6, vcc, %6, %14, vcc\n\tv_addc_co_u32_e32 %7, vcc, %7, %15, vcc"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7) : "vcc");
        asm volatile("v_add_co_u32_e32 %0, vcc, %0, %8\n\tv_addc_co_u32_e32 %1, vcc, %1, %9, vcc\n\t"
                     "v_addc_co_u32_e32 %2, vcc, %2, %10, vcc\n\tv_addc_co_u32_e32 %3, vcc, %3, %11, vcc\n\t"
                     "v_addc_co_u32_e32 %4, vcc, %4, %12, vcc\n\tv_addc_co_u32_e32 %5, vcc, %5, %13, vcc\n\t"
                     "v_addc_co_u32_e32 %6, vcc, %6, %14, vcc\n\tv_addc_co_u32_e32 %7, vcc, %7, %15, vcc"
                     : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                     : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
extern "C" __global__ void __launch_bounds__(256) k_add256_e64(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    for (uint32_t i = 0; i < iters; i++) {
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_addc_co_u32_e64 %1, s[42:43], %1, %9, s[40:41]\n\t"
                     "v_addc_co_u32_e64 %2, s[40:41], %2, %10, s[42:43]\n\tv_addc_co_u32_e64 %3, s[42:43], %3, %11, s[40:41]\n\t"
                     "v_addc_co_u32_e64 %4, s[40:41], %4, %12, s[42:43]\n\tv_addc_co_u32_e64 %5, s[42:43], %5, %13, s[40:41]\n\t"
                     "v_addc_co_u32_e64 %6, s[40:41], %6, %14, s[42:43]\n\tv_addc_co_u32_e64 %7, s[42:43], %7, %15, s[40:41]"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7) : "s40", "s41", "s42", "s43");
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_addc_co_u32_e64 %1, s[42:43], %1, %9, s[40:41]\n\t"
                     "v_addc_co_u32_e64 %2, s[40:41], %2, %10, s[42:43]\n\tv_addc_co_u32_e64 %3, s[42:43], %3, %11, s[40:41]\n\t"
                     "v_addc_co_u32_e64 %4, s[40:41], %4, %12, s[42:43]\n\tv_addc_co_u32_e64 %5, s[42:43], %5, %13, s[40:41]\n\t"
                     "v_addc_co_u32_e64 %6, s[40:41], %6, %14, s[42:43]\n\tv_addc_co_u32_e64 %7, s[42:43], %7, %15, s[40:41]"
                     : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                     : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7) : "s40", "s41", "s42", "s43");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
extern "C" __global__ void __launch_bounds__(256) k_cndmask(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    asm volatile("v_cmp_ne_u32 vcc, 0, %0" :: "v"(threadIdx.x & 1u) : "vcc");
    for (uint32_t i = 0; i < iters; i++) { BODYC; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
// v_mad_u64_u32 (the products' instruction): a_i <- x * y + b_i (64-bit accumulators), carry
// into VCC
#define MADS(D, S)                                                                             \
    asm volatile("v_mad_u64_u32 %0, vcc, %16, %17, %8\n\tv_mad_u64_u32 %1, vcc, %16, %17, %9\n\t"    \
                 "v_mad_u64_u32 %2, vcc, %16, %17, %10\n\tv_mad_u64_u32 %3, vcc, %16, %17, %11\n\t"  \
                 "v_mad_u64_u32 %4, vcc, %16, %17, %12\n\tv_mad_u64_u32 %5, vcc, %16, %17, %13\n\t"  \
                 "v_mad_u64_u32 %6, vcc, %16, %17, %14\n\tv_mad_u64_u32 %7, vcc, %16, %17, %15"        \
                 : "=v"(D##0), "=v"(D##1), "=v"(D##2), "=v"(D##3), "=v"(D##4), "=v"(D##5), "=v"(D##6), "=v"(D##7) \
                 : "v"(S##0), "v"(S##1), "v"(S##2), "v"(S##3), "v"(S##4), "v"(S##5), "v"(S##6), "v"(S##7), \
                   "v"(x), "v"(y) : "vcc")
extern "C" __global__ void __launch_bounds__(256) k_mad64(uint32_t iters, uint64_t* out) {
    R16(uint64_t, (uint64_t)threadIdx.x);
    const uint32_t x = threadIdx.x * 3u + 1u, y = threadIdx.x ^ 0x9E3779B9u;
    for (uint32_t i = 0; i < iters; i++) { MADS(a, b); MADS(b, a); }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
KERN3(k_fmaf32, float, "v_fma_f32")
KERN3(k_bfi, uint32_t, "v_bfi_b32")
KERN3(k_alignbit, uint32_t, "v_alignbit_b32")
KERN3(k_add3, uint32_t, "v_add3_u32")
KERN2(k_addf32, float, "v_add_f32")
// v_bitop3_b32 carries an 8-bit truth table (0x96 = a ^ b ^ c, the Keccak/Philox xor3)
#define BODY3B                                                                                 \
    asm volatile("v_bitop3_b32 %0, %8, %9, %10 bitop3:0x96\n\tv_bitop3_b32 %1, %9, %10, %11 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %2, %10, %11, %12 bitop3:0x96\n\tv_bitop3_b32 %3, %11, %12, %13 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %4, %12, %13, %14 bitop3:0x96\n\tv_bitop3_b32 %5, %13, %14, %15 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %6, %14, %15, %8 bitop3:0x96\n\tv_bitop3_b32 %7, %15, %8, %9 bitop3:0x96"       \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) \
                 : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));     \
    asm volatile("v_bitop3_b32 %0, %8, %9, %10 bitop3:0x96\n\tv_bitop3_b32 %1, %9, %10, %11 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %2, %10, %11, %12 bitop3:0x96\n\tv_bitop3_b32 %3, %11, %12, %13 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %4, %12, %13, %14 bitop3:0x96\n\tv_bitop3_b32 %5, %13, %14, %15 bitop3:0x96\n\t" \
                 "v_bitop3_b32 %6, %14, %15, %8 bitop3:0x96\n\tv_bitop3_b32 %7, %15, %8, %9 bitop3:0x96"       \
                 : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) \
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7))
extern "C" __global__ void __launch_bounds__(256) k_bitop3_d(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    for (uint32_t i = 0; i < iters; i++) { BODY3B; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
}
KERN3D(k_alignbit_d, uint32_t, "v_alignbit_b32")
KERN2(k_xor, uint32_t, "v_xor_b32")
// carry-out forms (the 256-bit add chain's instructions), carry into VCC

// the shader clock during an add loop: s_memtime (shader cycles) over s_memrealtime (100 MHz)
extern "C" __global__ void __launch_bounds__(256) k_clock(uint32_t iters, uint64_t* out) {
    R16(uint32_t, (uint32_t)threadIdx.x);
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = 0; i < iters; i++) { BODY2("v_add_u32"); }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK16;
    if (blockIdx.x == 0 && threadIdx.x == 0) { out[0] = c1 - c0; out[1] = r1 - r0; }
}

typedef void (*kfn)(uint32_t, uint64_t*);
int main(int argc, char** argv) {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // waves per SIMD (argument, default 4: the search kernels' occupancy); 256-thread blocks
    // put one wave on each of a CU's 4 SIMDs
    const int waves_per_simd = argc > 1 ? atoi(argv[1]) : 4;
    const int block = 256, grid = cus * waves_per_simd;
    printf("%d waves per SIMD\n", waves_per_simd);
    uint64_t* out;
    CHK(hipMalloc(&out, (size_t)grid * block * 8));
    struct { const char* name; kfn f; } ks[] = {
        {"v_mov_b32", k_mov32}, {"v_mov_b64", k_mov64}, {"v_pk_mov_b32", k_pkmov},
        {"v_not_b32", k_not32}, {"v_add_u32", k_add32}, {"v_mul_lo_u32", k_mullo},
        {"v_mul_hi_u32", k_mulhi}, {"v_mul_f64", k_fma64m},
        {"v_rcp_f64", k_rcp64}, {"v_fma_f32", k_fmaf32}, {"v_add_f32", k_addf32}, {"v_xor_b32", k_xor},
        {"v_bfi_b32", k_bfi}, {"v_alignbit_b32", k_alignbit}, {"v_add3_u32", k_add3},
        {"v_bfi_b32 (3 regs)", k_bfi_d}, {"v_add3_u32 (3 regs)", k_add3_d}, {"v_fma_f32 (3 regs)", k_fma_d},
        {"v_cndmask_b32 vcc", k_cndmask}, {"v_cndmask_b32 s[]", k_cndmask_s},
        {"v_cndmask_b32_e64 vcc", k_cndmask_e64vcc}, {"v_cndmask vcc<-SALU", k_cndmask_svcc}, {"v_mad_u64_u32", k_mad64},
        {"add256 chain e32/vcc", k_add256_e32}, {"add256 chain e64/sgpr", k_add256_e64},
        {"v_bitop3_b32 (3 regs)", k_bitop3_d},
        {"v_alignbit_b32 (3 regs)", k_alignbit_d}};
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const uint32_t iters = 4096;
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, 64u, out);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, iters, out);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        // wave-instructions per SIMD = iters x 16 x waves per SIMD
        const double cyc = ms * 1e-3 * 2.4e9 / ((double)iters * 16.0 * waves_per_simd);
        printf("%-20s %8.3f ms  %6.2f SIMD cycles per wave-instruction (at 2.4 GHz)\n", k.name, ms, cyc);
    }
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_clock, dim3(grid), dim3(block), 0, 0, iters, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms_clk; CHK(hipEventElapsedTime(&ms_clk, e0, e1));
    uint64_t h[2];
    CHK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / ((double)h[1] * 10.0);  // cycles per 10 ns tick
    // SIMD cycles per wave-instruction = the kernel's event time at the measured clock over
    // the instructions each SIMD issues.  (Round 3 divided ONE wave's s_memtime lifetime by
    // waves_per_simd x its instructions: that assumes every wave of the SIMD is resident for
    // the measured wave's whole life, which the dispatcher does not guarantee — at 8 waves it
    // read 0.75 cycles, below the 2-cycle wave64 issue floor.)  With 16 independent
    // instructions per wave these are latency-limited rates at that occupancy, not the VALU's
    // throughput (2 cycles per wave64 instruction, MI355X_MICROARCH.md).
    printf("shader clock during the add loop: %.3f GHz (one wave's s_memtime / s_memrealtime); "
           "v_add_u32: %.2f SIMD cycles per wave-instruction (event time at that clock)\n",
           ghz, ms_clk * 1e-3 * ghz * 1e9 / ((double)iters * 16.0 * waves_per_simd));
    return 0;
}
