// Micro-benchmark (diagnostic): issue cost on gfx950 of the data-movement and arithmetic
// instructions the interpreter spends its non-algorithmic VALU cycles on — 32- vs 64-bit
// register copies (operand reads / write-backs), per-limb selects, 32-bit multiplies (the
// EXP Horner chain's Hensel divisions) and the f64 ops of the division estimates.
// Each lane runs `iters` rounds of 16 independent instructions (inline asm, so the compiler
// cannot fold or reorder them); grid = 4 waves per SIMD, the search kernels' occupancy.
// Prints SIMD cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

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

typedef void (*kfn)(uint32_t, uint64_t*);
int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int block = 256, waves_per_simd = 4, grid = cus * waves_per_simd;
    uint64_t* out;
    CHK(hipMalloc(&out, (size_t)grid * block * 8));
    struct { const char* name; kfn f; } ks[] = {
        {"v_mov_b32", k_mov32}, {"v_mov_b64", k_mov64}, {"v_pk_mov_b32", k_pkmov},
        {"v_not_b32", k_not32}, {"v_add_u32", k_add32}, {"v_mul_lo_u32", k_mullo},
        {"v_mul_hi_u32", k_mulhi}, {"v_mul_f64", k_fma64m},
        {"v_rcp_f64", k_rcp64}};
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
        printf("%-14s %8.3f ms  %6.2f SIMD cycles per wave-instruction (at 2.4 GHz)\n", k.name, ms, cyc);
    }
    return 0;
}
