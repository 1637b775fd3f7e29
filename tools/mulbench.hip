// Micro-benchmark (diagnostic): issue cost of the multiply primitives on gfx950.
// Each lane runs `iters` rounds of 4 independent chains; grid = 2 waves per SIMD.
// Prints SIMD cycles per wave-instruction for each primitive.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../mythril_amd/csrc/u256.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

extern "C" __global__ void k_mad(uint32_t iters, uint64_t* out) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t m = 0x9E3779B9u + threadIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            a0 = (uint64_t)(uint32_t)a0 * m + a0; a1 = (uint64_t)(uint32_t)a1 * m + a1;
            a2 = (uint64_t)(uint32_t)a2 * m + a2; a3 = (uint64_t)(uint32_t)a3 * m + a3;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
}
extern "C" __global__ void k_add(uint32_t iters, uint64_t* out) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t m = 0x9E3779B9u + threadIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            a0 = a0 + (a1 ^ m); a1 = a1 + (a2 ^ m); a2 = a2 + (a3 ^ m); a3 = a3 + (a0 ^ m);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
}
extern "C" __global__ void k_mul256(uint32_t iters, uint64_t* out) {
    pf::u256 a, b;
    for (int i = 0; i < 8; i++) { a.l[i] = threadIdx.x * 77u + i; b.l[i] = 0x9E3779B9u * (i + 1); }
    for (uint32_t i = 0; i < iters; i++) a = pf::mul256(a, b);
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.l[0] ^ a.l[7];
}
extern "C" __global__ void k_mul256x2(uint32_t iters, uint64_t* out) {
    pf::u256 a, b, c;
    for (int i = 0; i < 8; i++) { a.l[i] = threadIdx.x * 77u + i; c.l[i] = a.l[i] ^ 0x55u; b.l[i] = 0x9E3779B9u * (i + 1); }
    for (uint32_t i = 0; i < iters; i++) { a = pf::mul256(a, b); c = pf::mul256(c, b); }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.l[0] ^ a.l[7] ^ c.l[3];
}
extern "C" __global__ void k_mad1(uint32_t iters, uint64_t* out) {
    uint64_t a0 = threadIdx.x;
    uint32_t m = 0x9E3779B9u + threadIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 64; j++) a0 = (uint64_t)(uint32_t)a0 * m + a0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}
extern "C" __global__ void k_sqr256(uint32_t iters, uint64_t* out) {
    pf::u256 a;
    for (int i = 0; i < 8; i++) a.l[i] = threadIdx.x * 77u + i + 3;
    for (uint32_t i = 0; i < iters; i++) a = pf::sqr256(a);
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.l[0] ^ a.l[7];
}
extern "C" __global__ void k_add256(uint32_t iters, uint64_t* out) {
    pf::u256 a, b;
    for (int i = 0; i < 8; i++) { a.l[i] = threadIdx.x * 77u + i; b.l[i] = 0x9E3779B9u * (i + 1); }
    for (uint32_t i = 0; i < iters; i++) { a = pf::add256(a, b); b.l[0] ^= a.l[7]; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.l[0] ^ a.l[7];
}

typedef void (*kfn)(uint32_t, uint64_t*);
int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int block = 256, grid = cus * 2;  // 2 waves per SIMD
    uint64_t* out;
    CHK(hipMalloc(&out, (size_t)grid * block * 8));
    struct { const char* name; kfn f; uint32_t iters; double per_iter; } ks[] = {
        {"mad_u64_u32", k_mad, 4096, 64}, {"add_u32(+xor)", k_add, 4096, 128},
        {"mad 1 chain", k_mad1, 4096, 64}, {"mul256", k_mul256, 8192, 1}, {"mul256 x2 indep", k_mul256x2, 8192, 2}, {"sqr256", k_sqr256, 8192, 1}, {"add256", k_add256, 8192, 1}};
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, 16u, out);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, k.iters, out);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        // waves per SIMD = 2; SIMD cycles at 2.4 GHz / (ops per wave x 2 waves)
        double cyc = ms * 1e-3 * 2.4e9 / (k.iters * k.per_iter * 2.0);
        printf("%-16s %8.3f ms  %8.2f SIMD cycles per op per wave\n", k.name, ms, cyc);
    }
    return 0;
}
