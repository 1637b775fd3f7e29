// pf_keccak.hip — batched Keccak-256 (original Keccak padding, as eth_hash / Mythril's
// support_utils.sha3) for hash concretisation: one lane = one message, the 25-lane state
// in 50 VGPRs, 24 rounds fully unrolled.  Messages are the 64-byte key||slot mapping
// preimages in the common case (one Keccak-f[1600] block, rate 136 B).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__constant__ uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

__device__ __forceinline__ uint64_t rol64(uint64_t x, int n) {
    return n == 0 ? x : ((x << n) | (x >> (64 - n)));
}

// state index i = x + 5*y
__device__ __forceinline__ void keccakf(uint64_t s[25]) {
    // rho offsets r[x + 5y] and pi: B[y + 5*((2x+3y)%5)] = rol(A[x+5y], r)
    constexpr int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                           25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
#pragma unroll 1
    for (int rnd = 0; rnd < 24; rnd++) {
        uint64_t C[5], D[5], B[25];
#pragma unroll
        for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
#pragma unroll
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rol64(C[(x + 1) % 5], 1);
#pragma unroll
        for (int x = 0; x < 5; x++)
#pragma unroll
            for (int y = 0; y < 5; y++) {
                int i = x + 5 * y;
                B[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(s[i] ^ D[x], R[i]);
            }
#pragma unroll
        for (int x = 0; x < 5; x++)
#pragma unroll
            for (int y = 0; y < 5; y++)
                s[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
        s[0] ^= kRC[rnd];
    }
}

__device__ __forceinline__ void absorb_and_squeeze(const uint8_t* __restrict__ p, uint64_t len,
                                                   uint8_t* __restrict__ out) {
    uint64_t s[25];
#pragma unroll
    for (int i = 0; i < 25; i++) s[i] = 0;
    const uint64_t rate = 136;
    uint64_t off = 0;
    const bool aligned8 = (((uintptr_t)p) & 7u) == 0;
    // full blocks
    while (len - off >= rate) {
#pragma unroll
        for (int i = 0; i < 17; i++) {
            uint64_t lane;
            if (aligned8) {
                lane = *(const uint64_t*)(p + off + 8 * i);
            } else {
                lane = 0;
                for (int b = 0; b < 8; b++) lane |= (uint64_t)p[off + 8 * i + b] << (8 * b);
            }
            s[i] ^= lane;
        }
        keccakf(s);
        off += rate;
    }
    // last (partial) block with pad10*1, domain byte 0x01
    const uint64_t rem = len - off;
#pragma unroll
    for (int i = 0; i < 17; i++) {
        uint64_t lane = 0;
        for (int b = 0; b < 8; b++) {
            uint64_t k = 8 * (uint64_t)i + b;
            uint64_t byte = 0;
            if (k < rem) byte = p[off + k];
            else if (k == rem) byte = 0x01;
            if (k == rate - 1) byte |= 0x80;
            lane |= byte << (8 * b);
        }
        s[i] ^= lane;
    }
    keccakf(s);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t v = s[i];
#pragma unroll
        for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(v >> (8 * b));
    }
}

}  // namespace

extern "C" __global__ void __launch_bounds__(256)
pf_keccak_var_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                     uint64_t n, uint8_t* __restrict__ out32) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = offsets[i], b = offsets[i + 1];
    absorb_and_squeeze(data + a, b - a, out32 + 32 * i);
}

// fixed-length messages; len % 8 == 0 and len < 136 is the single-block fast path
// (loads 8 bytes per state lane, stores the digest as 4 x u64).
extern "C" __global__ void __launch_bounds__(256)
pf_keccak_fixed_kernel(const uint8_t* __restrict__ data, uint32_t len, uint64_t n,
                       uint8_t* __restrict__ out32) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = data + i * (uint64_t)len;
    if ((len & 7u) == 0u && len < 136u && ((((uintptr_t)data) & 7u) == 0u)) {
        uint64_t s[25];
#pragma unroll
        for (int k = 0; k < 25; k++) s[k] = 0;
        const uint64_t* q = (const uint64_t*)p;
        const uint32_t nl = len >> 3;
#pragma unroll
        for (int k = 0; k < 17; k++) {
            uint64_t v = ((uint32_t)k < nl) ? q[k] : 0ull;
            if ((uint32_t)k == nl) v ^= 0x01ull;
            if (k == 16) v ^= 0x8000000000000000ull;
            s[k] ^= v;
        }
        keccakf(s);
        uint64_t* o = (uint64_t*)(out32 + 32 * i);
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = s[k];
    } else {
        absorb_and_squeeze(p, len, out32 + 32 * i);
    }
}
