// pf_keccak.hip — batched Keccak-256 (original Keccak padding, as eth_hash / Mythril's
// support_utils.sha3) for hash concretisation: one lane = one message.
//
// gfx950 layout of the permutation: the 25 64-bit lanes live as 50 32-bit halves in VGPRs
// (there is no 64-bit rotate or xor on the VALU, so working on halves costs nothing extra):
//   * 64-bit rotates   = 2 x v_alignbit_b32 (a rotate by 32 is a rename);
//   * theta            = column parities with 3-input xors (v_bitop3_b32, table 0x96), then
//                        a[i] ^= C[x-1] ^ rot1(C[x+1]) as one 3-input xor per half;
//   * rho + pi         = the in-place 24-cycle (one temp; after unrolling every move is a
//                        register rename);
//   * chi              = one v_bitop3_b32 per half: a ^ (~b & c) = truth table 0xD2 over
//                        (a, b, c) — gfx950-only instruction;
//   * iota             = two scalar-operand xors.
// ≈ 178 VALU instructions per round, ≈ 4,280 per Keccak-f[1600] (unrolled form: 61 VGPRs,
// no LDS, no scratch).
// Messages are the 64-byte key||slot mapping preimages in the common case (one block,
// rate 136 B); pf_keccak_fixed_kernel reads them as 16-byte vectors.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__constant__ uint32_t kRC[48] = {
    0x00000001u, 0x00000000u, 0x00008082u, 0x00000000u, 0x0000808Au, 0x80000000u,
    0x80008000u, 0x80000000u, 0x0000808Bu, 0x00000000u, 0x80000001u, 0x00000000u,
    0x80008081u, 0x80000000u, 0x00008009u, 0x80000000u, 0x0000008Au, 0x00000000u,
    0x00000088u, 0x00000000u, 0x80008009u, 0x00000000u, 0x8000000Au, 0x00000000u,
    0x8000808Bu, 0x00000000u, 0x0000008Bu, 0x80000000u, 0x00008089u, 0x80000000u,
    0x00008003u, 0x80000000u, 0x00008002u, 0x80000000u, 0x00000080u, 0x80000000u,
    0x0000800Au, 0x00000000u, 0x8000000Au, 0x80000000u, 0x80008081u, 0x80000000u,
    0x00008080u, 0x80000000u, 0x80000001u, 0x00000000u, 0x80008008u, 0x80000000u};

struct Lane {
    uint32_t lo, hi;
};

// rotate left by a compile-time amount
template <int N>
__device__ __forceinline__ Lane rotl(Lane v) {
    static_assert(N >= 0 && N < 64, "rotation");
    if constexpr (N == 0) {
        return v;
    } else if constexpr (N == 32) {
        return Lane{v.hi, v.lo};
    } else if constexpr (N < 32) {
        return Lane{__builtin_amdgcn_alignbit(v.lo, v.hi, 32 - N),
                    __builtin_amdgcn_alignbit(v.hi, v.lo, 32 - N)};
    } else {
        return Lane{__builtin_amdgcn_alignbit(v.hi, v.lo, 64 - N),
                    __builtin_amdgcn_alignbit(v.lo, v.hi, 64 - N)};
    }
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, (unsigned char)0x96);  // a ^ b ^ c
}

__device__ __forceinline__ uint32_t chi(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, (unsigned char)0xD2);  // a ^ (~b & c)
}

// the pi cycle (lane index order) and the rho offsets along it
constexpr int kPi[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4,
                         15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
constexpr int kRho[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14,
                          27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};

template <int I>
__device__ __forceinline__ void rho_pi_step(Lane a[25], Lane& t) {
    if constexpr (I < 24) {
        const Lane next = a[kPi[I]];
        a[kPi[I]] = rotl<kRho[I]>(t);
        t = next;
        rho_pi_step<I + 1>(a, t);
    }
}

__device__ __forceinline__ void keccak_round(Lane a[25], uint32_t rc_lo, uint32_t rc_hi) {
    // theta
    Lane C[5], R[5];
#pragma unroll
    for (int x = 0; x < 5; x++) {
        C[x].lo = xor3(xor3(a[x].lo, a[x + 5].lo, a[x + 10].lo), a[x + 15].lo, a[x + 20].lo);
        C[x].hi = xor3(xor3(a[x].hi, a[x + 5].hi, a[x + 10].hi), a[x + 15].hi, a[x + 20].hi);
    }
#pragma unroll
    for (int x = 0; x < 5; x++) R[x] = rotl<1>(C[(x + 1) % 5]);
#ifdef PF_KECCAK_THETA2
    // D[x] = C[x-1] ^ rot1(C[x+1]) once per column, then two-source xors into the 25 lanes:
    // 10 + 50 two-source ops instead of 50 three-source ones
#pragma unroll
    for (int x = 0; x < 5; x++) {
        const uint32_t dlo = C[(x + 4) % 5].lo ^ R[x].lo, dhi = C[(x + 4) % 5].hi ^ R[x].hi;
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
            a[x + y].lo ^= dlo;
            a[x + y].hi ^= dhi;
        }
    }
#else
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
            a[x + y].lo = xor3(a[x + y].lo, C[(x + 4) % 5].lo, R[x].lo);
            a[x + y].hi = xor3(a[x + y].hi, C[(x + 4) % 5].hi, R[x].hi);
        }
#endif
    // rho + pi
    Lane t = a[1];
    rho_pi_step<0>(a, t);
    // chi
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
        Lane b[5];
#pragma unroll
        for (int x = 0; x < 5; x++) b[x] = a[y + x];
#pragma unroll
        for (int x = 0; x < 5; x++) {
            a[y + x].lo = chi(b[x].lo, b[(x + 1) % 5].lo, b[(x + 2) % 5].lo);
            a[y + x].hi = chi(b[x].hi, b[(x + 1) % 5].hi, b[(x + 2) % 5].hi);
        }
    }
    // iota
    a[0].lo ^= rc_lo;
    a[0].hi ^= rc_hi;
}

// kUnrolled: all 24 rounds unrolled (~4.3k instructions, 34 KB of code): the pi cycle has
// order 24, so every lane move becomes a register rename — the rolled loop pays ~110 moves
// per round at its back edge.  The rolled form serves the multi-block general path.
template <bool kUnrolled>
__device__ __forceinline__ void keccakf(Lane a[25]) {
    if constexpr (kUnrolled) {
#pragma unroll
        for (int rnd = 0; rnd < 24; rnd++) keccak_round(a, kRC[2 * rnd], kRC[2 * rnd + 1]);
    } else {
#pragma unroll 1
        for (int rnd = 0; rnd < 24; rnd++) keccak_round(a, kRC[2 * rnd], kRC[2 * rnd + 1]);
    }
}

__device__ __forceinline__ void squeeze(const Lane a[25], uint8_t* __restrict__ out) {
    if ((((uintptr_t)out) & 15u) == 0u) {
        uint4* o = (uint4*)out;
        o[0] = make_uint4(a[0].lo, a[0].hi, a[1].lo, a[1].hi);
        o[1] = make_uint4(a[2].lo, a[2].hi, a[3].lo, a[3].hi);
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int b = 0; b < 4; b++) {
                out[8 * i + b] = (uint8_t)(a[i].lo >> (8 * b));
                out[8 * i + 4 + b] = (uint8_t)(a[i].hi >> (8 * b));
            }
    }
}

// General path: any length, any alignment (pad10*1 with domain byte 0x01).  Each block is
// staged bytewise through the thread's own LDS column ([word][thread], no bank conflicts, no
// barrier: a thread reads only what it wrote) so the state absorbs it with 34 static-offset
// LDS reads — byte loads straight into the state would keep up to 136 of them in flight
// (the compiler hoists them) and triple the kernel's VGPR budget.
constexpr int kGenThreads = 256;

__device__ __forceinline__ void absorb_staged(Lane a[25], uint32_t* __restrict__ col,
                                              const uint8_t* __restrict__ p, uint32_t nbytes,
                                              bool last) {
#pragma unroll 1
    for (int w = 0; w < 34; w++) col[w * kGenThreads] = 0u;
#pragma unroll 1
    for (uint32_t k = 0; k < nbytes; k++)
        col[(k >> 2) * kGenThreads] |= (uint32_t)p[k] << (8 * (k & 3));
    if (last) {
        col[(nbytes >> 2) * kGenThreads] ^= 0x01u << (8 * (nbytes & 3));
        col[33 * kGenThreads] ^= 0x80000000u;
    }
#pragma unroll
    for (int i = 0; i < 17; i++) {
        a[i].lo ^= col[(2 * i) * kGenThreads];
        a[i].hi ^= col[(2 * i + 1) * kGenThreads];
    }
}

__device__ __forceinline__ void absorb_and_squeeze(uint32_t* __restrict__ col,
                                                   const uint8_t* __restrict__ p, uint64_t len,
                                                   uint8_t* __restrict__ out) {
    Lane a[25];
#pragma unroll
    for (int i = 0; i < 25; i++) a[i] = Lane{0u, 0u};
    const uint64_t rate = 136;
    uint64_t off = 0;
    while (len - off >= rate) {
        absorb_staged(a, col, p + off, (uint32_t)rate, false);
        keccakf<false>(a);
        off += rate;
    }
    absorb_staged(a, col, p + off, (uint32_t)(len - off), true);
    keccakf<false>(a);
    squeeze(a, out);
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kGenThreads)
pf_keccak_var_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                     uint64_t n, uint8_t* __restrict__ out32) {
    __shared__ uint32_t stage[34 * kGenThreads];
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = offsets[i], b = offsets[i + 1];
    absorb_and_squeeze(stage + threadIdx.x, data + a, b - a, out32 + 32 * i);
}

// fixed-length messages, general case (any length / alignment)
extern "C" __global__ void __launch_bounds__(kGenThreads)
pf_keccak_stride_kernel(const uint8_t* __restrict__ data, uint32_t len, uint64_t n,
                        uint8_t* __restrict__ out32) {
    __shared__ uint32_t stage[34 * kGenThreads];
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    absorb_and_squeeze(stage + threadIdx.x, data + i * (uint64_t)len, len, out32 + 32 * i);
}

// Persistent form of the fixed-length fast path (PF_KECCAK_PERSIST): a chip-filling grid in
// which every lane walks messages i, i + stride, ...; the next message's 16-byte chunks are
// loaded while the current permutation runs, so a wave's load latency overlaps its own
// VALU work instead of relying on other waves alone.
// NQ: 16-byte chunks per message (4 for the 64-byte key||slot preimages), a template so the
// prefetch buffer holds only the chunks that exist
template <int NQ>
__device__ __forceinline__ void keccak_persist(const uint8_t* __restrict__ data, uint32_t len, uint64_t n,
                                               uint8_t* __restrict__ out32) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr uint32_t nq = NQ;
    uint4 nxt[NQ];
#pragma unroll
    for (int k = 0; k < NQ; k++)
        nxt[k] = i < n ? ((const uint4*)(data + i * (uint64_t)len))[k] : make_uint4(0u, 0u, 0u, 0u);
    for (; i < n; i += stride) {
        Lane a[25];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint4 v = k < NQ ? nxt[k < NQ ? k : 0] : make_uint4(0u, 0u, 0u, 0u);
            a[2 * k] = Lane{v.x, v.y};
            a[2 * k + 1] = Lane{v.z, v.w};
        }
        const uint64_t j = i + stride;
#pragma unroll
        for (int k = 0; k < NQ; k++)
            nxt[k] = j < n ? ((const uint4*)(data + j * (uint64_t)len))[k] : make_uint4(0u, 0u, 0u, 0u);
        a[16] = Lane{0u, 0x80000000u};
#pragma unroll
        for (int k = 17; k < 25; k++) a[k] = Lane{0u, 0u};
#pragma unroll
        for (int k = 0; k < 17; k++)
            if ((uint32_t)k == (len >> 3)) a[k].lo ^= 0x01u;
        keccakf<true>(a);
        squeeze(a, out32 + 32 * i);
    }
}

// the 64-byte key||slot preimages (config 4); other lengths take pf_keccak_fixed_kernel
extern "C" __global__ void __launch_bounds__(256)
pf_keccak_fixed64_persist_kernel(const uint8_t* __restrict__ data, uint64_t n, uint8_t* __restrict__ out32) {
    keccak_persist<4>(data, 64u, n, out32);
}

#ifdef PF_KECCAK_ILP2
// Probe (PF_KECCAK_ILP2): two messages per lane, i and i + ceil(n/2), their permutations
// interleaved round by round — two independent dependency chains per wave instead of one.
__device__ __forceinline__ void load_fixed(Lane a[25], const uint8_t* __restrict__ data, uint32_t len,
                                           uint64_t i, bool live) {
    const uint4* q = (const uint4*)(data + i * (uint64_t)len);
    const uint32_t nq = len >> 4;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint4 v = (live && (uint32_t)k < nq) ? q[k] : make_uint4(0u, 0u, 0u, 0u);
        a[2 * k] = Lane{v.x, v.y};
        a[2 * k + 1] = Lane{v.z, v.w};
    }
    a[16] = Lane{0u, 0x80000000u};
#pragma unroll
    for (int k = 17; k < 25; k++) a[k] = Lane{0u, 0u};
#pragma unroll
    for (int k = 0; k < 17; k++)
        if ((uint32_t)k == (len >> 3)) a[k].lo ^= 0x01u;
}

extern "C" __global__ void __launch_bounds__(256)
pf_keccak_fixed2_kernel(const uint8_t* __restrict__ data, uint32_t len, uint64_t n,
                        uint8_t* __restrict__ out32) {
    const uint64_t half = (n + 1) / 2;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= half) return;
    const uint64_t j = i + half;
    const bool has_j = j < n;
    Lane a[25], b[25];
    load_fixed(a, data, len, i, true);
    load_fixed(b, data, len, has_j ? j : i, has_j);
#pragma unroll
    for (int rnd = 0; rnd < 24; rnd++) {
        keccak_round(a, kRC[2 * rnd], kRC[2 * rnd + 1]);
        keccak_round(b, kRC[2 * rnd], kRC[2 * rnd + 1]);
    }
    squeeze(a, out32 + 32 * i);
    if (has_j) squeeze(b, out32 + 32 * j);
}
#endif

// fixed-length single-block fast path: the host launches it when len % 16 == 0,
// len < 136 and the buffer is 16-byte aligned (16-byte vector loads, two 16-byte digest
// stores, all 24 rounds unrolled).
extern "C" __global__ void __launch_bounds__(256)
pf_keccak_fixed_kernel(const uint8_t* __restrict__ data, uint32_t len, uint64_t n,
                       uint8_t* __restrict__ out32) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* q = (const uint4*)(data + i * (uint64_t)len);
    Lane a[25];
    const uint32_t nq = len >> 4;  // 16-byte chunks = state lane pairs
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint4 v = ((uint32_t)k < nq) ? q[k] : make_uint4(0u, 0u, 0u, 0u);
        a[2 * k] = Lane{v.x, v.y};
        a[2 * k + 1] = Lane{v.z, v.w};
    }
    a[16] = Lane{0u, 0x80000000u};
#pragma unroll
    for (int k = 17; k < 25; k++) a[k] = Lane{0u, 0u};
    // domain byte at offset len = low byte of state lane len/8
#pragma unroll
    for (int k = 0; k < 17; k++)
        if ((uint32_t)k == (len >> 3)) a[k].lo ^= 0x01u;
    keccakf<true>(a);
    squeeze(a, out32 + 32 * i);
}
