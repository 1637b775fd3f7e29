// Launch cost of a grid of short waves (the early-exit search of a small batch launches
// ~1,000-4,000 waves that mostly find their set decided and leave): kernels that do almost
// nothing, with and without the search kernel's per-wave resources — 10 KiB of LDS, 2,320 B
// of scratch per lane, 128 VGPRs — at one and four waves per workgroup.  Timed with events
// over back-to-back launches.  Tool (tools/, not product).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/launchbench tools/launchbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

extern "C" __global__ void k_empty(uint32_t* out, uint32_t n) {
    if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFFu) out[0] = n;
}

template <int LDSB>
__global__ void k_lds(uint32_t* out, uint32_t n) {
    __shared__ uint32_t s[LDSB / 4];
    s[threadIdx.x] = n;
    __syncthreads();
    if (s[(threadIdx.x + 1) % blockDim.x] == 0xFFFFFFFFu) out[0] = n;
}

// private array indexed by a run-time value: the compiler keeps it in scratch
template <int LDSB>
__global__ void k_scratch(uint32_t* out, uint32_t n) {
    __shared__ uint32_t s[LDSB / 4];
    uint32_t a[580];
    a[(threadIdx.x * 7u + n) % 580u] = n;
    s[threadIdx.x] = a[(threadIdx.x + n) % 580u];
    __syncthreads();
    if (s[(threadIdx.x + 1) % blockDim.x] == 0xFFFFFFFFu) out[0] = n;
}

template <typename K>
int time_kernel(const char* name, K kern, uint32_t waves, uint32_t wg_waves, uint32_t* d) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const uint32_t blocks = (waves + wg_waves - 1) / wg_waves;
    for (int i = 0; i < 10; i++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wg_waves), 0, 0, d, 1u);
    CHK(hipEventRecord(a));
    const int reps = 200;
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wg_waves), 0, 0, d, 1u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, a, b));
    printf("%-28s waves %5u  wg %u  %8.2f us per launch\n", name, waves, wg_waves, 1e3f * ms / reps);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return 0;
}

int main() {
    uint32_t* d = nullptr;
    CHK(hipMalloc(&d, 64));
    for (uint32_t waves : {64u, 1024u, 4096u, 16384u}) {
        if (time_kernel("empty", k_empty, waves, 1, d)) return 1;
        if (time_kernel("lds 10 KiB", k_lds<10240>, waves, 1, d)) return 1;
        if (time_kernel("lds 10 KiB + scratch 2.3 KB", k_scratch<10240>, waves, 1, d)) return 1;
        if (time_kernel("lds 40 KiB + scratch, wg4", k_scratch<40960>, waves, 4, d)) return 1;
    }
    CHK(hipFree(d));
    return 0;
}
