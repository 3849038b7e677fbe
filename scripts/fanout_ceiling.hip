// fanout_ceiling.hip — what bounds k_fanout_route at config 4 (10M accounts: a directory of 2^25 slots, 7M emitted
// messages per step from 1M publishers): the random probe into the 8-B (256 MiB) and 16-B (512 MiB) probe tables, alone
// and in the fan-out kernel's memory pattern (the CSR target read, runs of ~7 per publisher, + the probe + 8 B written).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fanout_ceiling scripts/fanout_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using u32x2 = unsigned int __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h;
}

// W = slot bytes (8 or 16): one random probe per item into `slots` slots
template <int W>
__global__ __launch_bounds__(256) void k_gather(const void* __restrict__ tab, uint32_t slots, uint32_t n, uint32_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t s = mix32(i * 2654435761u) & (slots - 1u);
        uint32_t x;
        if (W == 8) { const u32x2 v = static_cast<const u32x2*>(tab)[s]; x = v.x ^ v.y; }
        else { const u32x4 v = static_cast<const u32x4*>(tab)[s]; x = v.x ^ v.w; }
        out[i] = x;
    }
}

// the fan-out pattern: message i reads csr_tgt[i] (contiguous: the publishers' CSR runs), probes slot(tgt), writes 8 B
template <int W>
__global__ __launch_bounds__(256) void k_fan(const uint32_t* __restrict__ tgt, const void* __restrict__ tab, uint32_t slots,
                                             uint32_t n, uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t t = tgt[i];
        const uint32_t s = mix32(t * 0x9E3779B1u) & (slots - 1u);
        uint32_t x, y;
        if (W == 8) { const u32x2 v = static_cast<const u32x2*>(tab)[s]; x = v.x; y = v.y; }
        else { const u32x4 v = static_cast<const u32x4*>(tab)[s]; x = v.x; y = v.w; }
        o1[i] = x ^ t;
        o2[i] = y;
    }
}

__global__ void k_fill(u32x4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)i;
        a[i] = u32x4{mix32(x * 2654435761u + 1u), mix32(x * 2246822519u + 7u), mix32(x * 3266489917u + 3u), mix32(x ^ 0x9e3779b9u)};
    }
}

__global__ void k_targets(uint32_t* __restrict__ t, uint32_t n, uint32_t n_acc) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) t[i] = mix32(i + 17u) % n_acc;
}

int main() {
    const uint32_t n = 7u << 20, n_acc = 10000000u, slots = 1u << 25;  // 2^25 slots: next_pow2(2 x 10M)
    void* tab;
    uint32_t *tgt, *out;
    CK(hipMalloc(&tab, (size_t)slots * 16));
    CK(hipMalloc(&tgt, (size_t)n * 4));
    CK(hipMalloc(&out, (size_t)n * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, static_cast<u32x4*>(tab), (size_t)slots);
    hipLaunchKernelGGL(k_targets, dim3(8192), dim3(256), 0, 0, tgt, n, n_acc);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double items, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-52s %8.1f us  %7.2f G items/s\n", name, ms * 1e3, items / ms / 1e6);
        fflush(stdout);
    };
    const dim3 g(8192), b(256);
    timeit("gather 8-B slot, 256 MiB table (7M probes)", n, [&] { hipLaunchKernelGGL(k_gather<8>, g, b, 0, 0, tab, slots, n, out); });
    timeit("gather 16-B slot, 512 MiB table (7M probes)", n, [&] { hipLaunchKernelGGL(k_gather<16>, g, b, 0, 0, tab, slots, n, out); });
    timeit("gather 8-B slot, 128 MiB table", n, [&] { hipLaunchKernelGGL(k_gather<8>, g, b, 0, 0, tab, slots / 2, n, out); });
    timeit("fan-out pattern, 8-B table (256 MiB)", n, [&] { hipLaunchKernelGGL(k_fan<8>, g, b, 0, 0, tgt, tab, slots, n, out, out + n); });
    timeit("fan-out pattern, 16-B table (512 MiB)", n, [&] { hipLaunchKernelGGL(k_fan<16>, g, b, 0, 0, tgt, tab, slots, n, out, out + n); });
    return 0;
}
