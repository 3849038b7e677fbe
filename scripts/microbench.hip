// microbench.hip — memory-system ceilings on MI355X for the routing engine's access patterns.
//   copy / read stream (HBM peak as a kernel sees it), random 16-B / 32-B gathers from tables of
//   64 MB .. 1 GB (the directory probe), and the route kernel's mix (32-B header stream + 32-B probe
//   + 8-B write).  Build: hipcc --offload-arch=gfx950 -O3 -o build/microbench scripts/microbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h;
}

__global__ void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

__global__ void k_read(const u32x4* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t x = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = a[i]; x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) out[0] = x;
}

// one lookup per thread-iteration: W bytes (16 or 32) at a random slot of a table of `mask+1` 32-B slots
template <int W>
__global__ void k_gather(const u32x4* __restrict__ tab, uint64_t mask, uint32_t n, uint32_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t s = mix32(i * 2654435761u) & mask;
        u32x4 a = tab[2 * s];
        uint32_t x = a.x ^ a.w;
        if (W == 32) { u32x4 b = tab[2 * s + 1]; x ^= b.y ^ b.z; }
        out[i] = x;
    }
}

// lane pairs fetch one 32-B slot together (16 B each) then swap halves: one contiguous 32 B per pair per instruction
__global__ void k_gather_pair(const u32x4* __restrict__ tab, uint64_t mask, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t mine = mix32(i * 2654435761u) & mask;
        const uint64_t other = __shfl_xor((unsigned long long)mine, 1);
        // instruction 1: even lane's slot; instruction 2: odd lane's slot
        const uint64_t s0 = (lane & 1) ? other : mine;
        const uint64_t s1 = (lane & 1) ? mine : other;
        const u32x4 v0 = tab[2 * s0 + (lane & 1)];
        const u32x4 v1 = tab[2 * s1 + (lane & 1)];
        uint32_t x0 = v0.x ^ v0.w, x1 = v1.y ^ v1.z;
        const uint32_t y0 = __shfl_xor(x0, 1), y1 = __shfl_xor(x1, 1);
        out[i] = (lane & 1) ? (x1 ^ y1) : (x0 ^ y0);
    }
}

// the route kernel's memory pattern: stream a 32-B header, probe a 32-B slot, write 8 B
__global__ void k_route_mix(const u32x4* __restrict__ hdr, const u32x4* __restrict__ tab, uint64_t mask, uint32_t n,
                            uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32x4 a = __builtin_nontemporal_load(hdr + 2 * (size_t)i);
        const u32x4 b = __builtin_nontemporal_load(hdr + 2 * (size_t)i + 1);
        const uint64_t s = mix32(a.x ^ b.x ^ a.z) & mask;
        const u32x4 c = tab[2 * s];
        const u32x4 d = tab[2 * s + 1];
        o1[i] = c.x ^ d.w;
        o2[i] = c.y ^ d.z;
    }
}

// ILP form: each thread issues K independent random 32-B probes before consuming any
template <int K>
__global__ void k_gather_ilp(const u32x4* __restrict__ tab, uint64_t mask, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * K) {
        u32x4 a[K], b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = i0 + k * stride;
            const uint64_t s = mix32(i * 2654435761u) & mask;
            a[k] = tab[2 * s];
            b[k] = tab[2 * s + 1];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = i0 + k * stride;
            if (i < n) out[i] = a[k].x ^ b[k].w;
        }
    }
}

// route mix with the next header group prefetched while the current probes are in flight
template <int K>
__global__ void k_route_mix_pipe(const u32x4* __restrict__ hdr, const u32x4* __restrict__ tab, uint64_t mask, uint32_t n,
                                 uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 ha[K], hb[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const size_t i = t + (size_t)k * stride;
        if (i < n) { ha[k] = __builtin_nontemporal_load(hdr + 2 * i); hb[k] = __builtin_nontemporal_load(hdr + 2 * i + 1); }
    }
    for (uint32_t i0 = t; i0 < n; i0 += stride * K) {
        u32x4 c[K], d[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t s = mix32(ha[k].x ^ hb[k].x ^ ha[k].z) & mask;
            c[k] = tab[2 * s];
            d[k] = tab[2 * s + 1];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const size_t i = i0 + (size_t)(K + k) * stride;
            if (i < n) { ha[k] = __builtin_nontemporal_load(hdr + 2 * i); hb[k] = __builtin_nontemporal_load(hdr + 2 * i + 1); }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = i0 + k * stride;
            if (i < n) { o1[i] = c[k].x ^ d[k].w; o2[i] = c[k].y ^ d[k].z; }
        }
    }
}

__global__ void k_fill_random(u32x4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)i;
        a[i] = u32x4{mix32(x * 2654435761u + 1u), mix32(x * 2246822519u + 7u), mix32(x * 3266489917u + 3u), mix32(x ^ 0x9e3779b9u)};
    }
}

// route mix with plain (temporal) header loads
__global__ void k_route_mix_t(const u32x4* __restrict__ hdr, const u32x4* __restrict__ tab, uint64_t mask, uint32_t n,
                              uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32x4 a = hdr[2 * (size_t)i];
        const u32x4 b = hdr[2 * (size_t)i + 1];
        const uint64_t s = mix32(a.x ^ b.x ^ a.z) & mask;
        const u32x4 c = tab[2 * s];
        const u32x4 d = tab[2 * s + 1];
        o1[i] = c.x ^ d.w;
        o2[i] = c.y ^ d.z;
    }
}

int main(int argc, char** argv) {
    const size_t stream_bytes = 2ull << 30;
    const uint32_t n = 64u << 20;
    u32x4 *a, *b;
    uint32_t* out;
    CK(hipMalloc(&a, stream_bytes));
    CK(hipMalloc(&b, stream_bytes));
    CK(hipMalloc(&out, (size_t)n * 8));
    hipLaunchKernelGGL(k_fill_random, dim3(4096), dim3(256), 0, 0, a, stream_bytes / 16);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, double items, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-34s %8.3f ms  %8.1f GB/s  %7.2f G items/s\n", name, ms, bytes / ms / 1e6, items / ms / 1e6);
    };
    const size_t n16 = stream_bytes / 16;
    const int grid = 256 * 16;
    timeit("copy 2 GiB (r+w)", 2.0 * stream_bytes, (double)n16, [&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n16); });
    timeit("read 2 GiB", (double)stream_bytes, (double)n16, [&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n16, out); });
    for (size_t tb : {16ull << 20, 64ull << 20, 256ull << 20, 1024ull << 20}) {
        const uint64_t mask = tb / 32 - 1;
        char nm[64];
        snprintf(nm, sizeof nm, "gather16 table %zu MB", tb >> 20);
        timeit(nm, 16.0 * n + 4.0 * n, n, [&] { hipLaunchKernelGGL(k_gather<16>, dim3(grid), dim3(256), 0, 0, b, mask, n, out); });
        snprintf(nm, sizeof nm, "gather32 table %zu MB", tb >> 20);
        timeit(nm, 32.0 * n + 4.0 * n, n, [&] { hipLaunchKernelGGL(k_gather<32>, dim3(grid), dim3(256), 0, 0, b, mask, n, out); });
        snprintf(nm, sizeof nm, "gather32 pair table %zu MB", tb >> 20);
        timeit(nm, 32.0 * n + 4.0 * n, n, [&] { hipLaunchKernelGGL(k_gather_pair, dim3(grid), dim3(256), 0, 0, b, mask, n, out); });
        snprintf(nm, sizeof nm, "route mix table %zu MB", tb >> 20);
        timeit(nm, 72.0 * n, n, [&] { hipLaunchKernelGGL(k_route_mix, dim3(grid), dim3(256), 0, 0, a, b, mask, n, out, out + n); });
        snprintf(nm, sizeof nm, "route mix (temporal hdr) %zu MB", tb >> 20);
        timeit(nm, 72.0 * n, n, [&] { hipLaunchKernelGGL(k_route_mix_t, dim3(grid), dim3(256), 0, 0, a, b, mask, n, out, out + n); });
        snprintf(nm, sizeof nm, "gather32 ilp4 table %zu MB", tb >> 20);
        timeit(nm, 32.0 * n + 4.0 * n, n, [&] { hipLaunchKernelGGL(k_gather_ilp<4>, dim3(grid), dim3(256), 0, 0, b, mask, n, out); });
        snprintf(nm, sizeof nm, "gather32 ilp8 table %zu MB", tb >> 20);
        timeit(nm, 32.0 * n + 4.0 * n, n, [&] { hipLaunchKernelGGL(k_gather_ilp<8>, dim3(grid), dim3(256), 0, 0, b, mask, n, out); });
        for (int g : {1024, 4096, 16384}) {
            snprintf(nm, sizeof nm, "route pipe4 g%d table %zu MB", g, tb >> 20);
            timeit(nm, 72.0 * n, n, [&] { hipLaunchKernelGGL(k_route_mix_pipe<4>, dim3(g), dim3(256), 0, 0, a, b, mask, n, out, out + n); });
        }
        snprintf(nm, sizeof nm, "route pipe8 g4096 table %zu MB", tb >> 20);
        timeit(nm, 72.0 * n, n, [&] { hipLaunchKernelGGL(k_route_mix_pipe<8>, dim3(4096), dim3(256), 0, 0, a, b, mask, n, out, out + n); });
    }
    return 0;
}
