// probe_ceiling.hip — what bounds k_route's directory probe on MI355X, and what an XCD-sliced probe table could gain.
//   1. random 8-B probes into tables of 1 .. 64 MiB, every workgroup probing the whole table (the L2 knee: 8 XCDs x
//      4 MiB of non-coherent L2; each XCD caches its own copy of whatever it touches);
//   2. the same 16 MiB table cut into 8 slices of 2 MiB, workgroup b probing only slice b % 8 (the slice of the XCD
//      it is dispatched to, round-robin) — the best an XCD-sliced table could do once messages are grouped by slice —
//      and slice (b / 8) % 8 as the control (every XCD then touches every slice);
//   3. k_route's memory pattern with the 8-B table (32-B header stream + 8-B probe + 8-B write) unsliced and sliced,
//      against the streaming pass any grouping by slice would add first (read 32-B headers, write 12-B records).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_ceiling scripts/probe_ceiling.hip (tools/ travels to the GPU box)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using u32x2 = unsigned int __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h;
}

// SLICE: 0 = whole table; 1 = slice of this block's XCD (b % 8); 2 = slice (b / 8) % 8 (control: all XCDs, all slices)
template <int SLICE>
__global__ __launch_bounds__(256) void k_gather8(const u32x2* __restrict__ tab, uint32_t slots, uint32_t n,
                                                 uint32_t* __restrict__ out) {
    const uint32_t per = slots / 8u;
    const uint32_t x = SLICE == 1 ? (blockIdx.x % 8u) : (blockIdx.x / 8u) % 8u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t h = mix32(i * 2654435761u);
        const uint32_t s = SLICE == 0 ? (h & (slots - 1u)) : x * per + (h & (per - 1u));
        const u32x2 v = tab[s];
        out[i] = v.x ^ v.y;
    }
}

// k_route's pattern with the 8-B probe table: 32-B header (non-temporal), probe slot from the header's hash, 8-B out
template <int SLICE>
__global__ __launch_bounds__(256) void k_route8(const u32x4* __restrict__ hdr, const u32x2* __restrict__ tab, uint32_t slots,
                                                uint32_t n, uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    const uint32_t per = slots / 8u;
    const uint32_t x = SLICE == 1 ? (blockIdx.x % 8u) : (blockIdx.x / 8u) % 8u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32x4 a = __builtin_nontemporal_load(hdr + 2 * (size_t)i);
        const u32x4 b = __builtin_nontemporal_load(hdr + 2 * (size_t)i + 1);
        const uint32_t h = mix32(a.x ^ b.x ^ a.z);
        const uint32_t s = SLICE == 0 ? (h & (slots - 1u)) : x * per + (h & (per - 1u));
        const u32x2 v = tab[s];
        o1[i] = v.x ^ a.y;
        o2[i] = v.y ^ b.w;
    }
}

// k_route's pattern against a bucketized 8-B table (8 slots per 64-B line, `nbk` buckets, not a power of two): the
// whole line read as 4 x 16-B loads, and a second line (the key's other bucket) for `second_pct` % of the messages
__global__ __launch_bounds__(256) void k_route8_bucket(const u32x4* __restrict__ hdr, const u32x4* __restrict__ tab, uint32_t nbk,
                                                       uint32_t second_pct, uint32_t n, uint32_t* __restrict__ o1,
                                                       uint32_t* __restrict__ o2) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32x4 a = __builtin_nontemporal_load(hdr + 2 * (size_t)i);
        const u32x4 b = __builtin_nontemporal_load(hdr + 2 * (size_t)i + 1);
        const uint32_t h = mix32(a.x ^ b.x ^ a.z);
        uint32_t bk = (uint32_t)(((uint64_t)h * nbk) >> 32);
        const u32x4* line = tab + (size_t)bk * 4;
        u32x4 v0 = line[0], v1 = line[1], v2 = line[2], v3 = line[3];
        uint32_t x = v0.x ^ v1.y ^ v2.z ^ v3.w;
        if ((h & 127u) * 100u < second_pct * 128u) {  // the other bucket
            bk = (uint32_t)(((uint64_t)mix32(h + 0x9E3779B9u) * nbk) >> 32);
            line = tab + (size_t)bk * 4;
            v0 = line[0]; v1 = line[1]; v2 = line[2]; v3 = line[3];
            x ^= v0.y ^ v1.z ^ v2.w ^ v3.x;
        }
        o1[i] = x ^ a.y;
        o2[i] = x ^ b.w;
    }
}

// the grouping pass a sliced table needs first, at its cheapest: stream the headers, write a 12-B record per message
// (slot start, key, index) — here to a contiguous position, i.e. without the partition's ranking and scatter
__global__ __launch_bounds__(256) void k_group_floor(const u32x4* __restrict__ hdr, uint32_t n, uint32_t* __restrict__ rec) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32x4 a = __builtin_nontemporal_load(hdr + 2 * (size_t)i);
        const u32x4 b = __builtin_nontemporal_load(hdr + 2 * (size_t)i + 1);
        rec[i] = mix32(a.x ^ b.x ^ a.z);
        rec[n + i] = a.z;
        rec[2 * (size_t)n + i] = i;
    }
}

__global__ void k_fill_random(u32x4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)i;
        a[i] = u32x4{mix32(x * 2654435761u + 1u), mix32(x * 2246822519u + 7u), mix32(x * 3266489917u + 3u), mix32(x ^ 0x9e3779b9u)};
    }
}

int main() {
    const uint32_t n = 64u << 20;
    const size_t hdr_bytes = (size_t)n * 32;
    u32x4 *hdr, *tab;
    uint32_t* out;
    CK(hipMalloc(&hdr, hdr_bytes));
    CK(hipMalloc(&tab, 64ull << 20));
    CK(hipMalloc(&out, (size_t)n * 12));
    hipLaunchKernelGGL(k_fill_random, dim3(4096), dim3(256), 0, 0, hdr, hdr_bytes / 16);
    hipLaunchKernelGGL(k_fill_random, dim3(4096), dim3(256), 0, 0, tab, (64ull << 20) / 16);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double items, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-44s %8.3f ms  %7.2f G items/s\n", name, ms, items / ms / 1e6);
    };
    const dim3 g(8192), b(256);
    const u32x2* t8 = reinterpret_cast<const u32x2*>(tab);
    char nm[96];
    for (uint32_t mb : {1u, 2u, 4u, 8u, 16u, 32u, 64u}) {
        const uint32_t slots = (mb << 20) / 8;
        snprintf(nm, sizeof nm, "gather8 whole table %u MiB", mb);
        timeit(nm, n, [&] { hipLaunchKernelGGL(k_gather8<0>, g, b, 0, 0, t8, slots, n, out); });
    }
    for (uint32_t mb : {16u, 64u}) {
        const uint32_t slots = (mb << 20) / 8;
        snprintf(nm, sizeof nm, "gather8 %u MiB, own-XCD slice of %u MiB", mb, mb / 8);
        timeit(nm, n, [&] { hipLaunchKernelGGL(k_gather8<1>, g, b, 0, 0, t8, slots, n, out); });
        snprintf(nm, sizeof nm, "gather8 %u MiB, slice b/8 (control)", mb);
        timeit(nm, n, [&] { hipLaunchKernelGGL(k_gather8<2>, g, b, 0, 0, t8, slots, n, out); });
    }
    const uint32_t s16 = (16u << 20) / 8;
    timeit("route8 pattern, 16 MiB table", n, [&] { hipLaunchKernelGGL(k_route8<0>, g, b, 0, 0, hdr, t8, s16, n, out, out + n); });
    timeit("route8 pattern, own-XCD 2 MiB slices", n, [&] { hipLaunchKernelGGL(k_route8<1>, g, b, 0, 0, hdr, t8, s16, n, out, out + n); });
    timeit("route8 pattern, slices b/8 (control)", n, [&] { hipLaunchKernelGGL(k_route8<2>, g, b, 0, 0, hdr, t8, s16, n, out, out + n); });
    timeit("grouping floor: 32-B hdr in, 12-B rec out", n, [&] { hipLaunchKernelGGL(k_group_floor, g, b, 0, 0, hdr, n, out); });
    // bucketized 8-B table for 1M entries: load 0.8 / 0.9 -> 9.8 / 8.7 MB; 0 / 13 / 25 % second-bucket reads
    for (uint32_t nbk : {163840u, 145636u, 262144u}) {
        for (uint32_t pct : {0u, 13u, 25u}) {
            snprintf(nm, sizeof nm, "route8 bucket table %.1f MB, %u%% 2nd", nbk * 64.0 / 1048576.0, pct);
            timeit(nm, n, [&] { hipLaunchKernelGGL(k_route8_bucket, g, b, 0, 0, hdr, tab, nbk, pct, n, out, out + n); });
        }
    }
    return 0;
}
