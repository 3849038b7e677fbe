// stage4_ceiling.hip — the memory-pattern floors of stage 4's two-level counting sort at config 2 (64M messages, 1M
// activations = 20-bit keys, 10 + 10 bits), against which k_radix_pass / k_seg_count / k_seg_scatter are judged.
// Every floor moves the bytes of its kernel in the kernel's own global access pattern, with no ranking at all: the input
// is laid out so each element's rank is known from its position (tiles and segments already in digit order, four
// elements per digit, as a uniform 4096-element tile has on average), so what remains is the streaming read, the
// scattered runs of the write, and — in the "+lds" variants — the LDS traffic the real kernels cannot avoid.
//   msd      read act (4 B, stream) -> write {key, index} (8 B) to bucket-major runs: 4 pairs (32 B) per digit per tile
//   count    read pairs (8 B, stream) [+ one LDS atomic per element on its low digit, 1024 counters]
//   scatter  read pairs (8 B, stream) -> write index (4 B) to its final position: runs of 4 (16 B) per key per
//            segment, keys 64 elements apart (each 64-B line gets 16 B from 4 segments)
//   + the streaming floors of the same byte counts (contiguous writes).
// "occ3": the launch reserves dynamic LDS so at most 3 workgroups share a CU, the occupancy the real scatter kernels run
// at (4 per CU made config 2's stage 4 slower — more partial lines in flight per L2).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/stage4_ceiling scripts/stage4_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t kTile = 4096;   // MSD tile / level-2 segment
constexpr uint32_t kDig = 1024;    // 10-bit digits
constexpr uint32_t kRun = kTile / kDig;

using u32x2 = unsigned int __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 ld_nt(const uint2* p) {
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    return make_uint2(v.x, v.y);
}

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h;
}

// act of element e: tile-local digit order (digit = (e % tile) / 4), random low digit
__global__ void k_fill_act(uint32_t* __restrict__ act, uint32_t n) {
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u)
        act[e] = (((e % kTile) / kRun) << 10) | (mix32(e) & (kDig - 1u));
}

// pairs of level 2: segment-local low-digit order (low digit = (i % seg) / 4), index random
__global__ void k_fill_pairs(uint2* __restrict__ p, uint32_t n) {
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u)
        p[e] = make_uint2((mix32(e * 7u) & ~(kDig - 1u)) | ((e % kTile) / kRun), mix32(e) % n);
}

// XCD-aware tile order as k_radix_pass (consecutive tiles on one XCD): block b -> tile
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t ntiles) {
    const uint32_t per = ntiles / 8u;
    if (b >= per * 8u) return b;
    return (b % 8u) * per + b / 8u;
}

template <bool XCD>
__global__ __launch_bounds__(256) void k_msd_floor(const uint32_t* __restrict__ act, uint32_t n, uint32_t ntiles,
                                                   uint2* __restrict__ out) {
    const uint32_t t = XCD ? xcd_tile(blockIdx.x, ntiles) : blockIdx.x;
#pragma unroll 4
    for (uint32_t j = 0; j < kTile / 256u; ++j) {
        const uint32_t i = j * 256u + threadIdx.x, e = t * kTile + i;
        const uint32_t a = __builtin_nontemporal_load(act + e);
        const uint32_t d = a >> 10;
        const uint32_t g = d * (ntiles * kRun) + t * kRun + (i % kRun);
        out[g] = make_uint2(a, e);
    }
}

// the same with the real kernel's LDS staging: elements through an 8-B LDS image (write at a scattered position,
// read back in order) before the global write
__global__ __launch_bounds__(256) void k_msd_floor_lds(const uint32_t* __restrict__ act, uint32_t n, uint32_t ntiles,
                                                       uint2* __restrict__ out) {
    __shared__ uint2 stage[kTile];
    const uint32_t t = xcd_tile(blockIdx.x, ntiles);
    uint32_t a[16];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) a[j] = __builtin_nontemporal_load(act + t * kTile + j * 256u + threadIdx.x);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t i = j * 256u + threadIdx.x;
        const uint32_t p = (mix32(i) & (kTile - 1u));  // a scattered LDS position (a permutation is not needed for timing)
        stage[p ^ 0u] = make_uint2(a[j], t * kTile + i);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t i = j * 256u + threadIdx.x;
        const uint2 kv = stage[i];
        const uint32_t d = i / kRun;
        const uint32_t g = d * (ntiles * kRun) + t * kRun + (i % kRun);
        out[g] = make_uint2(kv.x | (d << 10), kv.y);
    }
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_count_floor(const uint2* __restrict__ p, uint32_t n, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kDig];
    for (uint32_t i = threadIdx.x; i < kDig; i += 256) h[i] = 0;
    __syncthreads();
    uint32_t acc = 0;
    const uint32_t base = blockIdx.x * kTile;
#pragma unroll
    for (uint32_t j = 0; j < kTile / 256u; ++j) {
        const uint2 v = ld_nt(p + base + j * 256u + threadIdx.x);
        if (LDS) atomicAdd(&h[v.y & (kDig - 1u)], 1u);  // random low digits: the real count's bank pattern
        else acc += v.x ^ v.y;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kDig; i += 256) hist[(size_t)blockIdx.x * kDig + i] = LDS ? h[i] : acc;
}

// level 2 scatter: bucket = 16 consecutive segments (64K elements, uniform); element i of segment s (low digit k = i / 4)
// goes to bucket_start + k * 64 + s * 4 + i % 4
__global__ __launch_bounds__(256) void k_scatter_floor(const uint2* __restrict__ p, uint32_t n, uint32_t* __restrict__ order) {
    const uint32_t seg = blockIdx.x, bstart = (seg / 16u) * 16u * kTile, s = seg % 16u;
#pragma unroll 4
    for (uint32_t j = 0; j < kTile / 256u; ++j) {
        const uint32_t i = j * 256u + threadIdx.x;
        const uint2 v = ld_nt(p + seg * kTile + i);
        const uint32_t k = v.x & (kDig - 1u);
        order[bstart + k * 64u + s * kRun + (i % kRun)] = v.y;
    }
}

template <int RB, int WB>
__global__ __launch_bounds__(256) void k_stream(const uint32_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ out) {
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        uint32_t x = 0;
        if (RB == 4) x = __builtin_nontemporal_load(in + e);
        if (RB == 8) { const uint2 v = ld_nt(reinterpret_cast<const uint2*>(in) + e); x = v.x ^ v.y; }
        if (WB == 4) out[e] = x;
        if (WB == 8) reinterpret_cast<uint2*>(out)[e] = make_uint2(x, e);
        if (WB == 0 && x == 0x12345679u) out[0] = e;
    }
}

int main() {
    const uint32_t n = 64u << 20, ntiles = n / kTile;
    uint32_t *act, *order, *hist;
    uint2 *pairs, *pairs2;
    CK(hipMalloc(&act, (size_t)n * 4));
    CK(hipMalloc(&order, (size_t)n * 4));
    CK(hipMalloc(&pairs, (size_t)n * 8));
    CK(hipMalloc(&pairs2, (size_t)n * 8));
    CK(hipMalloc(&hist, (size_t)ntiles * kDig * 4));
    hipLaunchKernelGGL(k_fill_act, dim3(8192), dim3(256), 0, 0, act, n);
    hipLaunchKernelGGL(k_fill_pairs, dim3(8192), dim3(256), 0, 0, pairs, n);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto&& launch) {
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
        printf("%-58s %8.1f us  %6.2f TB/s (%.0f B/msg)\n", name, ms * 1e3, bytes / ms / 1e9, bytes / n);
        fflush(stdout);
    };
    const dim3 b(256), gs(8192);
    const size_t occ3 = 50 * 1024, occ3_lds = 18 * 1024;  // 3 x 50 KB <= 160 KB < 4 x 50 KB
    timeit("stream: read 4 B, write 8 B (MSD bytes, contiguous)", 12.0 * n, [&] { hipLaunchKernelGGL((k_stream<4, 8>), gs, b, 0, 0, act, n, reinterpret_cast<uint32_t*>(pairs2)); });
    timeit("msd floor: read act, 8-B runs of 4/digit/tile, linear tiles", 12.0 * n, [&] { hipLaunchKernelGGL(k_msd_floor<false>, dim3(ntiles), b, 0, 0, act, n, ntiles, pairs2); });
    timeit("msd floor: same, XCD-aware tile order", 12.0 * n, [&] { hipLaunchKernelGGL(k_msd_floor<true>, dim3(ntiles), b, 0, 0, act, n, ntiles, pairs2); });
    timeit("msd floor: XCD order, occ3", 12.0 * n, [&] { hipLaunchKernelGGL(k_msd_floor<true>, dim3(ntiles), b, occ3, 0, act, n, ntiles, pairs2); });
    timeit("msd floor + LDS staging image (XCD order)", 12.0 * n, [&] { hipLaunchKernelGGL(k_msd_floor_lds, dim3(ntiles), b, 0, 0, act, n, ntiles, pairs2); });
    timeit("msd floor + LDS staging image (XCD order), occ3", 12.0 * n, [&] { hipLaunchKernelGGL(k_msd_floor_lds, dim3(ntiles), b, occ3_lds, 0, act, n, ntiles, pairs2); });
    timeit("stream: read 8 B (count bytes)", 8.0 * n, [&] { hipLaunchKernelGGL((k_stream<8, 0>), gs, b, 0, 0, reinterpret_cast<uint32_t*>(pairs), n, order); });
    timeit("count floor: read pairs per segment, no LDS", 8.0 * n, [&] { hipLaunchKernelGGL(k_count_floor<false>, dim3(ntiles), b, 0, 0, pairs, n, hist); });
    timeit("count floor + 1 LDS atomic per element (1024 bins)", 8.0 * n, [&] { hipLaunchKernelGGL(k_count_floor<true>, dim3(ntiles), b, 0, 0, pairs, n, hist); });
    timeit("count floor + LDS atomics, occ3", 8.0 * n, [&] { hipLaunchKernelGGL(k_count_floor<true>, dim3(ntiles), b, occ3, 0, pairs, n, hist); });
    timeit("stream: read 8 B, write 4 B (scatter bytes)", 12.0 * n, [&] { hipLaunchKernelGGL((k_stream<8, 4>), gs, b, 0, 0, reinterpret_cast<uint32_t*>(pairs), n, order); });
    timeit("scatter floor: 16-B runs per key per segment", 12.0 * n, [&] { hipLaunchKernelGGL(k_scatter_floor, dim3(ntiles), b, 0, 0, pairs, n, order); });
    timeit("scatter floor, occ3", 12.0 * n, [&] { hipLaunchKernelGGL(k_scatter_floor, dim3(ntiles), b, occ3, 0, pairs, n, order); });
    return 0;
}
