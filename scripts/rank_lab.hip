// rank_lab.hip — stable in-tile ranking alternatives for stage 4's radix passes (lab, not the product).
// Each variant writes, for every element, its rank among the equal-digit elements of its wave's 1024-element
// stripe (wave w of a 4096-element tile owns elements [w*1024, w*1024+1024) in 16 steps of 64 lanes).
//   ballot  : the production method (BITS ballots per step, per-wave running counts in LDS)
//   atomic  : one returning LDS atomic per lane (ds_add_rtn_u32) on the per-wave counter; stable only if
//             same-address lanes of one instruction are serviced in lane order
//   leader  : BITS ballots, then ONE returning atomic per equal-digit group (its lowest lane), broadcast
//             with ds_bpermute; the 16 steps' atomics are independent so they pipeline
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/rank_lab.bin scripts/rank_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr uint32_t kItems = 16;

template <int BITS, int MODE>
__global__ __launch_bounds__(256) void k_rank(const uint32_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ rank_out) {
    constexpr uint32_t B = 1u << BITS;
    __shared__ uint32_t cnt[4][B];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    for (uint32_t b = threadIdx.x; b < B; b += 256)
        for (int q = 0; q < 4; ++q) cnt[q][b] = 0;
    const uint32_t wbase = blockIdx.x * 4096u + w * 1024u;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
    uint32_t key[kItems], rank[kItems];
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) key[j] = keys[wbase + j * 64u + lane] & (B - 1u);
    __syncthreads();
    if (MODE == 0) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) {
            const uint32_t d = key[j];
            uint64_t m = ~0ull;
#pragma unroll
            for (int b = 0; b < BITS; ++b) {
                const uint64_t bb = __ballot((d >> b) & 1u);
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t c = cnt[w][d];
            rank[j] = c + (uint32_t)__popcll(m & lt_mask);
            if ((m >> lane) == 1ull) cnt[w][d] = c + (uint32_t)__popcll(m);
        }
    } else if (MODE == 1) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) rank[j] = atomicAdd(&cnt[w][key[j]], 1u);
    } else {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) {
            const uint32_t d = key[j];
            uint64_t m = ~0ull;
#pragma unroll
            for (int b = 0; b < BITS; ++b) {
                const uint64_t bb = __ballot((d >> b) & 1u);
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
            uint32_t old = 0;
            if (lane == leader) old = atomicAdd(&cnt[w][d], (uint32_t)__popcll(m));
            old = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(leader << 2), (int)old);
            rank[j] = old + (uint32_t)__popcll(m & lt_mask);
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) rank_out[wbase + j * 64u + lane] = rank[j];
}

static uint64_t splitmix(uint64_t& x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    const uint32_t n = 64u << 20;
    std::vector<uint32_t> hk(n), r0(n), r1(n);
    uint32_t *keys, *ro;
    CK(hipMalloc(&keys, n * 4ull));
    CK(hipMalloc(&ro, n * 4ull));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto&& launch) {
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
        printf("%-40s %8.3f ms  %7.2f G keys/s\n", name, ms, n / ms / 1e6);
    };
    const char* dists[] = {"uniform", "zipf-ish (8 hot digits 50%)", "all-equal", "4 distinct"};
    for (int dist = 0; dist < 4; ++dist) {
        uint64_t x = 0x5EED0002 + dist;
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t z = splitmix(x);
            uint32_t k = (uint32_t)(z % 1000000u);
            if (dist == 1 && (z >> 40) % 2 == 0) k = (uint32_t)((z >> 20) % 8u) * 977u;
            if (dist == 2) k = 12345u;
            if (dist == 3) k = (uint32_t)((z >> 20) % 4u);
            hk[i] = k;
        }
        CK(hipMemcpy(keys, hk.data(), n * 4ull, hipMemcpyHostToDevice));
        printf("-- keys: %s\n", dists[dist]);
        for (int bits : {10, 8}) {
            char nm[96];
            auto run = [&](int mode) {
                const dim3 g(n / 4096), b(256);
                if (bits == 10) {
                    if (mode == 0) hipLaunchKernelGGL((k_rank<10, 0>), g, b, 0, 0, keys, n, ro);
                    if (mode == 1) hipLaunchKernelGGL((k_rank<10, 1>), g, b, 0, 0, keys, n, ro);
                    if (mode == 2) hipLaunchKernelGGL((k_rank<10, 2>), g, b, 0, 0, keys, n, ro);
                } else {
                    if (mode == 0) hipLaunchKernelGGL((k_rank<8, 0>), g, b, 0, 0, keys, n, ro);
                    if (mode == 1) hipLaunchKernelGGL((k_rank<8, 1>), g, b, 0, 0, keys, n, ro);
                    if (mode == 2) hipLaunchKernelGGL((k_rank<8, 2>), g, b, 0, 0, keys, n, ro);
                }
            };
            const char* mn[] = {"ballot", "atomic", "leader"};
            for (int mode = 0; mode < 3; ++mode) {
                snprintf(nm, sizeof nm, "%d-bit %s", bits, mn[mode]);
                timeit(nm, [&] { run(mode); });
                CK(hipMemcpy(mode == 0 ? r0.data() : r1.data(), ro, n * 4ull, hipMemcpyDeviceToHost));
                if (mode > 0) {
                    size_t bad = 0, first = 0;
                    for (uint32_t i = 0; i < n; ++i)
                        if (r0[i] != r1[i] && bad++ == 0) first = i;
                    printf("   %s vs ballot: %zu mismatches%s", mn[mode], bad, bad ? "" : "\n");
                    if (bad) printf(" (first at %zu: %u vs %u)\n", first, r1[first], r0[first]);
                }
            }
        }
    }
    return 0;
}
