// route_pattern_c3.hip — k_route's memory pattern at config 3's size, to place the one-GPU headline's route kernel
// (4.25 ms for 256M messages) against what its loads and stores alone cost:
//   256M 32-B headers streamed, one 8-B probe per message into an 8-B table of 2^25 slots (256 MiB: config 3's 16M
//   grains at load 0.5), 8 B written per message.  The probed key follows Zipf(1.1) over 16M grains (continuous
//   inverse-CDF approximation), each grain at a fixed random slot; "uniform" draws the grain uniformly instead.
//   A second probe for a fraction of the messages stands in for chains that cross into the next line.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/route_pattern_c3 scripts/route_pattern_c3.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using u32x2 = unsigned int __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h;
}

// header i: word 0 = the grain (Zipf or uniform rank), the rest filler
__global__ void k_fill_headers(u32x4* __restrict__ hdr, uint64_t n, uint32_t grains, int zipf) {
    const double a = 1.0 - 1.1;  // 1 - s
    const double tail = 1.0 - pow((double)grains, a);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = mix32((uint32_t)i * 2654435761u + (uint32_t)(i >> 32) * 40503u + 17u);
        uint32_t g;
        if (zipf) {
            const double u = (x + 0.5) / 4294967296.0;
            double r = pow(1.0 - u * tail, 1.0 / a);  // rank in [1, grains]
            g = (uint32_t)fmin(fmax(r, 1.0), (double)grains) - 1u;
        } else {
            g = x % grains;
        }
        hdr[2 * i] = u32x4{g, x, mix32(x + 1u), mix32(x + 2u)};
        hdr[2 * i + 1] = u32x4{mix32(x + 3u), mix32(x + 4u), 0u, (uint32_t)i};
    }
}

__global__ void k_fill_table(u32x2* __restrict__ t, uint64_t slots) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * blockDim.x)
        t[i] = u32x2{mix32((uint32_t)i), (uint32_t)i};
}

// one message per thread and grid-stride step, like k_route: header (non-temporal), hash -> slot, probe, 2 x 4-B out
__global__ __launch_bounds__(256) void k_pattern(const u32x4* __restrict__ hdr, const u32x2* __restrict__ tab, uint32_t mask,
                                                 uint64_t n, uint32_t second_pct, uint32_t* __restrict__ o1,
                                                 uint32_t* __restrict__ o2) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 a = __builtin_nontemporal_load(hdr + 2 * i);
        const u32x4 b = __builtin_nontemporal_load(hdr + 2 * i + 1);
        const uint32_t s = mix32(a.x * 0x9E3779B1u + 12345u) & mask;
        u32x2 v = tab[s];
        if ((mix32(a.x) & 127u) * 100u < second_pct * 128u) {
            const u32x2 w = tab[(s + 8u) & mask];
            v.x ^= w.y;
        }
        o1[i] = v.x ^ a.y;
        o2[i] = v.y ^ b.w;
    }
}

int main(int argc, char** argv) {
    const uint64_t n = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 256ull) << 20;
    const uint32_t grains = 16000000u;
    const uint64_t slots = 1ull << 25;
    u32x4* hdr;
    u32x2* tab;
    uint32_t* out;
    CK(hipMalloc(&hdr, n * 32));
    CK(hipMalloc(&tab, slots * 8));
    CK(hipMalloc(&out, n * 8));
    hipLaunchKernelGGL(k_fill_table, dim3(4096), dim3(256), 0, 0, tab, slots);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto&& launch) {
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
        printf("%-52s %8.3f ms  %7.2f G msgs/s  %6.2f TB/s of 72 B/msg\n", name, ms, n / ms / 1e6, n * 72.0 / ms / 1e9);
        fflush(stdout);
    };
    for (int zipf : {1, 0}) {
        hipLaunchKernelGGL(k_fill_headers, dim3(8192), dim3(256), 0, 0, hdr, n, grains, zipf);
        CK(hipDeviceSynchronize());
        for (uint32_t pct : {0u, 15u}) {
            for (uint32_t grid : {8192u, 65536u}) {
                char nm[96];
                snprintf(nm, sizeof nm, "%s, %u%% 2nd line, grid %u", zipf ? "Zipf(1.1) 16M grains" : "uniform 16M grains", pct, grid);
                timeit(nm, [&] { hipLaunchKernelGGL(k_pattern, dim3(grid), dim3(256), 0, 0, hdr, tab, (uint32_t)(slots - 1), n, pct,
                                                    out, out + n); });
            }
        }
    }
    return 0;
}
