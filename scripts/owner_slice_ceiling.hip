// owner_slice_ceiling.hip — what an XCD-sliced probe table would buy the OWNER of config 3 at 8 ranks (the hot rank:
// 54.8M received 8-B records, 29.5M of them for the Zipf-hot grain, the rest uniform over its ~2M grains; its 8-B probe
// table has 2^22 slots = 32 MiB, i.e. 4 MiB per XCD slice = one XCD's L2).  The memory pattern of the owner's route
// (8-B record in, one 8-B probe, 8 B out), three layouts:
//   A. arrival order (today): every workgroup probes the whole table;
//   B. records grouped by slice (what a (rank, slice) partition at the sender would deliver), workgroup b on XCD b % 8
//      routing slice b % 8, the hot grain's slice routed by every XCD (its one hot line is in every L2);
//   C. the same grouping, but each slice routed only by its XCD (the hot slice's XCD does 60 % of the work);
//   plus the ungrouped pattern's probe-free floor (stream 8 B in, 8 B out).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/owner_slice_ceiling scripts/owner_slice_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using u32x2 = unsigned int __attribute__((ext_vector_type(2)));

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h;
}

constexpr uint32_t kLog2Slots = 22, kSlots = 1u << kLog2Slots;

__device__ __forceinline__ void route_one(const u32x2* __restrict__ rec, const u32x2* __restrict__ tab, uint32_t i,
                                          uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    const u32x2 r = __builtin_nontemporal_load(rec + i);
    const uint32_t s = mix32(r.x) & (kSlots - 1u);
    const u32x2 v = tab[s];
    o1[i] = v.x ^ r.y;
    o2[i] = v.y;
}

// A: contiguous ranges, 4 records per thread per step
__global__ __launch_bounds__(256) void k_plain(const u32x2* __restrict__ rec, const u32x2* __restrict__ tab, uint32_t n,
                                               uint32_t* __restrict__ o1, uint32_t* __restrict__ o2) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) route_one(rec, tab, i, o1, o2);
}

// probe-free floor
__global__ __launch_bounds__(256) void k_stream(const u32x2* __restrict__ rec, uint32_t n, uint32_t* __restrict__ o1,
                                                uint32_t* __restrict__ o2) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const u32x2 r = __builtin_nontemporal_load(rec + i);
        o1[i] = r.x ^ 0x55u;
        o2[i] = r.y;
    }
}

// B / C: seg[q] = {begin, end} of the records workgroup group q routes; workgroup b takes group (b % 8) of XCD b % 8's list:
// list x = segs[x * per_x .. ), workgroups of XCD x stride over it.  SPREAD: the lists were built so every XCD gets an
// equal share (the hot slice cut across all of them); else each XCD gets exactly its slice.
__global__ __launch_bounds__(256) void k_sliced(const u32x2* __restrict__ rec, const u32x2* __restrict__ tab,
                                                const uint2* __restrict__ xrange, uint32_t* __restrict__ o1,
                                                uint32_t* __restrict__ o2) {
    const uint32_t x = blockIdx.x % 8u, j = blockIdx.x / 8u, nj = gridDim.x / 8u;
    // xrange[x * 2 + k]: up to two contiguous ranges per XCD (its own slice part, and a cut of the hot slice)
    for (uint32_t k = 0; k < 2; ++k) {
        const uint2 r = xrange[x * 2 + k];
        for (uint32_t i = r.x + j * 256u + threadIdx.x; i < r.y; i += nj * 256u) route_one(rec, tab, i, o1, o2);
    }
}

int main() {
    const uint32_t n = 57462374u;         // 54.8M records
    const uint32_t n_hot = 31 * (n / 57);  // ~29.5M (54 %) for one grain
    const uint32_t n_grains = 1971059u;
    // records: key = grain id (hot grain = 751170), meta = i
    std::vector<uint32_t> key(n);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    auto rnd = [&] { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (uint32_t)st; };
    const uint32_t hot_key = 751170u;
    for (uint32_t i = 0; i < n; ++i) key[i] = (rnd() % n) < n_hot ? hot_key : rnd() % n_grains;
    auto slice_of = [](uint32_t k) { return (mix32(k) & (kSlots - 1u)) >> (kLog2Slots - 3); };
    std::vector<u32x2> rec_a(n), rec_b;
    for (uint32_t i = 0; i < n; ++i) rec_a[i] = u32x2{key[i], i};
    // grouped by slice, stable
    std::vector<uint32_t> cnt(8, 0);
    for (uint32_t i = 0; i < n; ++i) cnt[slice_of(key[i])]++;
    std::vector<uint32_t> beg(9, 0);
    for (int s = 0; s < 8; ++s) beg[s + 1] = beg[s] + cnt[s];
    rec_b.resize(n);
    {
        std::vector<uint32_t> pos(beg.begin(), beg.end() - 1);
        for (uint32_t i = 0; i < n; ++i) rec_b[pos[slice_of(key[i])]++] = rec_a[i];
    }
    const uint32_t hs = slice_of(hot_key);
    printf("slices (M records):");
    for (int s = 0; s < 8; ++s) printf(" %.1f%s", cnt[s] / 1048576.0, s == (int)hs ? "*" : "");
    printf("\n");
    // C: XCD x gets slice x.  B: XCD x gets slice x (x != hs) and an equal cut of the hot slice so totals match
    std::vector<uint2> xr_c(16), xr_b(16);
    for (int x = 0; x < 8; ++x) {
        xr_c[2 * x] = make_uint2(beg[x], beg[x + 1]);
        xr_c[2 * x + 1] = make_uint2(0, 0);
    }
    {
        const uint64_t target = (n + 7) / 8;
        uint32_t cur = beg[hs];
        for (int x = 0; x < 8; ++x) {
            const uint32_t own = x == (int)hs ? 0u : cnt[x];
            const uint32_t take = (uint32_t)std::min<uint64_t>(target > own ? target - own : 0, beg[hs + 1] - cur);
            xr_b[2 * x] = x == (int)hs ? make_uint2(0, 0) : make_uint2(beg[x], beg[x + 1]);
            xr_b[2 * x + 1] = make_uint2(cur, cur + (x == 7 ? beg[hs + 1] - cur : take));
            cur += take;
        }
    }
    u32x2 *d_tab, *d_a, *d_b;
    uint32_t *o1, *o2;
    uint2 *d_xb, *d_xc;
    CK(hipMalloc(&d_tab, (size_t)kSlots * 8));
    CK(hipMalloc(&d_a, (size_t)n * 8));
    CK(hipMalloc(&d_b, (size_t)n * 8));
    CK(hipMalloc(&o1, (size_t)n * 4));
    CK(hipMalloc(&o2, (size_t)n * 4));
    CK(hipMalloc(&d_xb, 16 * sizeof(uint2)));
    CK(hipMalloc(&d_xc, 16 * sizeof(uint2)));
    {
        std::vector<u32x2> tab(kSlots);
        for (uint32_t s = 0; s < kSlots; ++s) tab[s] = u32x2{mix32(s + 1), mix32(s + 7)};
        CK(hipMemcpy(d_tab, tab.data(), (size_t)kSlots * 8, hipMemcpyHostToDevice));
    }
    CK(hipMemcpy(d_a, rec_a.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_b, rec_b.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_xb, xr_b.data(), 16 * sizeof(uint2), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_xc, xr_c.data(), 16 * sizeof(uint2), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto&& launch) {
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
        printf("%-72s %8.1f us  %7.1f G rec/s\n", name, ms * 1e3, (double)n / ms / 1e6);
        fflush(stdout);
    };
    const dim3 b(256);
    for (uint32_t g : {4096u, 8192u, 16384u}) {
        char nm[128];
        snprintf(nm, sizeof nm, "A  arrival order, whole 32 MiB table (grid %u)", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_plain, dim3(g), b, 0, 0, d_a, d_tab, n, o1, o2); });
        snprintf(nm, sizeof nm, "B  grouped by slice, own-XCD slices, hot slice spread (grid %u)", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_sliced, dim3(g), b, 0, 0, d_b, d_tab, d_xb, o1, o2); });
        snprintf(nm, sizeof nm, "C  grouped by slice, own-XCD slices only (grid %u)", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_sliced, dim3(g), b, 0, 0, d_b, d_tab, d_xc, o1, o2); });
        snprintf(nm, sizeof nm, "   grouped by slice, every XCD probes every slice (control, grid %u)", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_plain, dim3(g), b, 0, 0, d_b, d_tab, n, o1, o2); });
        snprintf(nm, sizeof nm, "   floor: stream 8 B in, 8 B out, no probe (grid %u)", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_stream, dim3(g), b, 0, 0, d_a, n, o1, o2); });
    }
    return 0;
}
