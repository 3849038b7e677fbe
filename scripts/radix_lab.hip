// radix_lab.hip — ablation bench for stage 4's stable radix pass (not part of the product).
// Includes the library's kernel TU so the production kernels and helpers are callable directly, and adds
// experimental forms of the down-sweep.  Keys: 64M uniform in [0, 1M) (config 2's activation handles).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/radix_lab.bin scripts/radix_lab.hip
#include "../orleans_amd/csrc/route_kernels.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace orl {
namespace {

// ITEMS per thread (tile = 256 * ITEMS), STORE: 0 none (one dummy word per tile), 1 SoA keys+idx, 2 AoS {key, idx}
template <int BITS, int ITEMS>
struct LabSmem {
    uint32_t cnt[kWaves][1u << BITS];
    uint32_t delta[1u << BITS];
    uint32_t stage_k[256 * ITEMS];
    uint32_t stage_i[256 * ITEMS];
    uint32_t wsum[kWaves];
};

template <int ITEMS>
__global__ __launch_bounds__(256) void k_lab_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift, uint32_t bins,
                                                  uint32_t* __restrict__ tile_hist) {
    __shared__ uint32_t hist[1u << kMaxDigitBits];
    for (uint32_t b = threadIdx.x; b < bins; b += 256) hist[b] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * 256 * ITEMS;
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t e = base + j * 256 + threadIdx.x;
        if (e < n) atomicAdd(&hist[(keys[e] >> shift) & (bins - 1)], 1u);
    }
    __syncthreads();
    uint32_t* row = tile_hist + (size_t)blockIdx.x * bins;
    for (uint32_t b = threadIdx.x; b < bins; b += 256) row[b] = hist[b];
}

template <int BITS, int ITEMS, int STORE, int IN = 0>
__global__ __launch_bounds__(256) void k_lab_down(const uint32_t* __restrict__ keys_in, uint32_t n, uint32_t shift,
                                                  const uint32_t* __restrict__ tile_off, uint32_t ntiles,
                                                  uint32_t* __restrict__ keys_out, uint32_t* __restrict__ idx_out,
                                                  uint2* __restrict__ pair_out) {
    constexpr uint32_t B = 1u << BITS;
    constexpr uint32_t PER = (B + 255u) / 256u;
    constexpr uint32_t TILE = 256u * ITEMS;
    __shared__ LabSmem<BITS, ITEMS> sm;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, ntiles);
    for (uint32_t b = threadIdx.x; b < B; b += 256) {
#pragma unroll
        for (uint32_t q = 0; q < kWaves; ++q) sm.cnt[q][b] = 0;
    }
    const uint32_t tbase = tile * TILE;
    const uint32_t wbase = tbase + w * (ITEMS * 64u);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64u - lane));
    uint32_t key[ITEMS], rank[ITEMS], idx[ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t e = wbase + j * 64u + lane;
        if (IN == 0) {
            key[j] = e < n ? keys_in[e] : 0u;
            idx[j] = e;
        } else {
            const uint2 v = e < n ? reinterpret_cast<const uint2*>(keys_in)[e] : make_uint2(0u, 0u);
            key[j] = v.x;
            idx[j] = v.y;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t e = wbase + j * 64u + lane;
        const bool valid = e < n;
        const uint32_t d = (key[j] >> shift) & (B - 1u);
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t c = sm.cnt[w][d];
        rank[j] = c + (uint32_t)__popcll(m & lt_mask);
        if (valid && (m >> lane) == 1ull) sm.cnt[w][d] = c + (uint32_t)__popcll(m);
    }
    __syncthreads();
    const uint32_t* orow = tile_off + (size_t)tile * B;
    uint32_t tot[PER];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t b = threadIdx.x * PER + q;
        uint32_t t = 0;
        if (b < B) {
#pragma unroll
            for (uint32_t ww = 0; ww < kWaves; ++ww) {
                const uint32_t c = sm.cnt[ww][b];
                sm.cnt[ww][b] = t;
                t += c;
            }
        }
        tot[q] = t;
        s += t;
    }
    uint32_t total;
    uint32_t run = block_excl_scan(s, sm.wsum, total);
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t b = threadIdx.x * PER + q;
        if (b < B) {
#pragma unroll
            for (uint32_t ww = 0; ww < kWaves; ++ww) sm.cnt[ww][b] += run;
            sm.delta[b] = orow[b] - run;
        }
        run += tot[q];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t e = wbase + j * 64u + lane;
        if (e < n) {
            const uint32_t d = (key[j] >> shift) & (B - 1u);
            const uint32_t lpos = sm.cnt[w][d] + rank[j];
            sm.stage_k[lpos] = key[j];
            sm.stage_i[lpos] = idx[j];
        }
    }
    __syncthreads();
    const uint32_t cnt = (n - tbase) < TILE ? (n - tbase) : TILE;
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t i = j * 256u + threadIdx.x;
        if (i < cnt) {
            const uint32_t k = sm.stage_k[i];
            const uint32_t g = sm.delta[(k >> shift) & (B - 1u)] + i;
            if (STORE == 1) {
                keys_out[g] = k;
                idx_out[g] = sm.stage_i[i];
            } else if (STORE == 2) {
                pair_out[g] = make_uint2(k, sm.stage_i[i]);
            } else {
                acc += g ^ sm.stage_i[i];
            }
        }
    }
    if (STORE == 0 && acc == 0x9E3779B9u) keys_out[tile] = acc;
}

template <int ITEMS>
__global__ __launch_bounds__(256) void k_lab_hist_aos(const uint2* __restrict__ pairs, uint32_t n, uint32_t shift, uint32_t bins,
                                                      uint32_t* __restrict__ tile_hist) {
    __shared__ uint32_t hist[1u << kMaxDigitBits];
    for (uint32_t b = threadIdx.x; b < bins; b += 256) hist[b] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * 256 * ITEMS;
#pragma unroll
    for (uint32_t j = 0; j < ITEMS; ++j) {
        const uint32_t e = base + j * 256 + threadIdx.x;
        if (e < n) atomicAdd(&hist[(pairs[e].x >> shift) & (bins - 1)], 1u);
    }
    __syncthreads();
    uint32_t* row = tile_hist + (size_t)blockIdx.x * bins;
    for (uint32_t b = threadIdx.x; b < bins; b += 256) row[b] = hist[b];
}

// Stores only: the scatter's global write pattern with no ranking (positions from a precomputed permutation-like map)
__global__ __launch_bounds__(256) void k_lab_runs(uint32_t n, uint32_t run, uint32_t* __restrict__ out) {
    // element e goes to bin b = (e / run) % 1024 within its tile; emulate runs of `run` elements per bin per tile
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    const uint32_t tile = e / 4096, within = e % 4096;
    const uint32_t bin = within / run, r = within % run;
    const uint32_t bins = 4096 / run;
    const uint32_t ntiles = n / 4096;
    out[(size_t)bin * ntiles * run + (size_t)tile * run + r] = e;
}

}  // namespace
}  // namespace orl

using namespace orl;

int main() {
    const uint32_t n = 64u << 20, n_act = 1000000;
    std::vector<uint32_t> hk(n);
    uint64_t x = 0x5EED0002;
    for (uint32_t i = 0; i < n; ++i) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        hk[i] = (uint32_t)(z % n_act);
    }
    uint32_t *keys, *ko, *io, *hist, *hist2;
    uint2* po;
    CK(hipMalloc(&keys, n * 4ull));
    CK(hipMalloc(&ko, n * 4ull));
    CK(hipMalloc(&io, n * 4ull));
    CK(hipMalloc(&po, n * 8ull));
    const uint32_t max_tiles = n / 1024;
    CK(hipMalloc(&hist, (size_t)max_tiles * 2048 * 4));
    CK(hipMalloc(&hist2, (size_t)max_tiles * 2048 * 4));
    Scratch s{};
    CK(hipMalloc(&s.col_sums, (size_t)(max_tiles / 64 + 1) * 2048 * 4));
    CK(hipMalloc(&s.col_tot, 2048 * 4));
    CK(hipMemcpy(keys, hk.data(), n * 4ull, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto&& launch) {
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
        printf("%-44s %8.3f ms  %8.1f GB/s  %7.2f G keys/s\n", name, ms, bytes / ms / 1e6, n / ms / 1e6);
    };
    const hipStream_t st = 0;
    auto prep = [&](int bits, uint32_t tile) {
        const uint32_t nt = n / tile;
        const uint32_t bins = 1u << bits;
        if (tile == 4096) hipLaunchKernelGGL(k_lab_hist<16>, dim3(nt), dim3(256), 0, st, keys, n, 0u, bins, hist);
        else if (tile == 8192) hipLaunchKernelGGL(k_lab_hist<32>, dim3(nt), dim3(256), 0, st, keys, n, 0u, bins, hist);
        else hipLaunchKernelGGL(k_lab_hist<8>, dim3(nt), dim3(256), 0, st, keys, n, 0u, bins, hist);
        col_scan(hist, nt, bins, s, st);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hist2, hist, (size_t)nt * bins * 4, hipMemcpyDeviceToDevice));
    };
    timeit("hist 4096 tiles, 1024 bins", 4.0 * n, [&] {
        hipLaunchKernelGGL(k_lab_hist<16>, dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, 1024u, hist);
    });
    timeit("col_scan 16384 x 1024", 4.0 * 2 * 16384 * 1024 * 2, [&] { col_scan(hist, n / 4096, 1024, s, st); });
    prep(10, 4096);
    timeit("prod k_radix_pass<10,act,pair>", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_radix_pass<10, IN_ACT, OUT_PAIR>), dim3(n / 4096), dim3(256), 0, st, keys, n, n_act, 0u, hist2, n / 4096, po, ko, io);
    });
    timeit("lab down 10b tile4096 STORE=0 (no stores)", 4.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 16, 0>), dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, hist2, n / 4096, ko, io, po);
    });
    timeit("lab down 10b tile4096 STORE=1 (SoA)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 16, 1>), dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, hist2, n / 4096, ko, io, po);
    });
    timeit("lab down 10b tile4096 STORE=2 (AoS)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 16, 2>), dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, hist2, n / 4096, ko, io, po);
    });
    prep(10, 8192);
    timeit("lab down 10b tile8192 STORE=1 (SoA)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 32, 1>), dim3(n / 8192), dim3(256), 0, st, keys, n, 0u, hist2, n / 8192, ko, io, po);
    });
    timeit("lab down 10b tile8192 STORE=2 (AoS)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 32, 2>), dim3(n / 8192), dim3(256), 0, st, keys, n, 0u, hist2, n / 8192, ko, io, po);
    });
    timeit("lab down 10b tile8192 STORE=0", 4.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 32, 0>), dim3(n / 8192), dim3(256), 0, st, keys, n, 0u, hist2, n / 8192, ko, io, po);
    });
    prep(7, 4096);
    timeit("lab down 7b tile4096 STORE=1 (SoA)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<7, 16, 1>), dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, hist2, n / 4096, ko, io, po);
    });
    timeit("lab down 7b tile4096 STORE=2 (AoS)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<7, 16, 2>), dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, hist2, n / 4096, ko, io, po);
    });
    prep(8, 4096);
    timeit("lab down 8b tile4096 STORE=1 (SoA)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<8, 16, 1>), dim3(n / 4096), dim3(256), 0, st, keys, n, 0u, hist2, n / 4096, ko, io, po);
    });
    prep(10, 2048);
    timeit("lab down 10b tile2048 STORE=1 (SoA)", 12.0 * n, [&] {
        hipLaunchKernelGGL((k_lab_down<10, 8, 1>), dim3(n / 2048), dim3(256), 0, st, keys, n, 0u, hist2, n / 2048, ko, io, po);
    });
    {
        // full stage-4 pipelines after the route kernel (its fused histogram of digit 0 is not timed)
        uint2* pa;
        uint2* pb;
        CK(hipMalloc(&pa, n * 8ull));
        CK(hipMalloc(&pb, n * 8ull));
        uint32_t* offs;
        CK(hipMalloc(&offs, (n_act + 2) * 4ull));
        const uint32_t nt = n / 4096;
        auto pipeline = [&](std::vector<int> bits) {
            int shift = 0;
            const int P = (int)bits.size();
            for (int p = 0; p < P; ++p) {
                const uint32_t bins = 1u << bits[p];
                if (p == 0) {
                    // route kernel already produced this histogram; recompute outside the timed region is not possible
                    // here, so it is produced by k_lab_hist and accounted separately below
                } else {
                    hipLaunchKernelGGL(k_lab_hist_aos<16>, dim3(nt), dim3(256), 0, st, (p % 2) ? pa : pb, n, (uint32_t)shift, bins, hist);
                }
                col_scan(hist, nt, bins, s, st);
                const bool last = p == P - 1;
                uint2* pin = (p % 2) ? pa : pb;
                uint2* pout = (p % 2) ? pb : pa;
#define LAB(BB) \
    if (p == 0 && !last) hipLaunchKernelGGL((k_lab_down<BB, 16, 2, 0>), dim3(nt), dim3(256), 0, st, keys, n, (uint32_t)shift, hist, nt, ko, io, pout); \
    else if (!last) hipLaunchKernelGGL((k_lab_down<BB, 16, 2, 1>), dim3(nt), dim3(256), 0, st, (const uint32_t*)pin, n, (uint32_t)shift, hist, nt, ko, io, pout); \
    else hipLaunchKernelGGL((k_lab_down<BB, 16, 1, 1>), dim3(nt), dim3(256), 0, st, (const uint32_t*)pin, n, (uint32_t)shift, hist, nt, ko, io, pout);
                if (bits[p] == 10) { LAB(10) } else if (bits[p] == 7) { LAB(7) } else if (bits[p] == 6) { LAB(6) } else if (bits[p] == 8) { LAB(8) } else { LAB(4) }
#undef LAB
                shift += bits[p];
            }
            { (void)hipMemsetD32Async((hipDeviceptr_t)offs, kNoOffset, n_act + 2, st);
              hipLaunchKernelGGL(k_offsets_mark, dim3((n / 16 + 255) / 256), dim3(256), 0, st, ko, n, n_act + 2, offs);
              hipLaunchKernelGGL(k_offsets_fill, dim3((n_act + 2 + 255) / 256), dim3(256), 0, st, ko, n, n_act + 2, offs); }
        };
        timeit("pipeline 10+10 (AoS mid) excl. hist0", 28.0 * n, [&] {
            hipLaunchKernelGGL(k_lab_hist<16>, dim3(nt), dim3(256), 0, st, keys, n, 0u, 1024u, hist);
            pipeline({10, 10});
        });
        timeit("pipeline 7+7+6 (AoS mid) excl. hist0", 44.0 * n, [&] {
            hipLaunchKernelGGL(k_lab_hist<16>, dim3(nt), dim3(256), 0, st, keys, n, 0u, 128u, hist);
            pipeline({7, 7, 6});
        });
        timeit("pipeline 8+8+4 (AoS mid) excl. hist0", 44.0 * n, [&] {
            hipLaunchKernelGGL(k_lab_hist<16>, dim3(nt), dim3(256), 0, st, keys, n, 0u, 256u, hist);
            pipeline({8, 8, 4});
        });
        timeit("k_offsets", 4.0 * n, [&] {
            { (void)hipMemsetD32Async((hipDeviceptr_t)offs, kNoOffset, n_act + 2, st);
              hipLaunchKernelGGL(k_offsets_mark, dim3((n / 16 + 255) / 256), dim3(256), 0, st, ko, n, n_act + 2, offs);
              hipLaunchKernelGGL(k_offsets_fill, dim3((n_act + 2 + 255) / 256), dim3(256), 0, st, ko, n, n_act + 2, offs); }
        });
        prep(10, 4096);
        timeit("prod k_radix_pass<10,act,pair> again", 12.0 * n, [&] {
            hipLaunchKernelGGL((k_radix_pass<10, IN_ACT, OUT_PAIR>), dim3(n / 4096), dim3(256), 0, st, keys, n, n_act, 0u, hist2, n / 4096, po, ko, io);
        });
    }
    for (uint32_t run : {1u, 4u, 16u, 64u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "store runs of %u x 4 B", run);
        timeit(nm, 4.0 * n, [&] { hipLaunchKernelGGL(k_lab_runs, dim3(n / 256), dim3(256), 0, st, n, run, ko); });
    }
    return 0;
}
