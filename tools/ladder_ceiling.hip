// Verify-kernel arithmetic ceiling on gfx950 (diagnostics): the scalar-multiplication work of one
// p256_verify_kernel lane -- 64 x (4 doublings + 1 mixed addition) + 17 comb mixed additions,
// the same p29_dbl / p29_add_aff_lean code -- on register-resident points: no table build, no
// inversions, no scalar recoding, no table or comb loads, no s^-1, no final check. Same
// occupancy (256-thread workgroups, 4 waves per SIMD) and the same grid as the real kernel for
// a batch of n tuples, so it also carries the same wave quantisation. The real kernel's time
// against this one says how much of it is the ladder's instruction stream itself.
// Usage: ladder_ceiling [n ...]
#include <cstdio>
#include <cstdlib>
#include "../smartbft_amd/csrc/p256_f29.hpp"
using namespace sbft;

// spread = 0: workgroup b takes tuples [256 b, 256 b + 256). spread = 1: the grid is a whole
// number of resident rounds and workgroup b takes tuples [b n / G, (b + 1) n / G) (wave-level
// tail lanes idle): same work, no partial last round.
__global__ __launch_bounds__(256, 4) void ladder_only(uint32_t* out, uint32_t n, int spread) {
    uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (spread) {
        const uint32_t lo = (uint32_t)((uint64_t)blockIdx.x * n / gridDim.x);
        const uint32_t hi = (uint32_t)((uint64_t)(blockIdx.x + 1) * n / gridDim.x);
        gid = lo + threadIdx.x;
        if (lo + (threadIdx.x & ~63u) >= hi) return;  // a wave with no tuple of this block
    }
    jp29 acc;
    f29 x2, y2;
#pragma unroll
    for (int i = 0; i < 9; ++i) {  // limbs in [0, 2^29), limb 8 < 2^24: normal form N
        const uint32_t m = i == 8 ? 0x00FFFFFFu : F29_MASK;
        acc.x.v[i] = (gid * 0x9E3779B1u + 17u * i) & m;
        acc.y.v[i] = (gid * 0x85EBCA77u + 29u * i) & m;
        acc.z.v[i] = (gid * 0xC2B2AE3Du + 31u * i + 1u) & m;
        x2.v[i] = (gid * 0x27D4EB2Fu + 7u * i) & m;
        y2.v[i] = (gid * 0x165667B1u + 3u * i) & m;
    }
#pragma unroll 1
    for (int d = 0; d < 64; ++d) {
#pragma unroll 1
        for (int k = 0; k < 4; ++k) p29_dbl(acc, acc);
        p29_add_aff_lean(acc, x2, y2);
        x2.v[0] ^= (uint32_t)d;  // keep the addend live per step
    }
#pragma unroll 1
    for (int c = 0; c < 17; ++c) {
        p29_add_aff_lean(acc, x2, y2);
        y2.v[1] ^= (uint32_t)c;
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s ^= acc.x.v[i] ^ acc.y.v[i] ^ acc.z.v[i];
    if (gid < n) out[gid] = s;
}

int main(int argc, char** argv) {
    uint32_t* d;
    const uint32_t nmax = 1u << 21;
    if (hipMalloc(&d, nmax * 4) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int k = 1; k < (argc > 1 ? argc : 4); ++k) {
        const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[k], nullptr, 10)
                                    : (k == 1 ? 1000000u : k == 2 ? 1048576u : 786432u);
        if (n == 0 || n > nmax) continue;
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const unsigned g0 = (n + 255) / 256, slots = 4u * (unsigned)cus;  // resident workgroups
        for (int spread = 0; spread < 2; ++spread) {
            const unsigned grid = spread ? (g0 + slots - 1) / slots * slots : g0;
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                (void)hipEventRecord(a);
                hipLaunchKernelGGL(ladder_only, dim3(grid), dim3(256), 0, 0, d, n, spread);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                if (rep && ms < best) best = ms;
            }
            printf("{\"n\": %u, \"spread\": %d, \"grid\": %u, \"ladder_only_ms\": %.3f, \"ladder_only_per_s\": %.1f}\n", n,
                   spread, grid, best, n / best * 1e3);
        }
    }
    (void)hipFree(d);
    return 0;
}
