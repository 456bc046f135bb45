// Timing probe (not linked anywhere): the half kernel's ladder digit alone, at the latency
// kernels' occupancy (one wavefront per SIMD: 256-thread workgroups, one per CU), quad form
// (q4_*: the wide kernel) and pair form (p29_*_plw: the four-lane kernel). Prints shader-clock
// cycles per digit of wave 0 and the launch time, so field-arithmetic variants (-D switches of
// p256_f29.hpp) can be compared without the whole kernel.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=1000000 \
//        [-DSBFT_...] -o tools/isa/digit_bench tools/isa/digit_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../smartbft_amd/csrc/p256_f29.hpp"
using namespace sbft;

__global__ __launch_bounds__(256) void quad_digits(u32* io, unsigned long long* clk, int L) {
    const int t = threadIdx.x;
    u32* b = io + (size_t)blockIdx.x * 54 * 256;
    q4w q;
    f29 x2, y2, ut;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        q.xy.v[i] = b[i * 256 + t];
        q.wm.v[i] = b[(9 + i) * 256 + t];
        q.z.v[i] = b[(18 + i) * 256 + t];
        q.w.v[i] = b[(27 + i) * 256 + t];
        x2.v[i] = b[(36 + i) * 256 + t];
        y2.v[i] = b[(45 + i) * 256 + t];
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int d = 0; d < L; ++d) {
        __builtin_amdgcn_sched_barrier(0);
#ifdef ROLLED_DBL  // the three plain doublings as a loop: ~2.3k instead of ~3.9k instructions of loop body
#pragma unroll 1
#else
#pragma unroll
#endif
        for (int k = 0; k < 3; ++k) q4_dbl<false>(q, x2, ut);
        q4_dbl<true>(q, x2, ut);
        q4_add_rest(q, y2, ut);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (t == 0 && blockIdx.x == 0) clk[0] = c1 - c0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        b[i * 256 + t] = q.xy.v[i];
        b[(9 + i) * 256 + t] = q.wm.v[i];
        b[(18 + i) * 256 + t] = q.z.v[i];
        b[(27 + i) * 256 + t] = q.w.v[i];
    }
}

__global__ __launch_bounds__(256) void pair_digits(u32* io, unsigned long long* clk, int L) {
    const int t = threadIdx.x;
    u32* b = io + (size_t)blockIdx.x * 54 * 256;
    plw29 q;
    f29 x2, y2;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        q.xb.v[i] = b[i * 256 + t];
        q.zy.v[i] = b[(9 + i) * 256 + t];
        q.zo.v[i] = b[(18 + i) * 256 + t];
        q.w.v[i] = b[(27 + i) * 256 + t];
        x2.v[i] = b[(36 + i) * 256 + t];
        y2.v[i] = b[(45 + i) * 256 + t];
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int d = 0; d < L; ++d) {
        __builtin_amdgcn_sched_barrier(0);
#ifdef ROLLED_DBL
#pragma unroll 1
#else
#pragma unroll
#endif
        for (int k = 0; k < 4; ++k) p29_dbl_plw(q);
        p29_add_aff_plw(q, x2, y2);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    if (t == 0 && blockIdx.x == 0) clk[1] = c1 - c0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        b[i * 256 + t] = q.xb.v[i];
        b[(9 + i) * 256 + t] = q.zy.v[i];
        b[(18 + i) * 256 + t] = q.zo.v[i];
        b[(27 + i) * 256 + t] = q.w.v[i];
    }
}

int main(int argc, char** argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 256;
    const int G = argc > 2 ? atoi(argv[2]) : 256;  // workgroups: one per CU
    const size_t words = (size_t)G * 54 * 256;
    u32* h = (u32*)malloc(words * 4);
    unsigned s = 12345;
    for (size_t i = 0; i < words; ++i) {  // limbs below 2^28: valid operands for every contract
        s = s * 1103515245u + 12345u;
        h[i] = (s >> 4) & 0x0fffffffu;
    }
    u32* io;
    unsigned long long* clk;
    if (hipMalloc(&io, words * 4) || hipMalloc(&clk, 16)) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* name[2] = {"quad", "pair"};
    for (int k = 0; k < 2; ++k) {
        float best = 1e30f;
        unsigned long long cbest = ~0ull;
        for (int rep = 0; rep < 6; ++rep) {
            if (hipMemcpy(io, h, words * 4, hipMemcpyHostToDevice)) return 1;
            (void)hipEventRecord(e0, 0);
            if (k == 0) hipLaunchKernelGGL(quad_digits, dim3(G), dim3(256), 0, 0, io, clk, L);
            else hipLaunchKernelGGL(pair_digits, dim3(G), dim3(256), 0, 0, io, clk, L);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1)) return 2;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c[2];
            if (hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost)) return 2;
            if (rep > 0 && ms < best) best = ms;
            if (rep > 0 && c[k] < cbest) cbest = c[k];
        }
        // s_memtime counts at a fixed 100 MHz on gfx950? No: the shader clock; report both
        printf("%s L=%d G=%d: %.1f us per launch, %.3f us per digit, memtime %llu per launch, %.1f per digit\n",
               name[k], L, G, best * 1e3, best * 1e3 / L, cbest, (double)cbest / L);
    }
    return 0;
}
