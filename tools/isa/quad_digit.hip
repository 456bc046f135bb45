// ISA probe (not linked anywhere): one digit of the half kernel's ladders, quad form (q4_*) and
// pair form (p29_*_plw), for instruction counts with tools/isa/count.py.
#include <hip/hip_runtime.h>
#include "../../smartbft_amd/csrc/p256_f29.hpp"
using namespace sbft;

__global__ __launch_bounds__(256) void quad_digit_kernel(u32* io, int L) {
    const int t = threadIdx.x;
    q4w q;
    f29 x2, y2, ut;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        q.xy.v[i] = io[i * 256 + t];
        q.z.v[i] = io[(18 + i) * 256 + t];
        q.w.v[i] = io[(27 + i) * 256 + t];
        q.wm.v[i] = io[(9 + i) * 256 + t];
        x2.v[i] = io[(36 + i) * 256 + t];
        y2.v[i] = io[(45 + i) * 256 + t];
    }
#pragma unroll 1
    for (int d = 0; d < L; ++d) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 3; ++k) q4_dbl<false>(q, x2, ut);
        q4_dbl<true>(q, x2, ut);
        q4_add_rest(q, y2, ut);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        io[i * 256 + t] = q.xy.v[i];
        io[(9 + i) * 256 + t] = q.wm.v[i];
        io[(18 + i) * 256 + t] = q.z.v[i];
        io[(27 + i) * 256 + t] = q.w.v[i];
    }
}

__global__ __launch_bounds__(256) void pair_digit_kernel(u32* io, int L) {
    const int t = threadIdx.x;
    plw29 q;
    f29 x2, y2;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        q.xb.v[i] = io[i * 256 + t];
        q.zy.v[i] = io[(9 + i) * 256 + t];
        q.zo.v[i] = io[(18 + i) * 256 + t];
        q.w.v[i] = io[(27 + i) * 256 + t];
        x2.v[i] = io[(36 + i) * 256 + t];
        y2.v[i] = io[(45 + i) * 256 + t];
    }
#pragma unroll 1
    for (int d = 0; d < L; ++d) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 4; ++k) p29_dbl_plw(q);
        p29_add_aff_plw(q, x2, y2);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        io[i * 256 + t] = q.xb.v[i];
        io[(9 + i) * 256 + t] = q.zy.v[i];
        io[(18 + i) * 256 + t] = q.zo.v[i];
        io[(27 + i) * 256 + t] = q.w.v[i];
    }
}
