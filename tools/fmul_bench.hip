// Microbenchmark: fp_mul / fp_sqr / fn_mul throughput vs occupancy (waves per SIMD), to
// calibrate the verify kernel's design (how many waves hide the madc dependency chains).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../smartbft_amd/csrc/p256_field.hpp"
using namespace sbft;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

template <int OP, int CHAINS>
__global__ __launch_bounds__(256) void k(u32* out, int iters) {
    fe x[CHAINS], y;
    for (int c = 0; c < CHAINS; ++c)
        for (int i = 0; i < 8; ++i) x[c].v[i] = threadIdx.x * 77 + i * 13 + blockIdx.x + c;
    for (int i = 0; i < 8; ++i) y.v[i] = threadIdx.x ^ (i * 0x9e3779b9u);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (OP == 0) fp_mul(x[c], x[c], y);
            else if (OP == 1) fp_sqr(x[c], x[c]);
            else fn_mul(x[c], x[c], y);
        }
    }
    u32 s = 0;
    for (int c = 0; c < CHAINS; ++c) for (int i = 0; i < 8; ++i) s ^= x[c].v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    u32* d;
    CHK(hipMalloc(&d, 256 * 64 * 256 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const int iters = 2000;
    auto run = [&](auto kern, const char* name, int chains) -> int {
        for (int wps : {1, 2, 4, 8}) {
            int blocks = 256 * wps;  // 256-thread blocks = 4 waves = 1 wave per SIMD per block
            kern<<<blocks, 256>>>(d, 10);
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0));
            kern<<<blocks, 256>>>(d, iters);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            double ops = (double)blocks * 256 * iters * chains;
            printf("%-8s chains=%d waves/SIMD=%d  %.3f ms  %.2f G ops/s\n", name, chains, wps, ms, ops / ms / 1e6);
        }
        return 0;
    };
    run(k<0, 1>, "fp_mul", 1);
    run(k<0, 2>, "fp_mul", 2);
    run(k<1, 1>, "fp_sqr", 1);
    run(k<1, 2>, "fp_sqr", 2);
    run(k<2, 1>, "fn_mul", 1);
    return 0;
}
