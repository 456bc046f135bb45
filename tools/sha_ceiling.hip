// SHA-256 compute ceiling on gfx950 (diagnostics): the compression of sha256_dev.hpp run on
// register-resident blocks (no memory traffic; each block's words are derived from the state,
// so nothing can be hoisted), M independent messages per lane interleaved (compress_multi, as
// sha256_lds_kernel uses it), at the occupancy the register count allows. Reports payload
// GB/s (64 B per lane-block): the ceiling any SHA-256 kernel with this instruction stream can
// reach, against which the real kernel's GB/s is compared.
#include <cstdio>
#include <cstdlib>
#include "../smartbft_amd/csrc/sha256_dev.hpp"
using namespace sbft;

template <int M>
__global__ __launch_bounds__(256) void reg_ceiling(uint32_t* out, int blocks) {
    uint32_t h[M][8], w[M][16];
    bool live[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        live[m] = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) h[m][i] = threadIdx.x * 8 + i + m;
    }
    for (int b = 0; b < blocks; ++b) {
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
            for (int i = 0; i < 16; ++i) w[m][i] = h[m][i & 7] ^ (uint32_t)(b * 16 + i);
        compress_multi<M>(h, w, live);
    }
    uint32_t x = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) x ^= h[m][0] ^ h[m][7];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int M>
static void run(int cus) {
    const int blocks = 64, grid = cus * 16;
    uint32_t* d;
    hipMalloc(&d, (size_t)grid * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(reg_ceiling<M>, dim3(grid), dim3(256), 0, 0, d, blocks);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;
    }
    const double bytes = (double)grid * 256 * M * blocks * 64;
    printf("M=%d messages/lane: %.3f ms  %.1f GB/s register-resident SHA-256 (payload bytes)\n", M, best,
           bytes / best / 1e6);
    hipFree(d);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<1>(cus);
    run<2>(cus);
    return 0;
}
