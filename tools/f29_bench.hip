// Microbenchmark + correctness dump: radix-2^29 field ops (p256_f29.hpp) against the 8x32 ones.
// Usage: f29_bench <dump.bin>   (tools/f29_check.py verifies the dump with Python big ints)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../smartbft_amd/csrc/p256_f29.hpp"
using namespace sbft;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

template <int OP, int CHAINS>
__global__ __launch_bounds__(256) void kbench(u32* out, int iters) {
    f29 x[CHAINS], y;
    fe xx[CHAINS], yy;
    for (int c = 0; c < CHAINS; ++c)
        for (int i = 0; i < 9; ++i) x[c].v[i] = (threadIdx.x * 77 + i * 13 + blockIdx.x + c) & F29_MASK;
    for (int i = 0; i < 9; ++i) y.v[i] = (threadIdx.x ^ (i * 0x9e3779b9u)) & F29_MASK;
    for (int c = 0; c < CHAINS; ++c)
        for (int i = 0; i < 8; ++i) xx[c].v[i] = threadIdx.x * 77 + i * 13 + blockIdx.x + c;
    for (int i = 0; i < 8; ++i) yy.v[i] = threadIdx.x ^ (i * 0x9e3779b9u);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (OP == 0) f29_mul(x[c], x[c], y);
            else if (OP == 1) f29_sqr(x[c], x[c]);
            else if (OP == 2) fp_mul(xx[c], xx[c], yy);
            else fp_sqr(xx[c], xx[c]);
        }
    }
    u32 s = 0;
    for (int c = 0; c < CHAINS; ++c) for (int i = 0; i < 9; ++i) s ^= x[c].v[i];
    for (int c = 0; c < CHAINS; ++c) for (int i = 0; i < 8; ++i) s ^= xx[c].v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// in: n x (a[8], b[8]) plain u256 < p. out: n x (mul[9], sqr[9], add-chain[9]) raw f29 limbs.
__global__ void kcheck(const u32* in, u32* out, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    fe a, b;
    for (int i = 0; i < 8; ++i) { a.v[i] = in[16 * t + i]; b.v[i] = in[16 * t + 8 + i]; }
    f29 fa = f29_from_u256(a), fb = f29_from_u256(b), m, s, d, e;
    f29_mul(m, fa, fb);
    f29_sqr(s, fa);
    // worst-case-ish bounds: (a - b) * 3(a + b) after one carry pass
    f29_sub(d, m, s);
    f29_add(e, m, s);
    f29_normalize(e, e);
    f29_muls(e, e, 3);
    f29_mul(d, d, e);
    for (int i = 0; i < 9; ++i) { out[27 * t + i] = m.v[i]; out[27 * t + 9 + i] = s.v[i]; out[27 * t + 18 + i] = d.v[i]; }
}

int main(int argc, char** argv) {
    u32* d;
    CHK(hipMalloc(&d, 256 * 64 * 256 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const int iters = 2000;
    auto run = [&](auto kern, const char* name, int chains) -> int {
        for (int wps : {2, 4, 8}) {
            int blocks = 256 * wps;
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
    run(kbench<0, 2>, "f29_mul", 2);
    run(kbench<1, 2>, "f29_sqr", 2);
    run(kbench<2, 2>, "fp_mul", 2);
    run(kbench<3, 2>, "fp_sqr", 2);
    if (argc > 1) {
        const int n = 4096;
        std::vector<u32> in(16 * n), out(27 * n);
        uint64_t st = 0x9E3779B97F4A7C15ull;
        for (auto& w : in) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; w = (u32)st; }
        for (int t = 0; t < n; ++t) { in[16 * t + 7] &= 0x7fffffffu; in[16 * t + 15] &= 0x7fffffffu; }  // < p
        for (int t = 0; t < 8; ++t) for (int i = 0; i < 8; ++i) { in[16 * t + i] = (t & 1) ? 0xffffffffu : 0u; }
        for (int i = 0; i < 8; ++i) { in[16 * 0 + 7] = 0x7fffffffu; }
        u32 *din, *dout;
        CHK(hipMalloc(&din, in.size() * 4)); CHK(hipMalloc(&dout, out.size() * 4));
        CHK(hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice));
        kcheck<<<(n + 255) / 256, 256>>>(din, dout, n);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
        FILE* f = fopen(argv[1], "wb");
        fwrite(in.data(), 4, in.size(), f);
        fwrite(out.data(), 4, out.size(), f);
        fclose(f);
        printf("dumped %d cases to %s\n", n, argv[1]);
    }
    return 0;
}
