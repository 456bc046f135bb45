// Cycle counts (s_memtime) of the keyed-verify building blocks on one wavefront: safegcd
// inverse, one general Jacobian addition, one fp_mul, one SHA-256 block. Diagnostics only.
#include <cstdio>
#include "../smartbft_amd/csrc/p256_inv.hpp"
#include "../smartbft_amd/csrc/p256_point.hpp"
#include "../smartbft_amd/csrc/sha256_dev.hpp"
using namespace sbft;

__global__ void phases(unsigned long long* out, const uint32_t* seed) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    inv::stage_divstep_table(dtab);
    fe a, b;
    for (int k = 0; k < 8; ++k) { a.v[k] = seed[k] ^ threadIdx.x; b.v[k] = seed[8 + k] + 3 * threadIdx.x; }
    a.v[7] &= 0x7fffffff;
    fe au;
    for (int k = 0; k < 8; ++k) au.v[k] = seed[k] * 7 + blockIdx.x;
    au.v[7] &= 0x7fffffff;
    unsigned long long tu0 = clock64();
    fe wu; inv::inv_mod_n(wu.v, au.v, dtab);
    unsigned long long tu1 = clock64();
    unsigned long long t0 = clock64();
    fe w; inv::inv_mod_n(w.v, a.v, dtab);
    unsigned long long t1 = clock64();
    fe m = a;
    for (int i = 0; i < 100; ++i) fp_mul(m, m, b);
    unsigned long long t2 = clock64();
    jp p = {a, b, m}, q = {b, m, a};
    bool inf = false;
    for (int i = 0; i < 10; ++i) pt_add_jac(p, inf, q, true);
    unsigned long long t3 = clock64();
    for (int i = 0; i < 10; ++i) pt_dbl(p, p);
    unsigned long long t4 = clock64();
    uint32_t h[8];
    sha256_one((const uint8_t*)seed, 55, h);
    unsigned long long t5 = clock64();
    for (int i = 0; i < 100; ++i) fn_mul(m, m, b);
    unsigned long long t6 = clock64();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0; out[1] = (t2 - t1) / 100; out[2] = (t3 - t2) / 10; out[3] = (t4 - t3) / 10;
        out[4] = t5 - t4; out[5] = (t6 - t5) / 100;
        out[6] = w.v[0] ^ m.v[0] ^ p.x.v[0] ^ h[0] ^ wu.v[0]; out[7] = tu1 - tu0;
    }
}

int main() {
    unsigned long long* d; uint32_t* s;
    hipMalloc(&d, 64); hipMalloc(&s, 256);
    uint32_t hs[64]; for (int i = 0; i < 64; ++i) hs[i] = 0x9e3779b9u * (i + 1);
    hipMemcpy(s, hs, 256, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(phases, dim3(1), dim3(64), 0, 0, d, s);
        unsigned long long h[8];
        hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
        printf("cycles: inv_mod_n uniform(SALU) %llu | lane-varying %llu | fp_mul %llu | pt_add_jac %llu | pt_dbl %llu | sha256 1 block %llu | fn_mul %llu\n",
               h[7], h[0], h[1], h[2], h[3], h[4], h[5]);
    }
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("clock rate attr (kHz): %d\n", clk);
    return 0;
}
