// Wall time (s_memrealtime, 100 MHz) of the half kernel's helper steps on a wavefront of their
// own: the (v, w) reduction (Lehmer rounds + exact steps) and one-lane safegcd s^-1, 48 active
// lanes per wavefront as in p256_verify_half_kernel, one wavefront per CU. Diagnostics only: the
// same work inside the kernel shares its CU's instruction cache with three verify wavefronts.
#include <cstdio>
#include <hip/hip_runtime.h>
#include "../smartbft_amd/csrc/p256_halfgcd.hpp"
using namespace sbft;

__global__ void parts(unsigned long long* out, const uint32_t* seed, int mode) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    inv::stage_divstep_table(dtab);
    const int lane = threadIdx.x;
    uint32_t u[8];
    for (int k = 0; k < 8; ++k) u[k] = seed[k] * (lane + 1) + 0x9e3779b9u * (blockIdx.x + 7) + k;
    u[7] &= 0x7fffffff;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    if (mode == 0 || mode == 2) {
        hgcd::state hs;
        hgcd::init(hs, u);
        int rounds = 0;
#pragma unroll 1
        for (int it = 0; it < 400; ++it) {
            const bool go = lane < 48 && hgcd::more(hs);
            if (!__any(go)) break;
            if (go && !((mode == 0) && hgcd::lehmer(hs))) hgcd::step(hs);
            ++rounds;
        }
        acc = hs.b[0] ^ hs.tb[0] ^ (uint32_t)rounds;
    } else if (mode == 3) {  // the quotient batches alone, six per lane, no multi-word update
        hgcd::state hs;
        hgcd::init(hs, u);
        for (int r = 0; r < 6; ++r) {
            const hgcd::lmat m = hgcd::lehmer_quotients(hs);
            acc ^= (uint32_t)m.k ^ (uint32_t)(int64_t)m.D;
            hs.b[4] ^= acc & 1u;
        }
    } else {
        uint32_t o[8];
        inv::inv_mod(o, u, dtab, false);
        acc = o[0];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) out[blockIdx.x] = (t1 - t0);
    if (acc == 0x12345678u) out[1023] = acc;
}

int main() {
    unsigned long long* d;
    uint32_t* s;
    hipMalloc(&d, 1024 * 8);
    hipMalloc(&s, 64);
    uint32_t hs[16];
    for (int i = 0; i < 16; ++i) hs[i] = 0x85ebca6bu * (i + 3);
    hipMemcpy(s, hs, 64, hipMemcpyHostToDevice);
    const char* names[4] = {"hgcd lehmer", "safegcd s^-1", "hgcd exact steps", "6 quotient batches"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 4; ++mode) {
            hipLaunchKernelGGL(parts, dim3(256), dim3(64), 0, 0, d, s, mode);
            unsigned long long h[256];
            hipMemcpy(h, d, 256 * 8, hipMemcpyDeviceToHost);
            double sum = 0, mx = 0;
            for (int i = 0; i < 256; ++i) {
                sum += h[i];
                mx = h[i] > mx ? h[i] : mx;
            }
            printf("%-18s rep %d: mean %.1f us, max %.1f us (one wavefront per CU, 48 lanes)\n", names[mode], rep,
                   sum / 256 / 100.0, mx / 100.0);
        }
    return 0;
}
