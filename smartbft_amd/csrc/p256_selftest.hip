// p256_selftest.hip — element-wise self-test kernel for the field/scalar primitives the
// verify and sign kernels are built from (exposed as sbft_gv_selftest_field). Tests compare
// each op against Python big integers on edge values (0, 1, p-1, p, 2^256-1, ...), which
// the end-to-end ECDSA vectors do not all reach.
#include "p256_inv.hpp"
#include "p256_point.hpp"
#include "sbft_kernels.h"

namespace sbft {

__global__ __launch_bounds__(256) void selftest_kernel(int op, const uint8_t* __restrict__ a,
                                                       const uint8_t* __restrict__ b,
                                                       uint8_t* __restrict__ out, uint32_t n) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    if (op == 10) inv::stage_divstep_table(dtab);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fe x = load_be32(a + 32ull * i), y = load_be32(b + 32ull * i);
    fe r = fe_zero();
    switch (op) {
    case 0: fp_mul(r, x, y); break;           // x*y*2^-256 mod p (lazy, < 2^256)
    case 1: fp_sqr(r, x); break;              // x^2*2^-256 mod p
    case 2: fp_add(r, x, y); break;           // x+y mod p (lazy)
    case 3: fp_sub(r, x, y); break;           // x-y mod p (lazy)
    case 4: fn_mul(r, x, y); break;           // x*y*2^-256 mod n (lazy)
    case 5: fp_inv(r, x); break;              // (Montgomery) x^-1 * 2^512 mod p
    case 6: fn_inv(r, x); break;              // (Montgomery) x^-1 * 2^512 mod n
    case 7: fp_canon(r, x); break;            // x mod p for x < 2^256
    case 8: fn_canon(r, x); break;            // x mod n for x < 2^256
    case 9: fn_add(r, x, y); break;           // x+y mod n, inputs < n
    case 10: inv::inv_mod_n(r.v, x.v, dtab); break; // x^-1 mod n (plain, safegcd), 0 < x < n
    default: break;
    }
    store_be32(out + 32ull * i, r);
}

}  // namespace sbft

extern "C" int sbft_launch_selftest(int op, const uint8_t* d_a, const uint8_t* d_b, uint8_t* d_out,
                                    uint32_t n, hipStream_t stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(sbft::selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, op, d_a, d_b,
                       d_out, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
