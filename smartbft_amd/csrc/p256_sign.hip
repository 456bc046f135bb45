// p256_sign.hip — batched P-256 key derivation and ECDSA signing with caller-chosen
// nonces, gfx950. This is the engine's api.Signer side (pkg/api/dependencies.go:46-52,
// called at view.go:481 / viewchanger.go:445,1259) and the generator of the synthetic
// signed workloads bench.py verifies. It is not on the verify hot path.
//
// Per lane: Q = d*G; R = k*G; r = x(R) mod n; s = k^-1 (e + r d) mod n (FIPS 186-5 6.4.1).
// status = 1 if d, k in [1, n-1] and r, s != 0, else 0 (outputs then undefined).
#include "p256_point.hpp"
#include "sbft_kernels.h"

namespace sbft {

SBFT_DEV void to_affine(fe& x, fe& y, const jp& p) {
    fe zi, zi2, zi3, t;
    fp_inv(zi, p.z);
    fp_sqr(zi2, zi);
    fp_mul(zi3, zi2, zi);
    const fe one_plain = {{1, 0, 0, 0, 0, 0, 0, 0}};
    fp_mul(t, p.x, zi2);
    fp_mul(t, t, one_plain);  // leave Montgomery form
    fp_canon(x, t);
    fp_mul(t, p.y, zi3);
    fp_mul(t, t, one_plain);
    fp_canon(y, t);
}

__global__ __launch_bounds__(256) void p256_sign_kernel(const uint8_t* __restrict__ dd,
                                                        const uint8_t* __restrict__ kk,
                                                        const uint8_t* __restrict__ ee,
                                                        uint8_t* __restrict__ qx_out,
                                                        uint8_t* __restrict__ qy_out,
                                                        uint8_t* __restrict__ r_out,
                                                        uint8_t* __restrict__ s_out,
                                                        uint8_t* __restrict__ status, uint32_t n) {
    __shared__ u32 gtab[2 * 8 * P256_GTAB4_ENTRIES];
    for (int i = threadIdx.x; i < 2 * 8 * P256_GTAB4_ENTRIES; i += blockDim.x) gtab[i] = C_GTAB[i];
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n) return;
    const fe d = load_be32(dd + 32ull * gid);
    const fe k = load_be32(kk + 32ull * gid);
    const fe e_raw = load_be32(ee + 32ull * gid);
    bool ok = !fe_is_zero_raw(d) && fe_lt(d, P256_N) && !fe_is_zero_raw(k) && fe_lt(k, P256_N);

    jp P;
    bool inf;
    fe x, y;
    pt_mul_base(P, inf, d, gtab);
    to_affine(x, y, P);
    store_be32(qx_out + 32ull * gid, x);
    store_be32(qy_out + 32ull * gid, y);

    pt_mul_base(P, inf, k, gtab);
    to_affine(x, y, P);
    fe r;
    fn_canon(r, x);  // x < p < 2n: one conditional subtraction
    fe e;
    fn_canon(e, e_raw);
    const fe r2n = fe_const(C_R2N);
    fe dm, rm, em, km, kinv, acc, s;
    fn_mul(dm, d, r2n);
    fn_mul(rm, r, r2n);
    fn_mul(em, e, r2n);
    fn_mul(acc, rm, dm);      // r d R
    fn_canon(acc, acc);
    fn_canon(em, em);
    fn_add(acc, acc, em);     // (e + r d) R
    fn_mul(km, k, r2n);
    fn_inv(kinv, km);         // k^-1 R
    fn_mul(acc, acc, kinv);   // (e + r d) k^-1 R
    const fe one_plain = {{1, 0, 0, 0, 0, 0, 0, 0}};
    fn_mul(s, acc, one_plain);
    fn_canon(s, s);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(s);
    store_be32(r_out + 32ull * gid, r);
    store_be32(s_out + 32ull * gid, s);
    status[gid] = ok ? 1 : 0;
}

}  // namespace sbft

extern "C" int sbft_launch_p256_sign(const uint8_t* d_d, const uint8_t* d_k, const uint8_t* d_e,
                                     uint8_t* d_qx, uint8_t* d_qy, uint8_t* d_r, uint8_t* d_s,
                                     uint8_t* d_status, uint32_t n, hipStream_t stream) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    const unsigned threads = 256;
    const unsigned blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(sbft::p256_sign_kernel, dim3(blocks), dim3(threads), 0, stream, d_d, d_k, d_e,
                       d_qx, d_qy, d_r, d_s, d_status, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
