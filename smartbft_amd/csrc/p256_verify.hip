// p256_verify.hip — batched ECDSA P-256 verification for gfx950.
//
// One verify per lane. Per lane (Go 1.24.1 crypto/ecdsa.Verify semantics, restated in
// oracle/p256_oracle.c, which the parity tests hold this kernel to bit for bit):
//   1. range checks r, s in [1, n-1]; Qx, Qy < p; Q on y^2 = x^3 - 3x + b
//   2. e = digest mod n; w = s^-1 mod n (Fermat, Montgomery mod n)
//   3. u1 = e*w, u2 = r*w
//   4. R = u1*G + u2*Q: one shared doubling chain (Straus/Shamir), radix-16 Booth
//      (signed) digits for both scalars; [1..8]Q built per lane (Jacobian, scratch),
//      [1..8]G read from an LDS copy of a precomputed affine table (mixed additions)
//   5. R = infinity -> reject; accept iff X == r*Z^2 or (r+n < p and X == (r+n)*Z^2)
// Exceptional additions (P + P, P + (-P), infinity) are branched per lane under a
// wave-uniform guard, so adversarial inputs take the slow path only when present.
//
// Inputs: SoA, 32-byte big-endian fields. Output: one verdict byte per tuple.
#include "p256_field.hpp"
#include "p256_tables.inc"
#include "sbft_kernels.h"

namespace sbft {

struct jp {
    fe x, y, z;
};

__device__ __constant__ static const u32 C_R2P[8] = P256_R2P_LIMBS;
__device__ __constant__ static const u32 C_ONEP[8] = P256_ONEP_LIMBS;
__device__ __constant__ static const u32 C_BM[8] = P256_BM_LIMBS;
__device__ __constant__ static const u32 C_R2N[8] = P256_R2N_LIMBS;
__device__ __constant__ static const u32 C_ONEN[8] = P256_ONEN_LIMBS;
__device__ __constant__ static const u32 C_GTAB[2 * 8 * P256_GTAB4_ENTRIES] = P256_GTAB4_DATA;

SBFT_DEV fe fe_const(const u32* c) {
    fe r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = c[k];
    return r;
}
SBFT_DEV fe fe_zero() {
    fe r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = 0;
    return r;
}
SBFT_DEV void fe_sel(fe& r, bool c, const fe& a) {  // r = c ? a : r
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = c ? a.v[k] : r.v[k];
}
SBFT_DEV void jp_sel(jp& r, bool c, const jp& a) {
    fe_sel(r.x, c, a.x);
    fe_sel(r.y, c, a.y);
    fe_sel(r.z, c, a.z);
}

// 32 big-endian bytes -> 8 little-endian limbs
SBFT_DEV fe load_be32(const uint8_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1];
    fe r;
    r.v[7] = __builtin_bswap32(a.x);
    r.v[6] = __builtin_bswap32(a.y);
    r.v[5] = __builtin_bswap32(a.z);
    r.v[4] = __builtin_bswap32(a.w);
    r.v[3] = __builtin_bswap32(b.x);
    r.v[2] = __builtin_bswap32(b.y);
    r.v[1] = __builtin_bswap32(b.z);
    r.v[0] = __builtin_bswap32(b.w);
    return r;
}

// ------------------------------------------------------------ scalar field
// Fermat inverse a^(n-2) mod n, Montgomery domain in and out.
// n-2 = FFFFFFFF 00000000 FFFFFFFF FFFFFFFF | BCE6FAAD A7179E84 F3B9CAC2 FC63254F
SBFT_DEV void fn_sqr_n(fe& r, int count) {
#pragma unroll 1
    for (int i = 0; i < count; ++i) fn_mul(r, r, r);
}
SBFT_DEV void fn_inv(fe& r, const fe& a) {
    fe x2, x4, x8, x16, x32, t;
    t = a;
    fn_mul(t, t, t);
    fn_mul(x2, t, a);  // 2^2-1
    t = x2;
    fn_sqr_n(t, 2);
    fn_mul(x4, t, x2);
    t = x4;
    fn_sqr_n(t, 4);
    fn_mul(x8, t, x4);
    t = x8;
    fn_sqr_n(t, 8);
    fn_mul(x16, t, x8);
    t = x16;
    fn_sqr_n(t, 16);
    fn_mul(x32, t, x16);
    t = x32;             // FFFFFFFF
    fn_sqr_n(t, 64);     // FFFFFFFF 00000000 00000000
    fn_mul(t, t, x32);   // FFFFFFFF 00000000 FFFFFFFF
    fn_sqr_n(t, 32);
    fn_mul(t, t, x32);   // FFFFFFFF 00000000 FFFFFFFF FFFFFFFF
    // low 128 bits, binary from the top
    const u32 low[4] = {0xFC63254Fu, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu};
#pragma unroll 1
    for (int w = 3; w >= 0; --w) {
        const u32 bits = low[w];
#pragma unroll 1
        for (int b = 31; b >= 0; --b) {
            fn_mul(t, t, t);
            if ((bits >> b) & 1u) fn_mul(t, t, a);
        }
    }
    r = t;
}

// ------------------------------------------------------------ point arithmetic
// Doubling, a = -3 (dbl-2001-b): 3M + 5S. Infinity (Z == 0) maps to infinity.
SBFT_DEV void pt_dbl(jp& r, const jp& p) {
    fe delta, gamma, beta, alpha, t0, t1, x3;
    fp_sqr(delta, p.z);
    fp_sqr(gamma, p.y);
    fp_mul(beta, p.x, gamma);
    fp_sub(t0, p.x, delta);
    fp_add(t1, p.x, delta);
    fp_mul(alpha, t0, t1);
    fp_add(t0, alpha, alpha);
    fp_add(alpha, t0, alpha);  // 3(X-d)(X+d)
    fp_sqr(t0, alpha);
    fp_add(beta, beta, beta);
    fp_add(beta, beta, beta);  // 4 beta
    fp_add(t1, beta, beta);    // 8 beta
    fp_sub(x3, t0, t1);
    fp_add(t0, p.y, p.z);
    fp_sqr(t0, t0);
    fp_sub(t0, t0, gamma);
    fp_sub(r.z, t0, delta);
    fp_sub(t0, beta, x3);
    fp_mul(t0, alpha, t0);
    fp_sqr(gamma, gamma);
    fp_add(gamma, gamma, gamma);
    fp_add(gamma, gamma, gamma);
    fp_add(gamma, gamma, gamma);  // 8 gamma^2
    fp_sub(r.y, t0, gamma);
    r.x = x3;
}

// acc += b (b Jacobian, never infinity). Handles acc = infinity, acc == b
// (doubling) and acc == -b (infinity). use == false leaves acc unchanged.
SBFT_DEV void pt_add_jac(jp& acc, bool& inf, const jp& b, bool use) {
    fe z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
    fp_sqr(z1z1, acc.z);
    fp_sqr(z2z2, b.z);
    fp_mul(u1, acc.x, z2z2);
    fp_mul(u2, b.x, z1z1);
    fp_mul(t, b.z, z2z2);
    fp_mul(s1, acc.y, t);
    fp_mul(t, acc.z, z1z1);
    fp_mul(s2, b.y, t);
    fp_sub(h, u2, u1);
    fp_sub(rr, s2, s1);
    const bool hz = fp_is_zero(h);
    const bool rz = fp_is_zero(rr);
    jp sum;
    fe hh, hhh, v;
    fp_sqr(hh, h);
    fp_mul(hhh, hh, h);
    fp_mul(v, u1, hh);
    fp_sqr(sum.x, rr);
    fp_sub(sum.x, sum.x, hhh);
    fp_sub(sum.x, sum.x, v);
    fp_sub(sum.x, sum.x, v);
    fp_sub(t, v, sum.x);
    fp_mul(sum.y, rr, t);
    fp_mul(t, s1, hhh);
    fp_sub(sum.y, sum.y, t);
    fp_mul(t, acc.z, b.z);
    fp_mul(sum.z, t, h);
    bool sum_inf = false;
    const bool live = use && !inf;
    const bool need_dbl = live && hz && rz;
    if (__builtin_expect(__any(need_dbl), 0)) {
        jp d;
        pt_dbl(d, acc);
        jp_sel(sum, need_dbl, d);
    }
    sum_inf = hz && !rz;
    // assemble: !use -> acc; inf -> b; else sum
    jp out = acc;
    bool out_inf = inf;
    jp_sel(out, live, sum);
    if (live) out_inf = sum_inf;
    jp_sel(out, use && inf, b);
    if (use && inf) out_inf = false;
    acc = out;
    inf = out_inf;
}

// acc += (x2, y2) affine (Montgomery), never infinity: mixed addition 8M + 3S.
SBFT_DEV void pt_add_aff(jp& acc, bool& inf, const fe& x2, const fe& y2, bool use) {
    fe z1z1, u2, s2, h, rr, t;
    fp_sqr(z1z1, acc.z);
    fp_mul(u2, x2, z1z1);
    fp_mul(t, acc.z, z1z1);
    fp_mul(s2, y2, t);
    fp_sub(h, u2, acc.x);
    fp_sub(rr, s2, acc.y);
    const bool hz = fp_is_zero(h);
    const bool rz = fp_is_zero(rr);
    jp sum;
    fe hh, hhh, v;
    fp_sqr(hh, h);
    fp_mul(hhh, hh, h);
    fp_mul(v, acc.x, hh);
    fp_sqr(sum.x, rr);
    fp_sub(sum.x, sum.x, hhh);
    fp_sub(sum.x, sum.x, v);
    fp_sub(sum.x, sum.x, v);
    fp_sub(t, v, sum.x);
    fp_mul(sum.y, rr, t);
    fp_mul(t, acc.y, hhh);
    fp_sub(sum.y, sum.y, t);
    fp_mul(sum.z, acc.z, h);
    const bool live = use && !inf;
    const bool need_dbl = live && hz && rz;
    if (__builtin_expect(__any(need_dbl), 0)) {
        jp d;
        pt_dbl(d, acc);
        jp_sel(sum, need_dbl, d);
    }
    const bool sum_inf = hz && !rz;
    jp out = acc;
    bool out_inf = inf;
    jp_sel(out, live, sum);
    if (live) out_inf = sum_inf;
    if (use && inf) {
        out.x = x2;
        out.y = y2;
        out.z = fe_const(C_ONEP);
        out_inf = false;
    }
    acc = out;
    inf = out_inf;
}

// Radix-16 Booth digit from the 5-bit window (b3 b2 b1 b0 b-1): value in [-8, 8].
SBFT_DEV int booth(u32 w5) { return (int)((w5 >> 1) + (w5 & 1u)) - (int)((w5 >> 4) << 4); }

// ------------------------------------------------------------ the kernel
__global__ __launch_bounds__(256) void p256_verify_kernel(const uint8_t* __restrict__ digest,
                                                          const uint8_t* __restrict__ rr,
                                                          const uint8_t* __restrict__ ss,
                                                          const uint8_t* __restrict__ qxx,
                                                          const uint8_t* __restrict__ qyy,
                                                          uint8_t* __restrict__ ok, uint32_t n) {
    __shared__ u32 gtab[2 * 8 * P256_GTAB4_ENTRIES];
    for (int i = threadIdx.x; i < 2 * 8 * P256_GTAB4_ENTRIES; i += blockDim.x) gtab[i] = C_GTAB[i];
    __syncthreads();

    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = gid < n;
    const uint32_t idx = active ? gid : (n - 1);

    const fe e_raw = load_be32(digest + 32ull * idx);
    const fe r = load_be32(rr + 32ull * idx);
    const fe s = load_be32(ss + 32ull * idx);
    const fe qx = load_be32(qxx + 32ull * idx);
    const fe qy = load_be32(qyy + 32ull * idx);

    // 1. range checks
    bool valid = !fe_is_zero_raw(r) && fe_lt(r, P256_N) && !fe_is_zero_raw(s) && fe_lt(s, P256_N) &&
                 fe_lt(qx, P256_P) && fe_lt(qy, P256_P);

    // Q to Montgomery form and on-curve check y^2 == x^3 - 3x + b
    const fe r2p = fe_const(C_R2P);
    jp q;
    fp_mul(q.x, qx, r2p);
    fp_mul(q.y, qy, r2p);
    q.z = fe_const(C_ONEP);
    {
        fe lhs, rhs, t;
        fp_sqr(lhs, q.y);
        fp_sqr(rhs, q.x);
        fp_mul(rhs, rhs, q.x);
        fp_add(t, q.x, q.x);
        fp_add(t, t, q.x);
        fp_sub(rhs, rhs, t);
        fp_add(rhs, rhs, fe_const(C_BM));
        fp_canon(lhs, lhs);
        fp_canon(rhs, rhs);
        valid = valid && fe_eq(lhs, rhs);
    }

    // 2-3. scalars
    fe e;
    fn_canon(e, e_raw);
    fe sm, w, u1, u2;
    fn_mul(sm, s, fe_const(C_R2N));  // s*R mod n
    fn_inv(w, sm);                    // s^-1 * R
    fn_mul(u1, e, w);                 // e*s^-1 (plain)
    fn_mul(u2, r, w);                 // r*s^-1 (plain)

    // 4. [1..8]Q in Jacobian form (scratch)
    jp tq[8];
    tq[0] = q;
    pt_dbl(tq[1], q);
#pragma unroll 1
    for (int k = 2; k < 8; ++k) {
        jp t = tq[k - 1];
        bool tinf = false;
        pt_add_jac(t, tinf, q, true);
        tq[k] = t;
    }

    jp acc;
    bool inf = true;
    acc.x = fe_zero();
    acc.y = fe_zero();
    acc.z = fe_zero();
    // window 64: the digit is bit 255
    {
        const bool b2 = (u2.v[7] >> 31) != 0;
        const bool b1 = (u1.v[7] >> 31) != 0;
        pt_add_jac(acc, inf, q, b2);
        fe gx, gy;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            gx.v[k] = gtab[k];
            gy.v[k] = gtab[8 + k];
        }
        pt_add_aff(acc, inf, gx, gy, b1);
    }
    fe k1 = u1, k2 = u2;
#pragma unroll 1
    for (int limb = 7; limb >= 0; --limb) {
        const u32 cur1 = k1.v[7], below1 = k1.v[6];
        const u32 cur2 = k2.v[7], below2 = k2.v[6];
#pragma unroll
        for (int k = 7; k > 0; --k) {
            k1.v[k] = k1.v[k - 1];
            k2.v[k] = k2.v[k - 1];
        }
        k1.v[0] = 0;
        k2.v[0] = 0;
        const u64 w1 = ((u64)cur1 << 1) | (below1 >> 31);
        const u64 w2 = ((u64)cur2 << 1) | (below2 >> 31);
#pragma unroll 1
        for (int nib = 7; nib >= 0; --nib) {
#pragma unroll 1
            for (int d = 0; d < 4; ++d) pt_dbl(acc, acc);
            const int d2 = booth((u32)(w2 >> (4 * nib)) & 31u);
            const int d1 = booth((u32)(w1 >> (4 * nib)) & 31u);
            // Q digit
            {
                const int m = d2 < 0 ? -d2 : d2;
                jp t = tq[m > 0 ? m - 1 : 0];
                if (d2 < 0) {
                    fe ny;
                    fp_sub(ny, fe_zero(), t.y);
                    t.y = ny;
                }
                pt_add_jac(acc, inf, t, d2 != 0);
            }
            // G digit
            {
                const int m = d1 < 0 ? -d1 : d1;
                const int base = (m > 0 ? m - 1 : 0) * 16;
                fe gx, gy;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    gx.v[k] = gtab[base + k];
                    gy.v[k] = gtab[base + 8 + k];
                }
                if (d1 < 0) {
                    fe ny;
                    fp_sub(ny, fe_zero(), gy);
                    gy = ny;
                }
                pt_add_aff(acc, inf, gx, gy, d1 != 0);
            }
        }
    }

    // 5. x(R) mod n == r, projectively
    bool accept = false;
    if (!inf) {
        fe z2, lhs, xc, rm;
        fp_sqr(z2, acc.z);
        fp_canon(xc, acc.x);
        fp_mul(rm, r, r2p);
        fp_mul(lhs, rm, z2);
        fp_canon(lhs, lhs);
        accept = fe_eq(lhs, xc);
        // r + n < p ?
        fe rn;
        u64 c = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            c = (u64)r.v[k] + P256_N[k] + c;
            rn.v[k] = lo32(c);
            c >>= 32;
        }
        if (c == 0 && fe_lt(rn, P256_P)) {
            fp_mul(rm, rn, r2p);
            fp_mul(lhs, rm, z2);
            fp_canon(lhs, lhs);
            accept = accept || fe_eq(lhs, xc);
        }
    }
    if (active) ok[gid] = (valid && accept) ? 1 : 0;
}

}  // namespace sbft

extern "C" int sbft_launch_p256_verify(const uint8_t* d_digest, const uint8_t* d_r, const uint8_t* d_s,
                                       const uint8_t* d_qx, const uint8_t* d_qy, uint8_t* d_ok,
                                       uint32_t n, hipStream_t stream) {
    if (n == 0) return 0;
    const unsigned threads = 256;
    const unsigned blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(sbft::p256_verify_kernel, dim3(blocks), dim3(threads), 0, stream, d_digest, d_r,
                       d_s, d_qx, d_qy, d_ok, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
