// p256_selftest.hip — element-wise self-test kernel for the field/scalar primitives the
// verify and sign kernels are built from (exposed as sbft_gv_selftest_field). Tests compare
// each op against Python big integers on edge values (0, 1, p-1, p, 2^256-1, ...), which
// the end-to-end ECDSA vectors do not all reach.
#include "p256_f29.hpp"
#include "p256_inv.hpp"
#include "p256_point.hpp"
#include "sbft_kernels.h"

namespace sbft {

// ---- radix-2^29 ladder layer (p256_f29.hpp), in and out as plain integers mod p ----
SBFT_DEV f29 to_mont29(const fe& a) {
    f29 r;
    f29_mul(r, f29_from_u256(a), f29_const(C29_R2));
    return r;
}
// affine (x, y) of a Jacobian point, canonical plain values
SBFT_DEV void affine29(const jp29& p, fe& x, fe& y, const uint32_t* dtab) {
    fe zp = f29_canon_plain(p.z), zi;
    inv::inv_mod_p(zi.v, zp.v, dtab);
    const f29 z = to_mont29(zi);
    f29 z2, z3, t;
    f29_sqr(z2, z);
    f29_mul(z3, z2, z);
    f29_mul(t, p.x, z2);
    x = f29_canon_plain(t);
    f29_mul(t, p.y, z3);
    y = f29_canon_plain(t);
}
// 2^5 P through the ladder's doubling, the loop unrolled U times
template <int U>
SBFT_DEV jp29 dbl5(jp29 acc) {
#pragma unroll U
    for (int d = 0; d < 5; ++d) p29_dbl(acc, acc);
    return acc;
}

// diagnostics of the unrolled loop: no aliasing (20), interleaved doubling (21), a
// scheduling barrier between iterations (22)
SBFT_DEV jp29 dbl5_noalias(jp29 acc) {
#pragma unroll 2
    for (int d = 0; d < 5; ++d) {
        jp29 t;
        p29_dbl(t, acc);
        acc = t;
    }
    return acc;
}
SBFT_DEV jp29 dbl5_il(jp29 acc) {
#pragma unroll 2
    for (int d = 0; d < 5; ++d) p29_dbl_i(acc, acc);
    return acc;
}
SBFT_DEV jp29 dbl5_sb(jp29 acc) {
#pragma unroll 2
    for (int d = 0; d < 5; ++d) {
        p29_dbl(acc, acc);
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

SBFT_DEV fe selftest_f29(int op, const fe& x, const fe& y, const uint32_t* dtab) {
    fe r = fe_zero();
    if (op == 11 || op == 12) {  // x*y, x^2 mod p through f29_mul / f29_sqr
        const f29 a = to_mont29(x), b = to_mont29(y);
        f29 t;
        if (op == 11) f29_mul(t, a, b);
        else f29_sqr(t, a);
        return f29_canon_plain(t);
    }
    if (op == 13) {  // x^-1 mod p (safegcd), 0 < x < p
        inv::inv_mod_p(r.v, x.v, dtab);
        return r;
    }
    // point ops on P = (x, y) (on the curve)
    jp29 p;
    p.x = to_mont29(x);
    p.y = to_mont29(y);
    p.z = f29_const(C29_ONE);
    fe ox, oy;
    switch (op) {
    case 14: affine29(dbl5<1>(p), ox, oy, dtab); return ox;  // x(32P)
    case 15: affine29(dbl5<2>(p), ox, oy, dtab); return ox;  // x(32P), unrolled doubling loop
    case 16: affine29(dbl5<1>(p), ox, oy, dtab); return oy;  // y(32P)
    case 17: {                                                // x(3P): mixed addition 2P + P
        jp29 t;
        p29_dbl(t, p);
        p29_add_aff_lean(t, p.x, p.y);
        affine29(t, ox, oy, dtab);
        return ox;
    }
    case 18: {                                                // y(6P): Jacobian addition 2P + 4P
        jp29 t2, t4;
        p29_dbl(t2, p);
        p29_dbl(t4, t2);
        p29_add_jac_lean(t4, t2);
        affine29(t4, ox, oy, dtab);
        return oy;
    }
    case 19: {                                                // y(3P) with -P negated twice
        jp29 t;
        p29_dbl(t, p);
        f29 ny;
        f29_neg(ny, p.y);
        f29_neg(ny, ny);
        p29_add_aff_lean(t, p.x, ny);
        affine29(t, ox, oy, dtab);
        return oy;
    }
    case 20: affine29(dbl5_noalias(p), ox, oy, dtab); return ox;
    case 21: affine29(dbl5_il(p), ox, oy, dtab); return ox;
    case 22: affine29(dbl5_sb(p), ox, oy, dtab); return ox;
    default: return r;
    }
}

// Ops 23..26 run on lane pairs (2t, 2t + 1), both lanes on element 2t's inputs, as the half
// kernel's ladder pairs do: 23 / 24 inv::inv_mod_pair mod p / mod n (x^-1, plain); 25 / 26 x / y
// of 33P through the lane-local W ladder (p29_dbl_plw x5, then p29_add_aff_plw with P itself,
// c = 1: W = Z^2). Every lane of the pair computes; both store the result.
SBFT_DEV fe selftest_pair(int op, const fe& x, const fe& y, const uint32_t* dtab, bool odd) {
    fe r = fe_zero();
    if (op == 23 || op == 24) {
        inv::inv_mod_pair(r.v, x.v, dtab, op == 23, odd);
        return r;
    }
    const f29 px = to_mont29(x), py = to_mont29(y), one = f29_const(C29_ONE);
    plw29 q;
    q.xb = px;
    q.zy = f29_sel_pair(one, py);
    q.zo = one;
    q.w = one;
    for (int k = 0; k < 5; ++k) p29_dbl_plw(q);
    p29_add_aff_plw(q, px, py);
    jp29 t;
    plw29_to(t, q);
    fe ox, oy;
    affine29(t, ox, oy, dtab);
    return op == 25 ? ox : oy;
}

// Ops 27..30 run on quads (4t .. 4t + 3), every lane on element 4t's inputs, as the wide half
// kernel's ladders do (q4_dbl / q4_add_rest / q4_add_full, c = 1: W = Z^2): 27 / 28 x / y of 33P
// (four doublings, a fifth carrying the addition's first step, the addition's rest with P itself);
// 29 / 30 x / y of 32P = 33P + (-P) (then a whole addition of -P, from the N+- Y of the first).
SBFT_DEV fe selftest_quad(int op, const fe& x, const fe& y, const uint32_t* dtab) {
    const f29 px = to_mont29(x), py = to_mont29(y), one = f29_const(C29_ONE);
    q4w q;
    q4w_init(q, px, py, one, one);
    f29 ut;
    for (int k = 0; k < 4; ++k) q4_dbl<false>(q, px, ut);
    q4_dbl<true>(q, px, ut);
    q4_add_rest(q, py, ut);
    if (op >= 29) {
        f29 ny;
        f29_neg(ny, py);
        q4_add_full(q, px, ny);
    }
    jp29 t;
    q4w_to(t, q);
    fe ox, oy;
    affine29(t, ox, oy, dtab);
    return (op & 1) ? ox : oy;
}

__global__ __launch_bounds__(256) void selftest_kernel(int op, const uint8_t* __restrict__ a,
                                                       const uint8_t* __restrict__ b,
                                                       uint8_t* __restrict__ out, uint32_t n) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    if (op == 10 || op >= 13) inv::stage_divstep_table(dtab);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (op >= 27 && op <= 30) {  // quads: no lane leaves before the others of its quad
        const uint32_t e = ((i & ~3u) < n ? i : n - 1) & ~3u;
        const fe x = load_be32(a + 32ull * e), y = load_be32(b + 32ull * e);
        const fe r = selftest_quad(op, x, y, dtab);
        if (i < n) store_be32(out + 32ull * i, r);
        return;
    }
    if (op >= 23 && op <= 26) {  // lane pairs: no lane leaves before its partner
        const uint32_t e = ((i & ~1u) < n ? i : n - 1) & ~1u;
        const fe x = load_be32(a + 32ull * e), y = load_be32(b + 32ull * e);
        const fe r = selftest_pair(op, x, y, dtab, (i & 1u) != 0);
        if (i < n) store_be32(out + 32ull * i, r);
        return;
    }
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
    default: r = selftest_f29(op, x, y, dtab); break;  // 11..19: the f29 ladder layer
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
