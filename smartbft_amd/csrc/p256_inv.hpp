// p256_inv.hpp — variable-time modular inversion mod the P-256 group order n (or the field
// prime p: the verify kernel's affine Q table) by batched
// divsteps (Bernstein–Yang "safegcd", 30 divsteps per batch on 32-bit words).
//
// Used where one inversion sits on a latency path: the keyed single-signature verify
// (p256_keyed.hip), where a Fermat chain (~250 sequential squarings mod n, ~95k VALU
// instructions) would dominate the launch. Verification data is public, so a variable-time
// inversion is acceptable (crypto/ecdsa.Verify's own inversion is variable time too).
//
// Header-only and free of HIP types so that tests/native can compile the same code for the
// CPU with g++ and check it against Python's pow(x, -1, n).
//
// Algorithm (restated from Bernstein & Yang, "Fast constant-time gcd computation and modular
// inversion", 2019, sections 8-10; original divstep with delta starting at 1):
//   f = n, g = x, d = 0, e = 1; invariant d*x = f, e*x = g (mod n).
//   repeat: take the low 32 bits of f, g; run 30 divsteps on them (5 per table lookup), accumulating the 2x2
//   transition matrix T (entries bounded by 2^30); then (f, g) <- T (f, g) / 2^30 exactly and
//   (d, e) <- T (d, e) / 2^30 mod n; until g == 0. Then f = +-1 and x^-1 = +-d.
//   At most 741 divsteps (25 batches) for 256-bit inputs (BY19 Theorem 11.2 bound).
// Numbers are signed radix-2^30: 9 limbs, limbs 0..7 in [0, 2^30), limb 8 signed.
#pragma once
#include <stdint.h>

#include "p256_inv_table.inc"
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#if defined(__HIPCC__)
#define SBFT_HD __host__ __device__ __forceinline__
#else
#define SBFT_HD static inline
#endif
#if defined(__HIPCC__)
#define SBFT_UNROLL1 _Pragma("unroll 1")
#define SBFT_UNROLL _Pragma("unroll")
#else
#define SBFT_UNROLL1
#define SBFT_UNROLL
#endif
#ifndef SBFT_INV_PIPE
#define SBFT_INV_PIPE 1  // inv_mod: the next batch's divsteps overlap this batch's updates
#endif

namespace sbft {
namespace inv {

// acc + a*b (signed 32 x 32 -> 64): one v_mad_i64_i32 on the device
SBFT_HD int64_t mac(int64_t acc, int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    int64_t r;
    uint64_t cc;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(acc));
    return r;
#else
    return acc + (int64_t)a * b;
#endif
}

struct s30 {
    int32_t v[9];
};

#define SBFT_M30 0x3fffffff
// n in radix 2^30 and n^-1 mod 2^30
#define SBFT_N30_INIT {0x3c632551, 0x0ee72b0b, 0x3179e84f, 0x39beab69, 0x3fffffbc, 0x3fffffff, 0x00000fff, 0x3fffc000, 0x0000ffff}
#define SBFT_NINV30 0x11ff43b1u  // n^-1 mod 2^30 (so that d + md*n = 0 mod 2^30 for md = -d * NINV30)
// the field prime p in radix 2^30; p = -1 mod 2^96, so p^-1 = -1 mod 2^30
#define SBFT_P30_INIT {0x3fffffff, 0x3fffffff, 0x3fffffff, 0x0000003f, 0x00000000, 0x00000000, 0x00001000, 0x3fffc000, 0x0000ffff}
#define SBFT_PINV30 0x3fffffffu

// The modulus of an inversion: P = false for the group order n, true for the field prime p.
// P is a run-time flag so that the two lanes of a verify pair can invert mod p and mod n in
// the same instruction stream (p256_verify_small_kernel<2>); constant P folds away when inlined.
SBFT_HD void mod30(int32_t m[9], bool P) {
    const int32_t N30[9] = SBFT_N30_INIT, P30[9] = SBFT_P30_INIT;
    for (int i = 0; i < 9; ++i) m[i] = P ? P30[i] : N30[i];
}

SBFT_HD void pack30(s30& r, const uint32_t a[8]) {
    // 8 x 32-bit little-endian limbs -> 9 x 30-bit limbs (value < 2^256)
    for (int i = 0; i < 9; ++i) {
        const int bit = 30 * i, w = bit >> 5, sh = bit & 31;
        uint64_t x = (uint64_t)a[w] >> sh;
        if (w + 1 < 8) x |= (uint64_t)a[w + 1] << (32 - sh);
        r.v[i] = (int32_t)(x & SBFT_M30);
    }
}

// 30 original divsteps on the low words of f (odd) and g, 5 at a time through the transition
// table (p256_inv_table.inc, tools/gen_inv_table.py): a step's outcome depends only on
// delta > 0 and the parity of g, so 5 steps depend on clamp(delta, -4, 5) and the low 5 bits
// of f and g. Returns delta; T = [u v; q r] with 2^30 (f', g') = T (f, g). `tab` is the table
// (in LDS on the device: one ~70-cycle ds_read per 5 divsteps on the dependent chain).
SBFT_HD int32_t divsteps30(int32_t delta, uint32_t f, uint32_t g, const uint32_t* tab, int32_t& u, int32_t& v,
                           int32_t& q, int32_t& r) {
    int32_t uu = 1, vv = 0, qq = 0, rr = 1;
    for (int j = 0; j < 6; ++j) {
        const int32_t dc = delta < -4 ? -4 : (delta > 5 ? 5 : delta);
        const uint32_t idx = ((uint32_t)(dc + 4) << 9) | (((f >> 1) & 15u) << 5) | (g & 31u);
        const uint32_t w = tab[idx];  // packed entry, tools/gen_inv_table.py
        const int32_t a = (int32_t)(w & 63u) - 8, b = (int32_t)((w >> 6) & 63u) - 6;
        const int32_t c = (int32_t)((w >> 12) & 63u) - 16, d = (int32_t)((w >> 18) & 63u) - 15;
        // low words advance by 5 divsteps (the low 5 bits of a f + b g and c f + d g are zero)
        const uint32_t nf = ((uint32_t)a * f + (uint32_t)b * g) >> 5;
        const uint32_t ng = ((uint32_t)c * f + (uint32_t)d * g) >> 5;
        f = nf;
        g = ng;
        // T <- M T
        const int32_t nu = a * uu + b * qq, nv = a * vv + b * rr;
        const int32_t nq = c * uu + d * qq, nr = c * vv + d * rr;
        uu = nu;
        vv = nv;
        qq = nq;
        rr = nr;
        const int32_t cst = (int32_t)((w >> 24) & 15u) - 3;
        delta = ((w >> 28) & 1u ? -delta : delta) + cst;
    }
    u = uu;
    v = vv;
    q = qq;
    r = rr;
    return delta;
}

// (f, g) <- T (f, g) / 2^30 (exact)
SBFT_HD void update_fg(s30& f, s30& g, int32_t u, int32_t v, int32_t q, int32_t r) {
    int64_t cf = mac(mac(0, u, f.v[0]), v, g.v[0]);
    int64_t cg = mac(mac(0, q, f.v[0]), r, g.v[0]);
    cf >>= 30;
    cg >>= 30;
    for (int i = 1; i < 9; ++i) {
        cf = mac(mac(cf, u, f.v[i]), v, g.v[i]);
        cg = mac(mac(cg, q, f.v[i]), r, g.v[i]);
        f.v[i - 1] = (int32_t)(cf & SBFT_M30);
        g.v[i - 1] = (int32_t)(cg & SBFT_M30);
        cf >>= 30;
        cg >>= 30;
    }
    f.v[8] = (int32_t)cf;
    g.v[8] = (int32_t)cg;
}

// (d, e) <- (T (d, e) + (md, me) m) / 2^30 with md, me chosen to clear the low 30 bits
// (m = n, or p when P). |d|, |e| grow by at most m per batch (|u| + |v| <= 2^30), so 25
// batches stay below 2^262.
SBFT_HD void update_de(s30& d, s30& e, int32_t u, int32_t v, int32_t q, int32_t r, bool P) {
    int32_t N30[9];
    mod30(N30, P);
    const uint32_t minv = P ? SBFT_PINV30 : SBFT_NINV30;
    int64_t cd = mac(mac(0, u, d.v[0]), v, e.v[0]);
    int64_t ce = mac(mac(0, q, d.v[0]), r, e.v[0]);
    const int32_t md = (int32_t)((0u - (uint32_t)cd * minv) & SBFT_M30);
    const int32_t me = (int32_t)((0u - (uint32_t)ce * minv) & SBFT_M30);
    cd = mac(cd, md, N30[0]);
    ce = mac(ce, me, N30[0]);
    cd >>= 30;
    ce >>= 30;
    for (int i = 1; i < 9; ++i) {
        cd = mac(mac(mac(cd, u, d.v[i]), v, e.v[i]), md, N30[i]);
        ce = mac(mac(mac(ce, q, d.v[i]), r, e.v[i]), me, N30[i]);
        d.v[i - 1] = (int32_t)(cd & SBFT_M30);
        e.v[i - 1] = (int32_t)(ce & SBFT_M30);
        cd >>= 30;
        ce >>= 30;
    }
    d.v[8] = (int32_t)cd;
    e.v[8] = (int32_t)ce;
}

SBFT_HD bool is_zero30(const s30& a) {
    int32_t o = 0;
    for (int i = 0; i < 9; ++i) o |= a.v[i];
    return o == 0;
}

// a += k * m for a small signed k (m = n, or p when P), renormalising limbs 0..7 to [0, 2^30)
SBFT_HD void add_kn(s30& a, int32_t k, bool P) {
    int32_t N30[9];
    mod30(N30, P);
    int64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        c += (int64_t)a.v[i] + (int64_t)k * N30[i];
        a.v[i] = (int32_t)(c & SBFT_M30);
        c >>= 30;
    }
    a.v[8] = (int32_t)(c + a.v[8] + (int64_t)k * N30[8]);
}

// a (normalised, |a| < 2^262) -> [0, m), then 8 x 32-bit limbs
SBFT_HD void reduce_unpack(uint32_t out[8], s30 a, bool P) {
    // a = t * 2^240 + low with t = a.v[8]; m = 2^256 - c with c < 2^225 (n: c < 2^128), so
    // k = -floor(a / 2^256) gets within a few m of [0, m)
    add_kn(a, -(a.v[8] >> 16), P);
    for (int it = 0; it < 4 && a.v[8] < 0; ++it) add_kn(a, 1, P);
    int32_t N30[9];
    mod30(N30, P);
    for (int it = 0; it < 4; ++it) {
        // a >= n ?
        bool ge = true;
        for (int i = 8; i >= 0; --i) {
            if (a.v[i] != N30[i]) {
                ge = a.v[i] > N30[i];
                break;
            }
        }
        if (!ge) break;
        add_kn(a, -1, P);
    }
    for (int w = 0; w < 8; ++w) {
        const int bit = 32 * w, i = bit / 30, sh = bit % 30;
        uint64_t x = (uint64_t)(uint32_t)a.v[i] >> sh;
        if (i + 1 < 9) x |= (uint64_t)(uint32_t)a.v[i + 1] << (30 - sh);
        if (i + 2 < 9 && 60 - sh < 64) x |= (uint64_t)(uint32_t)a.v[i + 2] << (60 - sh);
        out[w] = (uint32_t)x;
    }
}

// out = c x^-1 mod m for 0 < x < m and c < m (8 x 32-bit little-endian limbs; m = n, or p
// when P; c = null means 1). x = 0 gives 0. tab: SBFT_DIVSTEP5_TABLE (p256_inv_table.inc).
// Starting e at c instead of 1 keeps d x = c f, e x = c g (mod m), so the result comes out
// scaled for free (c = 2^256 mod n: the Montgomery form the fn_ arithmetic takes).
SBFT_HD void inv_mod(uint32_t out[8], const uint32_t x[8], const uint32_t* tab, bool P,
                     const uint32_t* c = nullptr) {
    s30 f, g, d, e;
    mod30(f.v, P);
    pack30(g, x);
    for (int i = 0; i < 9; ++i) {
        d.v[i] = 0;
        e.v[i] = 0;
    }
    if (c)
        pack30(e, c);
    else
        e.v[0] = 1;
    int32_t delta = 1;
#if SBFT_INV_PIPE
    // Software-pipelined: batch i+1's divsteps need only the low limb of T_i (f, g) / 2^30,
    // which limbs 0 and 1 give; so they are computed first, and the next batch's dependent
    // chain of table lookups runs while the full (f, g) and (d, e) updates of batch i fill its
    // wait cycles (the one-lane form is latency-bound: one wavefront per SIMD on the latency
    // kernels). The last batch's look-ahead is computed and dropped.
    int32_t u, v, q, r;
    delta = divsteps30(delta, (uint32_t)f.v[0], (uint32_t)g.v[0], tab, u, v, q, r);
SBFT_UNROLL1
    for (int batch = 0; batch < 26 && !is_zero30(g); ++batch) {
        const int64_t lf = (mac(mac(0, u, f.v[0]), v, g.v[0]) >> 30) + (int64_t)u * f.v[1] + (int64_t)v * g.v[1];
        const int64_t lg = (mac(mac(0, q, f.v[0]), r, g.v[0]) >> 30) + (int64_t)q * f.v[1] + (int64_t)r * g.v[1];
        int32_t u2, v2, q2, r2;
        const int32_t delta2 = divsteps30(delta, (uint32_t)lf & SBFT_M30, (uint32_t)lg & SBFT_M30, tab, u2, v2, q2, r2);
        update_de(d, e, u, v, q, r, P);
        update_fg(f, g, u, v, q, r);
        delta = delta2;
        u = u2;
        v = v2;
        q = q2;
        r = r2;
    }
#else
SBFT_UNROLL1
    for (int batch = 0; batch < 26 && !is_zero30(g); ++batch) {
        int32_t u, v, q, r;
        delta = divsteps30(delta, (uint32_t)f.v[0], (uint32_t)g.v[0], tab, u, v, q, r);
        update_de(d, e, u, v, q, r, P);
        update_fg(f, g, u, v, q, r);
    }
#endif
    // f = +-1: x^-1 = f * d
    if (f.v[8] < 0) {
        for (int i = 0; i < 9; ++i) d.v[i] = -d.v[i];
        add_kn(d, 0, P);  // renormalise limbs
    }
    reduce_unpack(out, d, P);
}
SBFT_HD void inv_mod_n(uint32_t out[8], const uint32_t x[8], const uint32_t* tab) { inv_mod(out, x, tab, false); }
SBFT_HD void inv_mod_p(uint32_t out[8], const uint32_t x[8], const uint32_t* tab) { inv_mod(out, x, tab, true); }
// c x^-1 mod n
SBFT_HD void inv_mod_n_scaled(uint32_t out[8], const uint32_t x[8], const uint32_t c[8], const uint32_t* tab) {
    inv_mod(out, x, tab, false, c);
}

#if defined(__HIPCC__)
// The same inversion on a whole wavefront, for latency paths (every lane passes the same x and
// c and gets the result). Lane i < 9 holds limb i of f, g, d, e (lanes >= 9 hold zeros). Each
// batch's 30 divsteps run wave-uniformly on the low words (LDS table, as above); the 2x2
// transition matrix then updates every limb at once, two or three 64-bit mads per number per
// lane, and the exact division by 2^30 is two parallel carry rounds (DPP shifts by one lane):
// limbs end in [-2, 2^30 + 4), the top limb signed. The serial 9-limb carry chains of
// update_fg / update_de (the one-lane form's critical path) are gone.
__device__ __forceinline__ int32_t lane_limb(const int32_t v[9], int li) {
    int32_t r = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) r = li == k ? v[k] : r;
    return r;
}
// (sum_i c_i 2^(30 i)) / 2^30 for c divisible by 2^30, limb i of c on lane i (lane 9 holds 0)
__device__ __forceinline__ int32_t div30_lanes(int64_t c, bool top) {
    const int32_t lo = (int32_t)((uint32_t)c & SBFT_M30);
    const int32_t lo_up = __builtin_amdgcn_update_dpp(0, lo, 0x101, 0xf, 0xf, true);  // row_shl:1: lane i+1's
    const int64_t x = (c >> 30) + (int64_t)lo_up;     // limb i of the quotient, |.| < 2^32
    const int32_t lo2 = top ? (int32_t)x : (int32_t)((uint32_t)x & SBFT_M30);
    const int32_t hi2 = top ? 0 : (int32_t)(x >> 30);  // in [-4, 4]
    const int32_t hi_dn = __builtin_amdgcn_update_dpp(0, hi2, 0x111, 0xf, 0xf, true);  // row_shr:1: lane i-1's
    return lo2 + hi_dn;
}
__device__ __forceinline__ void inv_mod_wave(uint32_t out[8], const uint32_t x[8], const uint32_t* tab, bool P,
                                             const uint32_t* c = nullptr) {
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const bool on = lane < 9, top = lane == 8;
    int32_t M[9];
    mod30(M, P);
    s30 xs, cs;
    pack30(xs, x);
    if (c) {
        pack30(cs, c);
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) cs.v[i] = i == 0 ? 1 : 0;
    }
    const int32_t m_i = on ? lane_limb(M, lane) : 0;
    int32_t f_i = m_i, g_i = on ? lane_limb(xs.v, lane) : 0, d_i = 0, e_i = on ? lane_limb(cs.v, lane) : 0;
    const uint32_t minv = P ? SBFT_PINV30 : SBFT_NINV30;
    int32_t delta = 1;
#if SBFT_INV_PIPE
    // pipelined as inv_mod: the next batch's divsteps start from the low limb of T (f, g) / 2^30
    // (limbs 0 and 1 of f and g), ahead of this batch's lane-parallel updates
    int32_t u, v, q, r;
    delta = divsteps30(delta, (uint32_t)__builtin_amdgcn_readlane(f_i, 0), (uint32_t)__builtin_amdgcn_readlane(g_i, 0),
                       tab, u, v, q, r);
    SBFT_UNROLL1
    for (int batch = 0; batch < 26; ++batch) {
        if (__builtin_amdgcn_ballot_w64(g_i != 0) == 0) break;  // g == 0
        const int32_t f0 = __builtin_amdgcn_readlane(f_i, 0), g0 = __builtin_amdgcn_readlane(g_i, 0);
        const int32_t f1 = __builtin_amdgcn_readlane(f_i, 1), g1 = __builtin_amdgcn_readlane(g_i, 1);
        const int64_t lf = (((int64_t)u * f0 + (int64_t)v * g0) >> 30) + (int64_t)u * f1 + (int64_t)v * g1;
        const int64_t lg = (((int64_t)q * f0 + (int64_t)r * g0) >> 30) + (int64_t)q * f1 + (int64_t)r * g1;
        int32_t u2, v2, q2, r2;
        const int32_t delta2 = divsteps30(delta, (uint32_t)lf, (uint32_t)lg, tab, u2, v2, q2, r2);
#else
    SBFT_UNROLL1
    for (int batch = 0; batch < 26; ++batch) {
        if (__builtin_amdgcn_ballot_w64(g_i != 0) == 0) break;  // g == 0
        const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane(f_i, 0), g0 = (uint32_t)__builtin_amdgcn_readlane(g_i, 0);
        int32_t u, v, q, r;
        delta = divsteps30(delta, f0, g0, tab, u, v, q, r);
#endif
        const int32_t d0 = __builtin_amdgcn_readlane(d_i, 0), e0 = __builtin_amdgcn_readlane(e_i, 0);
        const int64_t cd0 = (int64_t)u * d0 + (int64_t)v * e0, ce0 = (int64_t)q * d0 + (int64_t)r * e0;
        const int32_t md = (int32_t)((0u - (uint32_t)cd0 * minv) & SBFT_M30);
        const int32_t me = (int32_t)((0u - (uint32_t)ce0 * minv) & SBFT_M30);
        const int64_t cf = mac(mac(0, u, f_i), v, g_i);
        const int64_t cg = mac(mac(0, q, f_i), r, g_i);
        const int64_t cd = mac(mac(mac(0, u, d_i), v, e_i), md, m_i);
        const int64_t ce = mac(mac(mac(0, q, d_i), r, e_i), me, m_i);
        f_i = div30_lanes(cf, top);
        g_i = div30_lanes(cg, top);
        d_i = div30_lanes(cd, top);
        e_i = div30_lanes(ce, top);
        if (!on) f_i = g_i = d_i = e_i = 0;
#if SBFT_INV_PIPE
        delta = delta2;
        u = u2;
        v = v2;
        q = q2;
        r = r2;
#endif
    }
    s30 f, d;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        f.v[i] = __builtin_amdgcn_readlane(f_i, i);
        d.v[i] = __builtin_amdgcn_readlane(d_i, i);
    }
    add_kn(f, 0, P);  // canonical limbs: f = +-1
    if (f.v[8] < 0)
        for (int i = 0; i < 9; ++i) d.v[i] = -d.v[i];
    add_kn(d, 0, P);
    reduce_unpack(out, d, P);
}

// inv_mod on a lane pair (2t, 2t + 1) that holds the same x (the half kernel's table build: both
// lanes of a ladder pair invert the same z c). The even lane keeps (f, g), the odd lane (d, e),
// and each batch updates both with ONE update_de per lane: on (f, g) the low 30 bits of T (f, g)
// are zero, so the correction multiple update_de computes there is 0 and the update is
// update_fg's exact division. The divsteps run on both lanes from the even lane's low words (two
// DPP moves per batch, as the g == 0 test). Per batch one 9-limb update instead of two; the
// batches, divsteps and result are inv_mod's (c = 1). A pair's two lanes leave the loop together.
__device__ __forceinline__ int32_t pair_even(int32_t x) {  // the even lane's x, in both lanes
    return __builtin_amdgcn_mov_dpp(x, 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
}
__device__ __forceinline__ void inv_mod_pair(uint32_t out[8], const uint32_t x[8], const uint32_t* tab, bool P,
                                             bool odd) {
    int32_t M[9];
    mod30(M, P);
    s30 xs, a, b;  // even lane: a = f, b = g; odd lane: a = d, b = e
    pack30(xs, x);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = odd ? 0 : M[i];
        b.v[i] = odd ? (i == 0 ? 1 : 0) : xs.v[i];
    }
    int32_t u, v, q, r;
    int32_t delta = divsteps30(1, (uint32_t)M[0], (uint32_t)xs.v[0], tab, u, v, q, r);
    SBFT_UNROLL1
    for (int batch = 0; batch < 26; ++batch) {
        if (pair_even(is_zero30(b) ? 1 : 0)) break;  // g == 0
        // the next batch's divsteps from the low limb of T (f, g) / 2^30 (the even lane's)
        const int64_t lf = (mac(mac(0, u, a.v[0]), v, b.v[0]) >> 30) + (int64_t)u * a.v[1] + (int64_t)v * b.v[1];
        const int64_t lg = (mac(mac(0, q, a.v[0]), r, b.v[0]) >> 30) + (int64_t)q * a.v[1] + (int64_t)r * b.v[1];
        const uint32_t lf0 = (uint32_t)pair_even((int32_t)((uint32_t)lf & SBFT_M30));
        const uint32_t lg0 = (uint32_t)pair_even((int32_t)((uint32_t)lg & SBFT_M30));
        int32_t u2, v2, q2, r2;
        const int32_t delta2 = divsteps30(delta, lf0, lg0, tab, u2, v2, q2, r2);
        update_de(a, b, u, v, q, r, P);
        delta = delta2;
        u = u2;
        v = v2;
        q = q2;
        r = r2;
    }
    // f = +-1 (the even lane's a): x^-1 = f d, on the odd lane
    if (pair_even(a.v[8] < 0 ? 1 : 0)) {
#pragma unroll
        for (int i = 0; i < 9; ++i) a.v[i] = -a.v[i];
        add_kn(a, 0, P);
    }
    uint32_t o[8];
    reduce_unpack(o, a, P);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int32_t)o[i], 0xF5, 0xF, 0xF, false);
}
#endif

#if defined(__HIPCC__)
__device__ __constant__ static const uint32_t C_DIVSTEP5[SBFT_DIVSTEP5_WORDS] = SBFT_DIVSTEP5_TABLE;
// Copy the transition table into LDS (all threads of the block; ends with a barrier).
__device__ __forceinline__ void stage_divstep_table(uint32_t* lds) {
    for (uint32_t i = threadIdx.x; i < SBFT_DIVSTEP5_WORDS / 4; i += blockDim.x)
        reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(C_DIVSTEP5)[i];
    __syncthreads();
}
#endif

}  // namespace inv
}  // namespace sbft
