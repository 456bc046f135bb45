// p256_point.hpp — P-256 group arithmetic shared by the verify and sign kernels:
// Jacobian points (Montgomery coordinates mod p), exception-safe additions, the scalar
// inversion mod n and the field inversion mod p.
#pragma once
#include "p256_field.hpp"
#include "p256_tables.inc"

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
// Verify-side fixed-base table: [k]G, k = 1..128 (signed radix-256 windows), 8 KiB, staged
// into LDS once per workgroup.
#define GODD8_WORDS (2 * 8 * P256_GODD8_ENTRIES)
__device__ __constant__ static const u32 C_GODD8[GODD8_WORDS] = P256_GODD8_DATA;
__device__ __constant__ static const u32 C_G2X[8] = P256_G2X_LIMBS;
__device__ __constant__ static const u32 C_G2Y[8] = P256_G2Y_LIMBS;

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


// ---- lean additions for the verify loop (signed-odd digits: every add is live) ----
// acc += b with no case analysis. If H == 0 (acc == +-b: a doubling or a cancellation to
// infinity) the result is garbage and `exc` is raised; the caller re-verifies such tuples
// with the general routines (p256_verify.hip fixup kernel). Rare: adversarial inputs or
// scalars whose partial sums collide.
SBFT_DEV void pt_add_jac_lean(jp& acc, bool& exc, const jp& b) {
    fe z1z1, u2, s2, t, u1, s1, h, rr;
    fp_sqr(z1z1, acc.z);
    fp_mul(u2, b.x, z1z1);
    fp_mul(t, acc.z, z1z1);
    fp_mul(s2, b.y, t);
    fp_sqr(t, b.z);  // z2z2
    fp_mul(u1, acc.x, t);
    fp_mul(t, b.z, t);
    fp_mul(s1, acc.y, t);
    fp_sub(h, u2, u1);
    fp_sub(rr, s2, s1);
    exc = exc || fp_is_zero(h);
    fe hh, hhh;
    fp_sqr(hh, h);
    fp_mul(hhh, hh, h);
    fp_mul(u1, u1, hh);  // v = U1 H^2
    fp_mul(t, acc.z, b.z);
    fp_mul(acc.z, t, h);
    fp_sqr(t, rr);
    fp_sub(t, t, hhh);
    fp_sub(t, t, u1);
    fp_sub(acc.x, t, u1);
    fp_sub(t, u1, acc.x);
    fp_mul(t, rr, t);
    fp_mul(s1, s1, hhh);
    fp_sub(acc.y, t, s1);
}

// acc += (x2, y2) affine, same structure (8M + 3S on the common path).
SBFT_DEV void pt_add_aff_lean(jp& acc, bool& exc, const fe& x2, const fe& y2) {
    fe z1z1, u2, s2, h, rr;
    fp_sqr(z1z1, acc.z);
    fp_mul(u2, x2, z1z1);
    fp_mul(s2, acc.z, z1z1);
    fp_mul(s2, y2, s2);
    fp_sub(h, u2, acc.x);
    fp_sub(rr, s2, acc.y);
    exc = exc || fp_is_zero(h);
    fe hh, hhh;
    fp_sqr(hh, h);
    fp_mul(hhh, hh, h);
    fp_mul(u2, acc.x, hh);  // v = X1 H^2
    fp_mul(acc.z, acc.z, h);
    fp_sqr(s2, rr);
    fp_sub(s2, s2, hhh);
    fp_sub(s2, s2, u2);
    fp_sub(acc.x, s2, u2);
    fp_sub(s2, u2, acc.x);
    fp_mul(s2, rr, s2);
    fp_mul(hhh, acc.y, hhh);
    fp_sub(acc.y, s2, hhh);
}

// Radix-16 Booth digit from the 5-bit window (b3 b2 b1 b0 b-1): value in [-8, 8].
SBFT_DEV int booth(u32 w5) { return (int)((w5 >> 1) + (w5 & 1u)) - (int)((w5 >> 4) << 4); }
// Radix-256 Booth digit from the 9-bit window (b7..b0 b-1): value in [-128, 128].
SBFT_DEV int booth8(u32 w9) { return (int)((w9 >> 1) + (w9 & 1u)) - (int)((w9 >> 8) << 8); }


// Field inverse a^(p-2) mod p, Montgomery domain in and out (255 S + 12 M).
// p-2 = FFFFFFFF 00000001 00000000 00000000 00000000 FFFFFFFF FFFFFFFF FFFFFFFD
SBFT_DEV void fp_sqr_n(fe& r, int count) {
#pragma unroll 1
    for (int i = 0; i < count; ++i) fp_sqr(r, r);
}
SBFT_DEV void fp_inv(fe& r, const fe& a) {
    fe t2, t3, t6, t12, t15, t30, t32, t;
    fp_sqr(t, a);
    fp_mul(t2, t, a);  // 2^2-1
    fp_sqr(t, t2);
    fp_mul(t3, t, a);  // 2^3-1
    t = t3;
    fp_sqr_n(t, 3);
    fp_mul(t6, t, t3);
    t = t6;
    fp_sqr_n(t, 6);
    fp_mul(t12, t, t6);
    t = t12;
    fp_sqr_n(t, 3);
    fp_mul(t15, t, t3);
    t = t15;
    fp_sqr_n(t, 15);
    fp_mul(t30, t, t15);
    t = t30;
    fp_sqr_n(t, 2);
    fp_mul(t32, t, t2);   // FFFFFFFF
    t = t32;
    fp_sqr_n(t, 32);
    fp_mul(t, t, a);      // FFFFFFFF 00000001
    fp_sqr_n(t, 128);
    fp_mul(t, t, t32);    // ... 00000000 x3 FFFFFFFF
    fp_sqr_n(t, 32);
    fp_mul(t, t, t32);    // FFFFFFFF
    fp_sqr_n(t, 30);
    fp_mul(t, t, t30);    // 30 ones
    fp_sqr_n(t, 2);
    fp_mul(r, t, a);      // ...01
}

// a + b mod n, inputs < n, output < n.
SBFT_DEV void fn_add(fe& r, const fe& a, const fe& b) {
    fe s, t;
    u64 c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c = (u64)a.v[k] + b.v[k] + c;
        s.v[k] = lo32(c);
        c >>= 32;
    }
    u64 bw = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 d = (u64)s.v[k] - P256_N[k] - bw;
        t.v[k] = lo32(d);
        bw = d >> 63;
    }
    const bool take_t = (c != 0) || (bw == 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = take_t ? t.v[k] : s.v[k];
}

// [k]G with the radix-16 Booth windows over the LDS copy of C_GTAB (fixed-base, used by
// the signer and key derivation). k < 2^256; result may be infinity (k == 0 mod n).
SBFT_DEV void pt_mul_base(jp& acc, bool& inf, const fe& k, const u32* gtab) {
    inf = true;
    acc.x = fe_zero();
    acc.y = fe_zero();
    acc.z = fe_zero();
    {
        fe gx, gy;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            gx.v[i] = gtab[i];
            gy.v[i] = gtab[8 + i];
        }
        pt_add_aff(acc, inf, gx, gy, (k.v[7] >> 31) != 0);
    }
    fe kk = k;
#pragma unroll 1
    for (int limb = 7; limb >= 0; --limb) {
        const u32 cur = kk.v[7], below = kk.v[6];
#pragma unroll
        for (int i = 7; i > 0; --i) kk.v[i] = kk.v[i - 1];
        kk.v[0] = 0;
        const u64 w = ((u64)cur << 1) | (below >> 31);
#pragma unroll 1
        for (int nib = 7; nib >= 0; --nib) {
#pragma unroll 1
            for (int d = 0; d < 4; ++d) pt_dbl(acc, acc);
            const int dg = booth((u32)(w >> (4 * nib)) & 31u);
            const int m = dg < 0 ? -dg : dg;
            const int base = (m > 0 ? m - 1 : 0) * 16;
            fe gx, gy;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                gx.v[i] = gtab[base + i];
                gy.v[i] = gtab[base + 8 + i];
            }
            if (dg < 0) {
                fe ny;
                fp_sub(ny, fe_zero(), gy);
                gy = ny;
            }
            pt_add_aff(acc, inf, gx, gy, dg != 0);
        }
    }
}

// Big-endian 32-byte store of 8 little-endian limbs.
SBFT_DEV void store_be32(uint8_t* p, const fe& a) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(__builtin_bswap32(a.v[7]), __builtin_bswap32(a.v[6]), __builtin_bswap32(a.v[5]),
                      __builtin_bswap32(a.v[4]));
    q[1] = make_uint4(__builtin_bswap32(a.v[3]), __builtin_bswap32(a.v[2]), __builtin_bswap32(a.v[1]),
                      __builtin_bswap32(a.v[0]));
}

// Registered-key comb tables (p256_keyed.hip builds them; the keyed kernels of p256_keyed.hip
// and p256_verify.hip read them): table[w][j] = j 2^(8w) Q, w = 0..31, j = 0..255 (j = 0: zeros),
// affine, 8 x 32 Montgomery form (R = 2^256) mod p, canonical.
#define COMB_WINDOWS 32
#define COMB_ENTRIES 256
// uint4 units per entry (64 B: x limbs 0..7, y limbs 0..7) and per key table
#define COMB_ENTRY_U4 4
#define COMB_KEY_U4 (COMB_WINDOWS * COMB_ENTRIES * COMB_ENTRY_U4)

// byte w (0..31, little-endian) of a 256-bit value, w lane-varying
#ifndef SBFT_BYTE_OF_REGS
#define SBFT_BYTE_OF_REGS 0  // measured: no gain (profiles/r05ag_byteof_ab.txt)
#endif
// LLVM rewrites this select chain into a 32-B stack array and one indexed scratch load (the keyed
// wave kernel's 36-B private segment). SBFT_BYTE_OF_REGS=1 puts an empty asm after each select to
// keep it in registers (private segment 0); the keyed wave kernel measured 0.1-0.4 us slower that
// way (35.6-35.9 vs 35.3-35.5 us, profiles/r05ag_byteof_ab.txt): the scratch load issues early
// and hides behind the entry loads, the 14 extra VALU per byte do not.
SBFT_DEV u32 byte_of(const fe& a, u32 w) {
    const u32 limb_i = w >> 2;
    u32 limb = a.v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        limb = (limb_i == (u32)k) ? a.v[k] : limb;
#if SBFT_BYTE_OF_REGS
        asm("" : "+v"(limb));
#endif
    }
    return (limb >> (8 * (w & 3))) & 255u;
}

// x(R) mod n == r, projectively; r is the plain (non-Montgomery) 256-bit value in [1, n)
SBFT_DEV bool x_matches_r(const jp& R, const fe& r) {
    const fe r2p = fe_const(C_R2P);
    fe z2, lhs, xc, rm;
    fp_sqr(z2, R.z);
    fp_canon(xc, R.x);
    fp_mul(rm, r, r2p);
    fp_mul(lhs, rm, z2);
    fp_canon(lhs, lhs);
    bool accept = fe_eq(lhs, xc);
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
    return accept;
}

}  // namespace sbft
