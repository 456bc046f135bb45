// p256_field.hpp — P-256 field (mod p) and scalar (mod n) arithmetic for gfx950.
//
// Representation: 8 x 32-bit limbs, little-endian, one field element per lane
// (VALU integer work; MFMA is deliberately not used — see DESIGN.md). Measured on
// MI355X: v_mad_u64_u32 issues at ~34 T lane-ops/s, ~87% of the plain integer
// VALU rate (tools/valu_peak.hip), so the design goal is the fewest VALU
// instructions per product, not the fewest multiplies.
//
// Mod p: Montgomery form (R = 2^256) with the sparse reduction that P-256 allows:
// -p^-1 = 1 (mod 2^32), so the reduction multiplier of each word IS the word, and
// m*p = m*2^256 - m*2^224 + m*2^192 + m*2^96 - m becomes four 32-bit adds per
// column instead of eight products. Values are kept lazily reduced in [0, 2^256);
// fp_canon() maps to [0, p) where an exact comparison is needed.
//
// Mod n: generic product-scanning Montgomery (n has no special form).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sbft {

typedef uint32_t u32;
typedef uint64_t u64;

struct fe {
    u32 v[8];
};

#define SBFT_DEV __device__ __forceinline__

// ---------------------------------------------------------------- primitives
// acc += a*b with the 64-bit carry-out added into c2 (v_mad_u64_u32 carry-out
// lands in an SGPR lane mask, v_addc folds it back into a VGPR).
SBFT_DEV void madc(u64& acc, u32& c2, u32 a, u32 b) {
    u64 cc;
    asm(
        "v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "v_addc_co_u32 %2, vcc, 0, %2, %1"
        : "+v"(acc), "=&s"(cc), "+v"(c2)
        : "v"(a), "v"(b)
        : "vcc");
}
// acc += a*b, c2 = carry-out (first capture of a column: no zero-initialised c2 needed)
SBFT_DEV void madc_first(u64& acc, u32& c2, u32 a, u32 b) {
    u64 cc;
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "v_addc_co_u32 %2, vcc, 0, 0, %1"
        : "+v"(acc), "=&s"(cc), "=v"(c2)
        : "v"(a), "v"(b)
        : "vcc");
}
// acc + x (x zero-extended), one instruction
SBFT_DEV u64 mad1(u32 x, u64 acc) {
    u64 r, cc;
    asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(r), "=s"(cc) : "v"(x), "v"(acc));
    return r;
}
// acc + x (x sign-extended), one instruction
SBFT_DEV u64 madi1(u32 x, u64 acc) {
    u64 r, cc;
    asm("v_mad_i64_i32 %0, %1, %2, 1, %3" : "=v"(r), "=s"(cc) : "v"(x), "v"(acc));
    return r;
}
// zero-extend to a 64-bit register pair, one instruction
SBFT_DEV u64 z64(u32 x) {
    u64 r, cc;
    asm("v_mad_u64_u32 %0, %1, %2, 1, 0" : "=v"(r), "=s"(cc) : "v"(x));
    return r;
}
SBFT_DEV u32 lo32(u64 x) { return (u32)x; }
SBFT_DEV u32 hi32(u64 x) { return (u32)(x >> 32); }

// 256 x 256 -> 512 product, product scanning (Comba) with a 96-bit column accumulator.
SBFT_DEV void mul512(u32 t[16], const fe& a, const fe& b) {
    u64 acc = 0;
    u32 c2 = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        int nprod = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = k - i;
            if (j < 0 || j > 7) continue;
            // The carry-in can reach ~2^35, so even a column's first product may carry out
            // (limbs near 2^32-1): every product captures its carry.
            if (nprod == 0 && k == 0) acc = (u64)a.v[i] * b.v[j];
            else if (nprod == 0) madc_first(acc, c2, a.v[i], b.v[j]);
            else madc(acc, c2, a.v[i], b.v[j]);
            ++nprod;
        }
        if (nprod == 1 && k == 0) c2 = 0;
        t[k] = lo32(acc);
        acc = (acc >> 32) | ((u64)c2 << 32);
        c2 = 0;
    }
    t[15] = lo32(acc);
}

// Squaring: off-diagonal triangle once (28 products), doubled by a one-bit funnel shift
// (v_alignbit), then the 8 diagonal squares added pairwise with one v_mad_u64_u32 each and
// the carry chained through SGPR lane masks.
SBFT_DEV void sqr512(u32 t[16], const fe& a) {
    u32 x[16];
    u64 acc = 0;
    u32 c2 = 0;
    x[0] = 0;
#pragma unroll
    for (int k = 1; k < 14; ++k) {
        int nprod = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = k - i;
            if (j <= i || j > 7) continue;
            if (nprod == 0 && k == 1) acc = (u64)a.v[i] * a.v[j];
            else if (nprod == 0) madc_first(acc, c2, a.v[i], a.v[j]);
            else madc(acc, c2, a.v[i], a.v[j]);
            ++nprod;
        }
        if (nprod == 1 && k == 1) c2 = 0;
        x[k] = lo32(acc);
        acc = (acc >> 32) | ((u64)c2 << 32);
        c2 = 0;
    }
    x[14] = lo32(acc);
    x[15] = hi32(acc);
    // x2 = 2x (x < 2^511, so no bit is lost)
    u32 d[16];
    d[0] = 0;
#pragma unroll
    for (int i = 1; i < 16; ++i) d[i] = __builtin_amdgcn_alignbit(x[i], x[i - 1], 31);
    u64 cin = 0;  // lane mask
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 pair = ((u64)d[2 * k + 1] << 32) | d[2 * k];
        u64 sum, c1, c3;
        asm("v_mad_u64_u32 %0, %1, %2, %2, %3" : "=v"(sum), "=s"(c1) : "v"(a.v[k]), "v"(pair));
        u32 lo = lo32(sum), hi = hi32(sum);
        if (k == 0) {
            t[0] = lo;
            t[1] = hi;
            cin = c1;
            continue;
        }
        asm("v_addc_co_u32 %0, %2, %0, 0, %3\n\t"
            "v_addc_co_u32 %1, %2, %1, 0, %2"
            : "+v"(lo), "+v"(hi), "=&s"(c3)
            : "s"(cin));
        t[2 * k] = lo;
        t[2 * k + 1] = hi;
        cin = c1 | c3;
    }
}


// ------------------------------------------------------ carry-chain primitives
// Explicit v_add_co / v_addc / v_sub_co / v_subb chains: the compiler's own lowering of
// 64-bit C arithmetic costs ~4 instructions per limb here, these cost 1. Carries and
// borrows leave as wave lane masks (SGPR pairs), so "any lane needs a correction" is a
// plain scalar test.
typedef u64 lmask;

// r += b (in place), returns the carry-out lane mask
SBFT_DEV lmask add8_ip(fe& r, const fe& b) {
    lmask c;
    asm("v_add_co_u32 %0, vcc, %0, %9\n\t"
        "v_addc_co_u32 %1, vcc, %1, %10, vcc\n\t"
        "v_addc_co_u32 %2, vcc, %2, %11, vcc\n\t"
        "v_addc_co_u32 %3, vcc, %3, %12, vcc\n\t"
        "v_addc_co_u32 %4, vcc, %4, %13, vcc\n\t"
        "v_addc_co_u32 %5, vcc, %5, %14, vcc\n\t"
        "v_addc_co_u32 %6, vcc, %6, %15, vcc\n\t"
        "v_addc_co_u32 %7, vcc, %7, %16, vcc\n\t"
        "s_mov_b64 %8, vcc"
        : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
          "+v"(r.v[6]), "+v"(r.v[7]), "=s"(c)
        : "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]),
          "v"(b.v[7])
        : "vcc");
    return c;
}
// r -= b (in place), returns the borrow-out lane mask
SBFT_DEV lmask sub8_ip(fe& r, const fe& b) {
    lmask c;
    asm("v_sub_co_u32 %0, vcc, %0, %9\n\t"
        "v_subb_co_u32 %1, vcc, %1, %10, vcc\n\t"
        "v_subb_co_u32 %2, vcc, %2, %11, vcc\n\t"
        "v_subb_co_u32 %3, vcc, %3, %12, vcc\n\t"
        "v_subb_co_u32 %4, vcc, %4, %13, vcc\n\t"
        "v_subb_co_u32 %5, vcc, %5, %14, vcc\n\t"
        "v_subb_co_u32 %6, vcc, %6, %15, vcc\n\t"
        "v_subb_co_u32 %7, vcc, %7, %16, vcc\n\t"
        "s_mov_b64 %8, vcc"
        : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
          "+v"(r.v[6]), "+v"(r.v[7]), "=s"(c)
        : "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]),
          "v"(b.v[7])
        : "vcc");
    return c;
}
// r -= (lane in mask ? p : 0), in place; returns the borrow-out lane mask.
// p = [ffffffff ffffffff ffffffff 0 0 0 1 ffffffff] (little-endian limbs).
SBFT_DEV lmask subp_ip(fe& r, lmask mask) {
    lmask c;
    u32 m, t;
    asm("v_cndmask_b32 %8, 0, -1, %11\n\t"
        "v_cndmask_b32 %9, 0, 1, %11\n\t"
        "v_sub_co_u32 %0, vcc, %0, %8\n\t"
        "v_subb_co_u32 %1, vcc, %1, %8, vcc\n\t"
        "v_subb_co_u32 %2, vcc, %2, %8, vcc\n\t"
        "v_subb_co_u32 %3, vcc, %3, 0, vcc\n\t"
        "v_subb_co_u32 %4, vcc, %4, 0, vcc\n\t"
        "v_subb_co_u32 %5, vcc, %5, 0, vcc\n\t"
        "v_subb_co_u32 %6, vcc, %6, %9, vcc\n\t"
        "v_subb_co_u32 %7, vcc, %7, %8, vcc\n\t"
        "s_mov_b64 %10, vcc"
        : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
          "+v"(r.v[6]), "+v"(r.v[7]), "=&v"(m), "=&v"(t), "=s"(c)
        : "s"(mask)
        : "vcc");
    return c;
}
// r += (lane in mask ? p : 0), in place; returns the carry-out lane mask.
SBFT_DEV lmask addp_ip(fe& r, lmask mask) {
    lmask c;
    u32 m, t;
    asm("v_cndmask_b32 %8, 0, -1, %11\n\t"
        "v_cndmask_b32 %9, 0, 1, %11\n\t"
        "v_add_co_u32 %0, vcc, %0, %8\n\t"
        "v_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
        "v_addc_co_u32 %2, vcc, %2, %8, vcc\n\t"
        "v_addc_co_u32 %3, vcc, %3, 0, vcc\n\t"
        "v_addc_co_u32 %4, vcc, %4, 0, vcc\n\t"
        "v_addc_co_u32 %5, vcc, %5, 0, vcc\n\t"
        "v_addc_co_u32 %6, vcc, %6, %9, vcc\n\t"
        "v_addc_co_u32 %7, vcc, %7, %8, vcc\n\t"
        "s_mov_b64 %10, vcc"
        : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
          "+v"(r.v[6]), "+v"(r.v[7]), "=&v"(m), "=&v"(t), "=s"(c)
        : "s"(mask)
        : "vcc");
    return c;
}
// r -= top * p for a per-lane top in {0, 1} (Montgomery reduction tail).
SBFT_DEV void subp_top(fe& r, u32 top) {
    u32 m;
    asm("v_sub_u32 %8, 0, %9\n\t"
        "v_sub_co_u32 %0, vcc, %0, %8\n\t"
        "v_subb_co_u32 %1, vcc, %1, %8, vcc\n\t"
        "v_subb_co_u32 %2, vcc, %2, %8, vcc\n\t"
        "v_subb_co_u32 %3, vcc, %3, 0, vcc\n\t"
        "v_subb_co_u32 %4, vcc, %4, 0, vcc\n\t"
        "v_subb_co_u32 %5, vcc, %5, 0, vcc\n\t"
        "v_subb_co_u32 %6, vcc, %6, %9, vcc\n\t"
        "v_subb_co_u32 %7, vcc, %7, %8, vcc"
        : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
          "+v"(r.v[6]), "+v"(r.v[7]), "=&v"(m)
        : "v"(top)
        : "vcc");
}

// ------------------------------------------------------------------ mod p
__device__ __constant__ static const u32 P256_P[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0,
                                                      0,           0,           1,           0xffffffffu};

// Montgomery reduction t * 2^-256 mod p, t < 2^512 -> [0, 2^256).
// Column k of t + sum_i m_i * p * 2^(32 i) receives +m_{k-3} +m_{k-6} -m_{k-7} +m_{k-8}
// (the -m_k term zeroes the low word and is implicit); m_k = column k for k < 8.
SBFT_DEV void fp_redc(fe& r, const u32 t[16]) {
    const u32 m0 = t[0], m1 = t[1], m2 = t[2];
    u64 c;
    c = mad1(m0, z64(t[3]));
    const u32 m3 = lo32(c);
    c = madi1(hi32(c), mad1(m1, z64(t[4])));
    const u32 m4 = lo32(c);
    c = madi1(hi32(c), mad1(m2, z64(t[5])));
    const u32 m5 = lo32(c);
    c = madi1(hi32(c), mad1(m0, mad1(m3, z64(t[6]))));
    const u32 m6 = lo32(c);
    c = madi1(hi32(c), mad1(m1, mad1(m4, z64(t[7])))) - m0;
    const u32 m7 = lo32(c);
    u32 o[8];
    c = madi1(hi32(c), mad1(m0, mad1(m2, mad1(m5, z64(t[8]))))) - m1;
    o[0] = lo32(c);
    c = madi1(hi32(c), mad1(m1, mad1(m3, mad1(m6, z64(t[9]))))) - m2;
    o[1] = lo32(c);
    c = madi1(hi32(c), mad1(m2, mad1(m4, mad1(m7, z64(t[10]))))) - m3;
    o[2] = lo32(c);
    c = madi1(hi32(c), mad1(m3, mad1(m5, z64(t[11])))) - m4;
    o[3] = lo32(c);
    c = madi1(hi32(c), mad1(m4, mad1(m6, z64(t[12])))) - m5;
    o[4] = lo32(c);
    c = madi1(hi32(c), mad1(m5, mad1(m7, z64(t[13])))) - m6;
    o[5] = lo32(c);
    c = madi1(hi32(c), mad1(m6, z64(t[14]))) - m7;
    o[6] = lo32(c);
    c = madi1(hi32(c), mad1(m7, z64(t[15])));
    o[7] = lo32(c);
    // value = o + top*2^256 < 2^256 + p; subtract top*p.
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = o[k];
    subp_top(r, hi32(c));
}

SBFT_DEV void fp_mul(fe& r, const fe& a, const fe& b) {
    u32 t[16];
    mul512(t, a, b);
    fp_redc(r, t);
}
SBFT_DEV void fp_sqr(fe& r, const fe& a) {
    u32 t[16];
    sqr512(t, a);
    fp_redc(r, t);
}

// r = a + (mask ? k : 0) over 8 limbs; returns the carry-out.
SBFT_DEV u32 add_masked_p(fe& r, const fe& a, u32 mask) {
    const u32 top = mask & 1u;
    const u32 pm[8] = {mask, mask, mask, 0, 0, 0, top, mask};
    u64 c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c = (u64)a.v[k] + pm[k] + c;
        r.v[k] = lo32(c);
        c >>= 32;
    }
    return (u32)c;
}
SBFT_DEV u32 sub_masked_p(fe& r, const fe& a, u32 mask) {
    const u32 top = mask & 1u;
    const u32 pm[8] = {mask, mask, mask, 0, 0, 0, top, mask};
    u64 b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 d = (u64)a.v[k] - pm[k] - b;
        r.v[k] = lo32(d);
        b = d >> 63;
    }
    return (u32)b;
}

// a + b mod p, inputs and output in [0, 2^256): 8-limb add, subtract p on carry-out, and a
// second subtraction in the (rare) case the first did not borrow (value was >= 2^256 + p).
SBFT_DEV void fp_add(fe& r, const fe& a, const fe& b) {
    fe s = a;
    const lmask c = add8_ip(s, b);
    const lmask bw = subp_ip(s, c);
    const lmask again = c & ~bw;
    if (__builtin_expect(again != 0, 0)) subp_ip(s, again);
    r = s;
}
// a - b mod p, inputs and output in [0, 2^256): add p back on borrow, twice if b >= p made
// a - b + p still negative (rare).
SBFT_DEV void fp_sub(fe& r, const fe& a, const fe& b) {
    fe d = a;
    const lmask bw = sub8_ip(d, b);
    const lmask c = addp_ip(d, bw);
    const lmask again = bw & ~c;
    if (__builtin_expect(again != 0, 0)) addp_ip(d, again);
    r = d;
}
// [0, 2^256) -> [0, p)
SBFT_DEV void fp_canon(fe& r, const fe& a) {
    fe t;
    const u32 borrow = sub_masked_p(t, a, 0xffffffffu);
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = borrow ? a.v[k] : t.v[k];
}
SBFT_DEV bool fe_is_zero_raw(const fe& a) {
    u32 o = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) o |= a.v[k];
    return o == 0;
}
// a == 0 (mod p) for a lazily reduced value: a == 0 or a == p.
SBFT_DEV bool fp_is_zero(const fe& a) {
    u32 z = 0, q = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        z |= a.v[k];
        q |= a.v[k] ^ ((k < 3 || k == 7) ? 0xffffffffu : (k == 6 ? 1u : 0u));
    }
    return z == 0 || q == 0;
}
SBFT_DEV bool fe_eq(const fe& a, const fe& b) {
    u32 d = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d |= a.v[k] ^ b.v[k];
    return d == 0;
}
// a < m for 8-limb values
SBFT_DEV bool fe_lt(const fe& a, const u32* m) {
    u64 b = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 d = (u64)a.v[k] - m[k] - b;
        b = d >> 63;
    }
    return b != 0;
}

// ------------------------------------------------------------------ mod n
__device__ __constant__ static const u32 P256_N[8] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                                      0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
#define P256_N_PRIME 0xee00bc4fu /* -n^-1 mod 2^32 */

// Montgomery product mod n (R = 2^256), product scanning with interleaved m*n.
// Inputs < 2^256, output in [0, 2^256) (congruent, conditionally reduced once).
SBFT_DEV void fn_mul(fe& r, const fe& a, const fe& b) {
    u32 m[8];
    u32 o[8];
    u64 acc = 0;
    u32 c2 = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        int nprod = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = k - i;
            if (j < 0 || j > 7) continue;
            if (nprod == 0 && k == 0) acc = (u64)a.v[i] * b.v[j];
            else if (nprod == 0) madc_first(acc, c2, a.v[i], b.v[j]);
            else madc(acc, c2, a.v[i], b.v[j]);
            ++nprod;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int j = k - i;
            if (i >= k || j < 0 || j > 7) continue;
            if (nprod == 0) madc_first(acc, c2, m[i], P256_N[j]);
            else madc(acc, c2, m[i], P256_N[j]);
            ++nprod;
        }
        if (k < 8) {
            m[k] = lo32(acc) * P256_N_PRIME;
            if (nprod == 0) madc_first(acc, c2, m[k], P256_N[0]);  // low word becomes 0
            else madc(acc, c2, m[k], P256_N[0]);
            ++nprod;
        } else {
            o[k - 8] = lo32(acc);
        }
        if (nprod == 0) c2 = 0;
        if (k < 15) acc = (acc >> 32) | ((u64)c2 << 32);  // next column's first product resets c2
    }
    // value = o + hi*2^256 (hi in {0,1}); subtract n once if hi.
    const u32 top = hi32(acc);
    const u32 mask = 0u - top;
    u64 bw = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 d = (u64)o[k] - (P256_N[k] & mask) - bw;
        r.v[k] = lo32(d);
        bw = d >> 63;
    }
}
// [0, 2^256) -> [0, n)
SBFT_DEV void fn_canon(fe& r, const fe& a) {
    fe t;
    u64 bw = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 d = (u64)a.v[k] - P256_N[k] - bw;
        t.v[k] = lo32(d);
        bw = d >> 63;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = bw ? a.v[k] : t.v[k];
}

}  // namespace sbft
