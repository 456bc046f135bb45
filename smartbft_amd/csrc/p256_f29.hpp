// p256_f29.hpp — P-256 field arithmetic in radix 2^29 (9 signed limbs) for the verify hot loop.
//
// Why a second representation. With 8 x 32-bit limbs every v_mad_u64_u32 of a product column
// can carry out of its 64-bit accumulator, so each product costs a second instruction (v_addc)
// to catch the carry, and additions need 8-long carry chains plus a conditional subtraction
// of p. With 29-bit limbs a column of up to 9 products (each < 2^58) plus carries stays far
// below 2^63: every product is ONE v_mad_i64_i32 with no carry handling, and additions and
// subtractions are 9 independent v_add/v_sub (no carries, no reduction) because the limbs are
// signed and carry headroom is left in each 32-bit word.
//
// Value:  x = sum_i v[i] * 2^(29 i), v[i] signed 32-bit. Montgomery form mod p with R = 2^261.
// Normal form (every f29_mul / f29_sqr output): v[0..7] in [0, 2^29), v[8] signed, and
// |x| < 2^258 (see the bound in f29_mul).
//
// Reduction. p = 2^256 - 2^224 + 2^192 + 2^96 - 1 in radix 2^29 with non-negative digits above
// digit 0:  p = -1 + 2^9 * B^3 + 2^18 * B^6 + (2^29 - 2^21) * B^7 + (2^24 - 1) * B^8, B = 2^29.
// -p^-1 = 1 (mod 2^29), so the Montgomery multiplier of a column is its own low 29 bits m, and
// m*p adds four single-mad terms to columns k+3, k+6, k+7, k+8 (the -m at column k just
// clears the low bits that the arithmetic shift drops anyway).
//
// Caller contract (checked by the bound comments at each use in p256_verify.hip): for
// f29_mul(a, b) with |a.v[i]| <= A and |b.v[i]| <= B, 9*A*B + 2^60 < 2^63 (A*B <= 2^59.7:
// e.g. 2^29 x 2^30.6), and |a| * |b| < 2^517 so that the output is normal.
#pragma once
#include "p256_field.hpp"
#include "p256_tables.inc"

namespace sbft {

typedef int32_t i32;
typedef int64_t i64;

struct f29 {
    u32 v[9];
};

#define F29_MASK 0x1FFFFFFFu

// acc + a*b (signed 32 x 32 + 64), one v_mad_i64_i32. The empty asm makes the sum opaque so
// the compiler keeps the accumulation a chain of mads instead of re-associating it into a
// tree of 64-bit adds (a real asm v_mad costs an s_nop per instruction: the hazard recognizer
// treats the asm's carry-out SGPR write conservatively).
SBFT_DEV i64 smad(u32 a, u32 b, i64 acc) {
#ifdef SBFT_SMAD_ASM
    i64 r;
    u64 cc;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(acc));
    return r;
#else
    i64 r = (i64)(i32)a * (i64)(i32)b + acc;
    asm("" : "+v"(r));
    return r;
#endif
}
// acc >> 29 (arithmetic). SBFT_SHR_ASM pins it to one v_ashrrev_i64 so the compiler cannot
// fold the shift into the next mad's addend (which costs register-pair moves).
SBFT_DEV i64 sar29(i64 acc) {
#ifdef SBFT_SHR_ASM
    i64 r;
    asm("v_ashrrev_i64 %0, 29, %1" : "=v"(r) : "v"(acc));
    return r;
#else
    return acc >> 29;
#endif
}
// low 29 bits of acc as a limb whose range the compiler cannot see: a limb it proves
// non-negative turns a later sext(a) * sext(b) into a u64 mad plus a sign-correction mad and
// register-pair moves. The asm sits on the freshly masked value (no copy needed).
SBFT_DEV u32 lo29(i64 acc) {
    u32 t = (u32)acc & F29_MASK;
#ifndef SBFT_NO_OPAQUE_LIMBS
    asm("" : "+v"(t));
#endif
    return t;
}
// The reduction multipliers 2^9, 2^18, 2^29 - 2^21, 2^24 - 1, held in SGPRs the compiler cannot
// see through (otherwise m * 2^9 + acc becomes a 64-bit shift, mask and add: 3 instructions).
struct f29_red {
    u32 c9, c18, c7, c8;
};
SBFT_DEV f29_red f29_red_consts() {
    f29_red k = {1u << 9, 1u << 18, 0x1FE00000u, 0x00FFFFFFu};
    asm("" : "+s"(k.c9), "+s"(k.c18), "+s"(k.c7), "+s"(k.c8));
    return k;
}

// Montgomery product a*b*2^-261 mod p (normal form out, see the contract above).
SBFT_DEV void f29_mul(f29& r, const f29& a, const f29& b) {
    const f29_red K = f29_red_consts();
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
            if (j < 0 || j > 8) continue;
            acc = smad(a.v[i], b.v[j], acc);
        }
        if (k >= 3 && k - 3 <= 8) acc = smad(m[k - 3], K.c9, acc);
        if (k >= 6 && k - 6 <= 8) acc = smad(m[k - 6], K.c18, acc);
        if (k >= 7 && k - 7 <= 8) acc = smad(m[k - 7], K.c7, acc);
        if (k >= 8 && k - 8 <= 8) acc = smad(m[k - 8], K.c8, acc);
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
    r.v[8] = (u32)acc;
}

// a^2: off-diagonal products against the doubled operand (one mad each), then the squares.
// f29_sqr_d takes the doubled operand from the caller when it has it already (2Y, 2g in the
// doubling): d must be exactly 2a limb by limb.
SBFT_DEV void f29_sqr_d(f29& r, const f29& a, const f29& d2) {
    const f29_red K = f29_red_consts();
    const u32* d = d2.v;
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
            if (j <= i || j > 8) continue;
            acc = smad(a.v[i], d[j], acc);
        }
        if ((k & 1) == 0) acc = smad(a.v[k >> 1], a.v[k >> 1], acc);
        if (k >= 3 && k - 3 <= 8) acc = smad(m[k - 3], K.c9, acc);
        if (k >= 6 && k - 6 <= 8) acc = smad(m[k - 6], K.c18, acc);
        if (k >= 7 && k - 7 <= 8) acc = smad(m[k - 7], K.c7, acc);
        if (k >= 8 && k - 8 <= 8) acc = smad(m[k - 8], K.c8, acc);
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
    r.v[8] = (u32)acc;
}
SBFT_DEV void f29_sqr(f29& r, const f29& a) {
    f29 d;
#pragma unroll
    for (int i = 0; i < 9; ++i) d.v[i] = a.v[i] << 1;
    f29_sqr_d(r, a, d);
}

// N independent products (job x squares a[x] when bit x of SQ is set) with their mads
// interleaved job by job: back-to-back dependent 64-bit mads cost a wait state (s_nop) on
// gfx950, independent ones issue back to back. Outputs are written after all inputs are read.
template <int N, unsigned SQ>
SBFT_DEV void f29_mulv(f29* const* r, const f29* const* a, const f29* const* b) {
    const f29_red K = f29_red_consts();
    u32 d[N][9];
#pragma unroll
    for (int x = 0; x < N; ++x)
        if ((SQ >> x) & 1u)
#pragma unroll
            for (int i = 0; i < 9; ++i) d[x][i] = a[x]->v[i] << 1;
    u32 m[N][9], o[N][9];
    i64 acc[N];
#pragma unroll
    for (int x = 0; x < N; ++x) acc[x] = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
#pragma unroll
            for (int x = 0; x < N; ++x) {
                if ((SQ >> x) & 1u) {
                    if (j > i && j <= 8) acc[x] = smad(a[x]->v[i], d[x][j], acc[x]);
                } else {
                    if (j >= 0 && j <= 8) acc[x] = smad(a[x]->v[i], b[x]->v[j], acc[x]);
                }
            }
        }
#pragma unroll
        for (int x = 0; x < N; ++x)
            if (((SQ >> x) & 1u) && (k & 1) == 0) acc[x] = smad(a[x]->v[k >> 1], a[x]->v[k >> 1], acc[x]);
#pragma unroll
        for (int x = 0; x < N; ++x) {
            if (k >= 3 && k - 3 <= 8) acc[x] = smad(m[x][k - 3], K.c9, acc[x]);
        }
#pragma unroll
        for (int x = 0; x < N; ++x) {
            if (k >= 6 && k - 6 <= 8) acc[x] = smad(m[x][k - 6], K.c18, acc[x]);
        }
#pragma unroll
        for (int x = 0; x < N; ++x) {
            if (k >= 7 && k - 7 <= 8) acc[x] = smad(m[x][k - 7], K.c7, acc[x]);
        }
#pragma unroll
        for (int x = 0; x < N; ++x) {
            if (k >= 8 && k - 8 <= 8) acc[x] = smad(m[x][k - 8], K.c8, acc[x]);
        }
#pragma unroll
        for (int x = 0; x < N; ++x) {
            if (k < 9) m[x][k] = lo29(acc[x]);
            else o[x][k - 9] = lo29(acc[x]);
            acc[x] = sar29(acc[x]);
        }
    }
#pragma unroll
    for (int x = 0; x < N; ++x) {
        o[x][8] = (u32)acc[x];
#pragma unroll
        for (int i = 0; i < 9; ++i) r[x]->v[i] = o[x][i];
    }
}
SBFT_DEV void f29_mul2(f29& r0, const f29& a0, const f29& b0, f29& r1, const f29& a1, const f29& b1) {
    f29* const r[2] = {&r0, &r1};
    const f29* const a[2] = {&a0, &a1};
    const f29* const b[2] = {&b0, &b1};
    f29_mulv<2, 0u>(r, a, b);
}
SBFT_DEV void f29_mul3(f29& r0, const f29& a0, const f29& b0, f29& r1, const f29& a1, const f29& b1, f29& r2,
                       const f29& a2, const f29& b2) {
    f29* const r[3] = {&r0, &r1, &r2};
    const f29* const a[3] = {&a0, &a1, &a2};
    const f29* const b[3] = {&b0, &b1, &b2};
    f29_mulv<3, 0u>(r, a, b);
}
SBFT_DEV void f29_sqr2(f29& r0, const f29& a0, f29& r1, const f29& a1) {
    f29* const r[2] = {&r0, &r1};
    const f29* const a[2] = {&a0, &a1};
    f29_mulv<2, 3u>(r, a, a);
}

// (a b - c d) 2^-261 mod p with ONE Montgomery reduction: each column sums both products (a's
// terms and c's against -d, in two accumulators so no two dependent mads issue back to back)
// before its reduction step. It replaces two products and a subtraction (the additions' Y3 =
// r (V - X3) - Y1 H^3): 36 reduction mads and 17 (mask, shift) pairs fewer.
// Contract (f29_mul's, with both products in the column): 9 (A B + C D) + 2^60 < 2^63 for the
// limb bounds (A B + C D <= 2^59.6; the uses have 2^29.2 x 2^29.2 + 2^29.2 x 2^29 = 2^59.3), and
// |a b - c d| < 2^518 so that the output is normal (N).
#ifndef SBFT_MULSUB_CHAIN
#define SBFT_MULSUB_CHAIN 0  // 1: both products on one accumulator (no 64-bit add per column)
#endif
SBFT_DEV void f29_mul_sub(f29& r, const f29& a, const f29& b, const f29& c, const f29& d) {
    const f29_red K = f29_red_consts();
    u32 nd[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) nd[i] = 0u - d.v[i];
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        i64 acc1 = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
            if (j < 0 || j > 8) continue;
            acc = smad(a.v[i], b.v[j], acc);
            if (SBFT_MULSUB_CHAIN) acc = smad(c.v[i], nd[j], acc);
            else acc1 = smad(c.v[i], nd[j], acc1);
        }
        if (!SBFT_MULSUB_CHAIN) acc += acc1;
        if (k >= 3 && k - 3 <= 8) acc = smad(m[k - 3], K.c9, acc);
        if (k >= 6 && k - 6 <= 8) acc = smad(m[k - 6], K.c18, acc);
        if (k >= 7 && k - 7 <= 8) acc = smad(m[k - 7], K.c7, acc);
        if (k >= 8 && k - 8 <= 8) acc = smad(m[k - 8], K.c8, acc);
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
    r.v[8] = (u32)acc;
}

#ifndef SBFT_MULSUB
#define SBFT_MULSUB 1  // the additions' Y3 through f29_mul_sub (0: two products + subtraction)
#endif

// ---------------------------------------------------------------- products with addends
// Mont(a b) + sum_t c_t v_t (mod p) in one pass, c_t small signed constants (|c_t v_t limb| <
// 2^34). Montgomery's output comes out of columns 9..17, so adding v 2^261 to the column sums
// adds v to the result exactly: v's limb i goes into column 9 + i, one mad each, after the
// reduction multipliers m[] are taken from columns 0..8. The formulas' "X3 = u^2 - 4 b2",
// "Y3 = al t - 8 g^2" then need no subtraction loop and no separate normalisation:
// f29_fold_top takes the bits at 2^256 and up off the signed top limb (as f29_normalize does)
// and the output is N' (limbs 0..7 in (-2^25, 2^29 + 2^25), limb 8 in [0, 2^24), |x| < 2^257).
// Column contract: f29_mul's (the addend terms are < 2^34 against 2^63 of headroom); value:
// |Mont(a b)| < |a b| 2^-261 + p, plus |sum c_t v_t|, must stay below 2^260 (|h| <= 2^4).
// hmask = 0 skips the fold (the output then stays a plain product's N, for c_t = 0 lanes).
SBFT_DEV void f29_fold_top(f29& r, u32 top, u32 hmask) {
    const i32 h = ((i32)top >> 24) & (i32)hmask;
    r.v[8] = top - ((u32)h << 24);
    r.v[7] += (u32)h << 21;
    r.v[6] = (u32)((i32)r.v[6] + h * -(1 << 18));
    r.v[3] = (u32)((i32)r.v[3] + h * -(1 << 9));
    r.v[0] += (u32)h;
#ifndef SBFT_NO_OPAQUE_LIMBS
#pragma unroll
    for (int i = 0; i < 9; ++i) asm("" : "+v"(r.v[i]));
#endif
}
// Opaque small constants for the addends (SGPRs; a visible -4 becomes shifts and 64-bit adds).
SBFT_DEV u32 f29_kconst(i32 c) {
    u32 k = (u32)c;
    asm("" : "+s"(k));
    return k;
}
// Chain form (the throughput kernel: 4 waves per SIMD hide the dependent mads' wait states).
template <bool SQ, int NA>
SBFT_DEV void f29_mulsq_add(f29& r, const f29& a, const f29& b, const f29* const (&v)[NA], const u32 (&c)[NA]) {
    const f29_red K = f29_red_consts();
    u32 d[9];
    if (SQ)
#pragma unroll
        for (int i = 0; i < 9; ++i) d[i] = a.v[i] << 1;
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
            if (SQ) {
                if (j > i && j <= 8) acc = smad(a.v[i], d[j], acc);
            } else {
                if (j >= 0 && j <= 8) acc = smad(a.v[i], b.v[j], acc);
            }
        }
        if (SQ && (k & 1) == 0) acc = smad(a.v[k >> 1], a.v[k >> 1], acc);
        if (k >= 3 && k - 3 <= 8) acc = smad(m[k - 3], K.c9, acc);
        if (k >= 6 && k - 6 <= 8) acc = smad(m[k - 6], K.c18, acc);
        if (k >= 7 && k - 7 <= 8) acc = smad(m[k - 7], K.c7, acc);
        if (k >= 8 && k - 8 <= 8) acc = smad(m[k - 8], K.c8, acc);
        if (k >= 9)
#pragma unroll
            for (int t = 0; t < NA; ++t) acc = smad(v[t]->v[k - 9], c[t], acc);
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
#pragma unroll
    for (int t = 0; t < NA; ++t) acc = smad(v[t]->v[8], c[t], acc);
    f29_fold_top(r, (u32)acc, ~0u);
}
// Mont(a b - c^2) in one pass (chain form): the square's terms go into the same column sums
// with their signs flipped, c's cross terms as c_i (-2 c_j) and its diagonal as c_i (-c_i), so
// c^2 costs 45 mads and no reduction of its own. nc = -c, nc2 = -2c (limbs), supplied by the
// caller. Column contract: |a_i b_j| < 2^58.2 (9 of them), |c_i 2 c_j| < 2^59 (4 cross + 1
// diagonal per column), reduction terms < 2^58.1: < 2^62.4 with the carry, under 2^63
// (tests/test_f29_bounds.py checks the sums). Output N (limbs 0..7 in [0, 2^29), signed top,
// |r| < 2^258 for |a b - c^2| < 2^518).
SBFT_DEV void f29_mul_sqsub(f29& r, const f29& a, const f29& b, const f29& c, const f29& nc, const f29& nc2) {
    const f29_red K = f29_red_consts();
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
            if (j >= 0 && j <= 8) acc = smad(a.v[i], b.v[j], acc);
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int j = k - i;
            if (j > i && j <= 8) acc = smad(c.v[i], nc2.v[j], acc);
        }
        if ((k & 1) == 0 && (k >> 1) <= 8) acc = smad(c.v[k >> 1], nc.v[k >> 1], acc);
        if (k >= 3 && k - 3 <= 8) acc = smad(m[k - 3], K.c9, acc);
        if (k >= 6 && k - 6 <= 8) acc = smad(m[k - 6], K.c18, acc);
        if (k >= 7 && k - 7 <= 8) acc = smad(m[k - 7], K.c7, acc);
        if (k >= 8 && k - 8 <= 8) acc = smad(m[k - 8], K.c8, acc);
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
    r.v[8] = (u32)acc;
}

// alpha/2 = 3 a' / 2 (mod p) for a product output a' (limbs 0..7 in [0, 2^29), |a'| < 2^256.6):
// s = a' + (a' odd ? p : 0) is even (the value's parity is limb 0's), u = 3 s limb by limb
// (< 2^31.6, unsigned), one carry pass (limbs [0, 2^29 + 5)), then the halving: limb i takes
// u_i >> 1 plus limb i+1's low bit at bit 28 (u_0 is even). Out: limbs 0..7 in [0, 2^29 + 3),
// |out| < 1.5 (2^256.6 + p) < 2^258.1 -- f29_triple's contract.
SBFT_DEV void f29_triple_half(f29& r, const f29& a) {
    const u32 odd = 0u - (a.v[0] & 1u);
    constexpr u32 P29[9] = {0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x000001ffu, 0u, 0u, 0x00040000u, 0x1fe00000u,
                            0x00ffffffu};
    u32 t[9], c[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = (a.v[i] + (P29[i] & odd)) * 3u;
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = t[i] >> 29;  // 3 s_i < 2^31.6: carry 0..5
    u32 w[9];
    w[0] = t[0] & F29_MASK;
#pragma unroll
    for (int i = 1; i < 8; ++i) w[i] = (t[i] & F29_MASK) + c[i - 1];
    w[8] = t[8] + c[7];
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = (w[i] >> 1) + ((w[i + 1] & 1u) << 28);
    r.v[8] = (u32)((i32)w[8] >> 1);
#if !defined(SBFT_NO_OPAQUE_LIMBS) && !defined(SBFT_NO_OPAQUE_NORM)
#pragma unroll
    for (int i = 0; i < 9; ++i) asm("" : "+v"(r.v[i]));
#endif
}

// ILP form (lane pairs: one product per lane per step; see f29_mulsq_ilp below), per-lane
// constants c (VGPRs) and fold mask.
template <bool SQ, int NA>
SBFT_DEV void f29_mulsq_add_ilp(f29& r, const f29& a, const f29& b, const f29* const (&v)[NA], const u32 (&c)[NA],
                                u32 hmask);

SBFT_DEV void f29_add(f29& r, const f29& a, const f29& b) {
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
}
SBFT_DEV void f29_sub(f29& r, const f29& a, const f29& b) {
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] - b.v[i];
}
SBFT_DEV void f29_neg(f29& r, const f29& a) {
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = 0u - a.v[i];
}
// r = c * a for a small constant c (limbs grow by c)
SBFT_DEV void f29_muls(f29& r, const f29& a, u32 c) {
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] * c;
}
// Value-reducing normalisation for a sum like 3u - 4v (|limb| < 2^31, |x| < 2^260) -> N:
//  1. one parallel carry pass: limbs 0..7 into [-4, 2^29 + 4) (limb 8 takes limb 7's carry);
//  2. fold: h = limb8 >> 24 are the bits at 2^256 and up; drop them and add
//     h * (2^256 mod p) = h * (2^224 - 2^192 - 2^96 + 1), i.e. +h<<21 at limb 7, -h<<18 at
//     limb 6, -h<<9 at limb 3, +h at limb 0 (|h| <= 2^5 here, so the limbs move by < 2^26).
// Out: limbs 0..7 in (-2^26, 2^29 + 2^26), limb 8 in [0, 2^24), |x| < 2^257.
SBFT_DEV void f29_normalize(f29& r, const f29& a) {
    u32 c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = (u32)((i32)a.v[i] >> 29);
    f29 t;
    t.v[0] = a.v[0] & F29_MASK;
#pragma unroll
    for (int i = 1; i < 8; ++i) t.v[i] = (a.v[i] & F29_MASK) + c[i - 1];
    const u32 top = a.v[8] + c[7];
    const i32 h = (i32)top >> 24;
    t.v[8] = top & 0x00FFFFFFu;
    t.v[7] += (u32)h << 21;
    t.v[6] = (u32)((i32)t.v[6] + h * -(1 << 18));
    t.v[3] = (u32)((i32)t.v[3] + h * -(1 << 9));
    t.v[0] += (u32)h;
#if !defined(SBFT_NO_OPAQUE_LIMBS) && !defined(SBFT_NO_OPAQUE_NORM)
    // range-opaque like lo29: with the limbs' ranges visible (a masked word plus a small signed
    // carry), ROCm 7.2's lowering of a later sext * sext product miscompiled two inlined
    // back-to-back doublings (tests/test_gpu_field.py::test_f29_point_ops, unrolled loop)
#pragma unroll
    for (int i = 0; i < 9; ++i) asm("" : "+v"(t.v[i]));
#endif
    r = t;
}

// alpha = 3 a' for a product output a' (limbs 0..7 in [0, 2^29), |a'| < 2^256.6): one carry
// pass, no fold. Out: limbs 0..7 in [0, 2^29 + 2), limb 8 = 3 a'_8 + carry (|.| < 2^26.2),
// |alpha| < 2^258.2 -- limb bounds within N', and alpha^2, alpha t (|t| < 2^258.2) stay below
// 2^516.4, so their Montgomery outputs are < 2^256.6 like any product of N' values.
SBFT_DEV void f29_triple(f29& r, const f29& a) {
    u32 t[9], c[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) t[i] = a.v[i] * 3u;
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = t[i] >> 29;  // 3 a_i < 2^30.6: carry 0..2
    r.v[0] = t[0] & F29_MASK;
#pragma unroll
    for (int i = 1; i < 8; ++i) r.v[i] = (t[i] & F29_MASK) + c[i - 1];
    r.v[8] = t[8] + c[7];
#if !defined(SBFT_NO_OPAQUE_LIMBS) && !defined(SBFT_NO_OPAQUE_NORM)
#pragma unroll
    for (int i = 0; i < 9; ++i) asm("" : "+v"(r.v[i]));
#endif
}
#ifndef SBFT_TRIPLE_CARRY
#define SBFT_TRIPLE_CARRY 1  // alpha by f29_triple (0: f29_muls + f29_normalize)
#endif

// ---------------------------------------------------------------- exact zero tests mod p
// Common tail: limbs 0..7 in [0, 2^29), limb 8 signed, |x| < 2^258. The bits at 2^256 and up,
// h = limb8 >> 24 (|h| <= 4), are folded with 2^256 = 2^224 - 2^192 - 2^96 + 1 (mod p):
// y = (x mod 2^256) + h (2^224 - 2^192 - 2^96 + 1) lies in (-p, 2p), so after one carry pass
// x == 0 (mod p) iff y's limbs are all 0 or are p's.
SBFT_DEV bool f29_zero_tail(const u32 (&a)[9]) {
    const i32 h = (i32)a[8] >> 24;
    i32 v[9];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (i32)a[i];
    v[8] = (i32)(a[8] & 0x00FFFFFFu);
    v[7] += h * (1 << 21);
    v[6] -= h * (1 << 18);
    v[3] -= h * (1 << 9);
    v[0] += h;
    i32 c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const i32 x = v[i] + c;
        v[i] = x & (i32)F29_MASK;
        c = x >> 29;
    }
    v[8] += c;
    constexpr u32 P29[9] = {0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x000001ffu, 0u, 0u, 0x00040000u, 0x1fe00000u,
                            0x00ffffffu};
    u32 z = 0, q = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        z |= (u32)v[i];
        q |= (u32)v[i] ^ P29[i];
    }
    return z == 0 || q == 0;
}
// x == 0 (mod p) for x in normal form (an f29_mul / f29_sqr output): exact, ~50 VALU
// instructions, no multiplication (f29_canon_plain costs a product and a subtraction loop).
SBFT_DEV bool f29_zero_mod_p(const f29& a) { return f29_zero_tail(a.v); }
// The same for any x with |limb| < 2^31 and |x| < 2^260 (normalised and carried first).
SBFT_DEV bool f29_zero_mod_p_any(const f29& a) {
    f29 t;
    f29_normalize(t, a);  // limbs 0..7 in (-2^26, 2^29 + 2^26), limb 8 in [0, 2^24), |x| < 2^257
    u32 v[9];
    i32 c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const i32 x = (i32)t.v[i] + c;
        v[i] = (u32)x & F29_MASK;
        c = x >> 29;
    }
    v[8] = t.v[8] + (u32)c;
    return f29_zero_tail(v);
}

// ---------------------------------------------------------------- points
struct jp29 {
    f29 x, y, z;
};

__device__ __constant__ static const u32 C29_R2[9] = P256_F29_R2;
__device__ __constant__ static const u32 C29_ONE[9] = P256_F29_ONE;
__device__ __constant__ static const u32 C29_2P[9] = P256_F29_2P;
__device__ __constant__ static const u32 C29_G2X[9] = P256_F29_G2X;
__device__ __constant__ static const u32 C29_G2Y[9] = P256_F29_G2Y;

SBFT_DEV f29 f29_const(const u32* c) {
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = c[i];
    return r;
}

// Limb-bound bookkeeping below: N = f29_mul/f29_sqr output (limbs 0..7 in [0, 2^29)) or
// f29_normalize output (limbs 0..7 in (-2^26, 2^29 + 2^26)); N+- = difference of two mul
// outputs (|limb| < 2^29). Every product states its A x B limb bound (<= 2^59.83 allowed).

// Doubling, a = -3, in the form
//   d = Z^2, g = Y^2, b2 = 2XY^2, a' = (X - d)(X + d), u = 3a'^2
//   X3 = 3u - 4 b2 (= 9a'^2 - 8XY^2), Y3 = 3a'(2 b2 - X3) - 4 * 2g^2, Z3 = 2Y Z
// 6M + 2S, every intermediate inside the signed 32-bit limbs. In: X in N, Y in N or N+-,
// Z in N. Out: N (X3, Y3 normalised; Z3 a mul output).
// Z = 0 maps to Z3 = 0 (the caller's exceptional-case detector relies on it).
SBFT_DEV void p29_dbl_s(jp29& r, const jp29& p) {
    f29 d, g, b2, t0, t1, a1, a3, u, m;
    f29_sqr(d, p.z);                 // 2^29.2^2
    f29_sqr(g, p.y);
    f29_add(t0, g, g);               // 2g < 2^30
    f29_mul(b2, p.x, t0);            // 2^29.2 x 2^30
    f29_sub(t1, p.x, d);             // (-2^29, 2^29.2)
    f29_add(a1, p.x, d);             // < 2^30.1
    f29_mul(a1, t1, a1);             // a'  (2^29.2 x 2^30.1)
    f29_add(t1, p.y, p.y);           // 2Y < 2^30.2
    f29_mul(r.z, t1, p.z);           // Z3 = 2YZ (2^30.2 x 2^29.2)
    f29_muls(a3, a1, 3);             // 3a' < 2^30.6
    f29_mul(u, a1, a3);              // u = 3a'^2 (2^29 x 2^30.6)
    f29_mul(g, g, t0);               // 2g^2 (2^29 x 2^30)
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = 3 * u.v[i] - (b2.v[i] << 2);  // (-2^31, 2^30.6)
    f29_normalize(r.x, t1);
#pragma unroll
    for (int i = 0; i < 9; ++i) t0.v[i] = (b2.v[i] << 1) - r.x.v[i];  // (-2^29.2, 2^30)
    f29_mul(m, a1, t0);              // a'(2 b2 - X3) (2^29 x 2^30)
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = 3 * m.v[i] - (g.v[i] << 2);  // (-2^31, 2^30.6)
    f29_normalize(r.y, t1);
}

// acc += b (b Jacobian, N; b.y may be N+-) with no case analysis (12M + 4S). If H == 0
// (acc == +-b) the result has Z3 = 0, which every later doubling and addition keeps at 0:
// the caller checks Z once at the end and re-verifies such tuples on the general path.
SBFT_DEV void p29_add_jac_lean_s(jp29& acc, const jp29& b) {
    f29 z1z1, z2z2, u1, u2, s1, s2, t, h, rr, hh, hhh;
    f29_sqr(z1z1, acc.z);
    f29_mul(u2, b.x, z1z1);
    f29_mul(t, acc.z, z1z1);
    f29_mul(s2, b.y, t);
    f29_sqr(z2z2, b.z);
    f29_mul(u1, acc.x, z2z2);
    f29_mul(t, b.z, z2z2);
    f29_mul(s1, acc.y, t);
    f29_sub(h, u2, u1);              // N+-
    f29_sub(rr, s2, s1);             // N+-
    f29_sqr(hh, h);
    f29_mul(hhh, hh, h);
    f29_mul(u1, u1, hh);             // V = U1 H^2
    f29_mul(t, acc.z, b.z);
    f29_mul(acc.z, t, h);
    f29_sqr(t, rr);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = t.v[i] - hhh.v[i] - (u1.v[i] << 1);  // (-3 2^29, 2^29)
    f29_normalize(acc.x, t);
    f29_sub(t, u1, acc.x);           // (-2^29.2, 2^29 + 2^26)
    if (SBFT_MULSUB) {
        f29_mul_sub(acc.y, rr, t, s1, hhh);  // rr t - S1 H^3 (2^29 x 2^29.2 + 2^29 x 2^29): N
    } else {
        f29_mul(t, rr, t);
        f29_mul(s1, s1, hhh);
        f29_sub(acc.y, t, s1);       // N+-
    }
}

// acc += (x2, y2) affine (N; y2 may be N+-), same structure: 8M + 3S.
SBFT_DEV void p29_add_aff_lean_s(jp29& acc, const f29& x2, const f29& y2) {
    f29 z1z1, u2, s2, h, rr, hh, hhh, t;
    f29_sqr(z1z1, acc.z);
    f29_mul(u2, x2, z1z1);
    f29_mul(s2, acc.z, z1z1);
    f29_mul(s2, y2, s2);
    f29_sub(h, u2, acc.x);           // (-2^29.2, 2^29 + 2^4)
    f29_sub(rr, s2, acc.y);          // (-2^29.2, 2^29.2)
    f29_sqr(hh, h);
    f29_mul(hhh, hh, h);
    f29_mul(u2, acc.x, hh);          // V = X1 H^2
    f29_mul(acc.z, acc.z, h);
    f29_sqr(t, rr);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = t.v[i] - hhh.v[i] - (u2.v[i] << 1);
    f29_normalize(acc.x, t);
    f29_sub(t, u2, acc.x);           // (-2^29.2, 2^29 + 2^26)
    if (SBFT_MULSUB) {
        f29_mul_sub(acc.y, rr, t, acc.y, hhh);  // rr t - Y1 H^3 (2^29.2 x 2^29.2 + 2^29.2 x 2^29): N
    } else {
        f29_mul(t, rr, t);
        f29_mul(s2, acc.y, hhh);
        f29_sub(acc.y, t, s2);       // N+-
    }
}

SBFT_DEV void p29_dbl_i(jp29& r, const jp29& p) {
    f29 d, g, b2, t0, t1, a1, a3, u, m;
    f29_sqr2(d, p.z, g, p.y);        // 2^29.2^2 each
    f29_add(t0, g, g);               // 2g < 2^30
    f29_sub(t1, p.x, d);             // (-2^29, 2^29.2)
    f29_add(a1, p.x, d);             // < 2^30.1
    f29_mul2(b2, p.x, t0,            // 2XY^2 (2^29.2 x 2^30)
             a1, t1, a1);            // a'  (2^29.2 x 2^30.1)
    f29_add(t1, p.y, p.y);           // 2Y < 2^30.2
    f29_muls(a3, a1, 3);             // 3a' < 2^30.6
    f29_mul3(r.z, t1, p.z,           // Z3 = 2YZ (2^30.2 x 2^29.2)
             u, a1, a3,              // u = 3a'^2 (2^29 x 2^30.6)
             g, g, t0);              // 2g^2 (2^29 x 2^30)
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = 3 * u.v[i] - (b2.v[i] << 2);  // (-2^31, 2^30.6)
    f29_normalize(r.x, t1);
#pragma unroll
    for (int i = 0; i < 9; ++i) t0.v[i] = (b2.v[i] << 1) - r.x.v[i];  // (-2^29.2, 2^30)
    f29_mul(m, a1, t0);              // a'(2 b2 - X3) (2^29 x 2^30)
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = 3 * m.v[i] - (g.v[i] << 2);  // (-2^31, 2^30.6)
    f29_normalize(r.y, t1);
}

// acc += b (b Jacobian, N; b.y may be N+-) with no case analysis (12M + 4S). If H == 0
// (acc == +-b) the result has Z3 = 0, which every later doubling and addition keeps at 0:
// the caller checks Z once at the end and re-verifies such tuples on the general path.
SBFT_DEV void p29_add_jac_lean_i(jp29& acc, const jp29& b) {
    f29 z1z1, z2z2, u1, u2, s1, s2, t1, t2, z12, h, rr, hh, r2, hhh;
    f29_sqr2(z1z1, acc.z, z2z2, b.z);
    f29_mul2(u2, b.x, z1z1, t1, acc.z, z1z1);
    f29_mul3(u1, acc.x, z2z2, t2, b.z, z2z2, z12, acc.z, b.z);
    f29_mul2(s2, b.y, t1, s1, acc.y, t2);
    f29_sub(h, u2, u1);              // N+-
    f29_sub(rr, s2, s1);             // N+-
    f29_sqr2(hh, h, r2, rr);
    f29_mul3(hhh, hh, h, u1, u1, hh, acc.z, z12, h);  // H^3, V = U1 H^2, Z3 = Z1 Z2 H
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = r2.v[i] - hhh.v[i] - (u1.v[i] << 1);  // (-3 2^29, 2^29)
    f29_normalize(acc.x, t1);
    f29_sub(t1, u1, acc.x);          // (-2^29.2, 2^29 + 2^26)
    if (SBFT_MULSUB) {
        f29_mul_sub(acc.y, rr, t1, s1, hhh);  // rr t - S1 H^3: N
    } else {
        f29_mul2(t1, rr, t1, s1, s1, hhh);
        f29_sub(acc.y, t1, s1);      // N+-
    }
}

// acc += (x2, y2) affine (N; y2 may be N+-), same structure: 8M + 3S.
SBFT_DEV void p29_add_aff_lean_i(jp29& acc, const f29& x2, const f29& y2) {
    f29 z1z1, u2, s2, h, rr, hh, r2, hhh, t;
    f29_sqr(z1z1, acc.z);
    f29_mul2(u2, x2, z1z1, s2, acc.z, z1z1);
    f29_mul(s2, y2, s2);
    f29_sub(h, u2, acc.x);           // (-2^29.2, 2^29 + 2^4)
    f29_sub(rr, s2, acc.y);          // (-2^29.2, 2^29.2)
    f29_sqr2(hh, h, r2, rr);
    f29_mul3(hhh, hh, h, u2, acc.x, hh, acc.z, acc.z, h);  // H^3, V = X1 H^2, Z3 = Z1 H
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = r2.v[i] - hhh.v[i] - (u2.v[i] << 1);
    f29_normalize(acc.x, t);
    f29_sub(t, u2, acc.x);           // (-2^29.2, 2^29 + 2^26)
    if (SBFT_MULSUB) {
        f29_mul_sub(acc.y, rr, t, acc.y, hhh);  // rr t - Y1 H^3: N
    } else {
        f29_mul2(t, rr, t, s2, acc.y, hhh);
        f29_sub(acc.y, t, s2);       // N+-
    }
}

// dbl-2001-b shape (3M + 5S in the literature) under the signed-limb bounds: 4M + 4S and two
// more normalisations than p29_dbl_s, i.e. 72 fewer 64-bit mads per doubling.
//   d = Z^2, g = Y^2, b2 = X (2g) = 2 X Y^2, a' = (X - d)(X + d), al = norm(3 a') (alpha),
//   X3 = norm(al^2 - 4 b2), Z3 = 2 Y Z, L4 = norm(4 g^2),
//   Y3 = norm(al (2 b2 - X3) - 2 L4)      [= alpha (4 beta - X3) - 8 gamma^2]
// In: X in N or N', Y in N' or N+-, Z in N. Out: X3, Y3 in N', Z3 in N. Z = 0 maps to Z3 = 0.
SBFT_DEV void p29_dbl_b(jp29& r, const jp29& p) {
    f29 d, g, t0, t1, a1, al, b2, m, l;
    f29_sqr(d, p.z);                 // 2^29.2^2
    f29_sqr(g, p.y);
    f29_add(t0, g, g);               // 2g < 2^30
    f29_mul(b2, p.x, t0);            // 2^29.2 x 2^30
    f29_sub(t1, p.x, d);             // |.| < 2^29.2
    f29_add(a1, p.x, d);             // < 2^30.1
    f29_mul(a1, t1, a1);             // a' (2^29.2 x 2^30.1)
    f29_muls(al, a1, 3);             // 3a' < 2^30.6, |3a'| < 2^259.6
    f29_normalize(al, al);           // alpha (N')
    f29_add(t1, p.y, p.y);           // 2Y < 2^30.2
    f29_mul(r.z, t1, p.z);           // Z3 = 2YZ (2^30.2 x 2^29.2)
    f29_sqr(m, al);                  // alpha^2 (2^29.2^2)
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = m.v[i] - (b2.v[i] << 2);  // (-2^31, 2^29)
    f29_normalize(r.x, t1);          // X3 (N')
    f29_sqr(l, g);                   // gamma^2 (N)
#pragma unroll
    for (int i = 0; i < 9; ++i) l.v[i] <<= 2;                      // 4L < 2^31
    f29_normalize(l, l);             // 4L (N')
#pragma unroll
    for (int i = 0; i < 9; ++i) t0.v[i] = (b2.v[i] << 1) - r.x.v[i];  // (-2^29.2, 2^30 + 2^26)
    f29_mul(m, al, t0);              // alpha (2 b2 - X3) (2^29.2 x 2^30.1)
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = m.v[i] - (l.v[i] << 1);   // (-2^30.2, 2^29 + 2^27)
    f29_normalize(r.y, t1);          // Y3 (N')
}

// p29_dbl_b with X3 and Y3 as products with addends (f29_mulsq_add): the same 4M + 4S, but
// X3 = al^2 - 4 b2 and Y3 = al (2 b2 - X3) - 8 g^2 leave their products already folded to N',
// so the two subtraction loops, the 4L scaling and three normalisations are gone.
// Value bounds: b2, l = g^2 < 2^256.6 (products of N' values), so |X3| < 2^259, |Y3| < 2^259.3
// before the fold. In/out as p29_dbl_b (X3, Y3 in N', Z3 a product output in N).
SBFT_DEV void p29_dbl_f(jp29& r, const jp29& p) {
    f29 d, g, t0, t1, a1, al, b2, l, x3;
    f29 y2;
    f29_add(y2, p.y, p.y);           // 2Y < 2^30.2
    f29_sqr(d, p.z);                 // 2^29.2^2
    f29_sqr_d(g, p.y, y2);
    f29_add(t0, g, g);               // 2g < 2^30
    f29_mul(b2, p.x, t0);            // 2^29.2 x 2^30
    f29_sub(t1, p.x, d);             // |.| < 2^29.2
    f29_add(a1, p.x, d);             // < 2^30.1
    f29_mul(a1, t1, a1);             // a' (2^29.2 x 2^30.1)
    if (SBFT_TRIPLE_CARRY) {
        f29_triple(al, a1);          // alpha (limbs < 2^29 + 2, |alpha| < 2^258.2)
    } else {
        f29_muls(al, a1, 3);         // 3a' < 2^30.6, |3a'| < 2^259.6
        f29_normalize(al, al);       // alpha (N')
    }
    f29_mul(r.z, y2, p.z);           // Z3 = 2YZ (2^30.2 x 2^29.2)
    {
        const f29* const v[1] = {&b2};
        const u32 c[1] = {f29_kconst(-4)};
        f29_mulsq_add<true, 1>(x3, al, al, v, c);  // X3 = alpha^2 - 4 b2 (2^29.2^2; -4 b2 < 2^31): N'
    }
    f29_sqr_d(l, g, t0);             // gamma^2 (N)
#pragma unroll
    for (int i = 0; i < 9; ++i) t0.v[i] = (b2.v[i] << 1) - x3.v[i];  // (-2^29.2, 2^30 + 2^25)
    {
        const f29* const v[1] = {&l};
        const u32 c[1] = {f29_kconst(-8)};
        f29_mulsq_add<false, 1>(r.y, al, t0, v, c);  // Y3 = alpha t0 - 8 L (2^29.2 x 2^30.1): N'
    }
    r.x = x3;
}

// p29_dbl_f on the representative scaled by 1/2 ((X, Y, Z) ~ (X/4, Y/8, Z/2), the same point):
//   d = Z^2, g = Y^2, b = X g, a' = (X - d)(X + d), h = 3 a' / 2 (f29_triple_half),
//   X3 = h^2 - 2 b, Y3 = h (b - X3) - g^2, Z3 = Y Z
// The 8 of dbl-2001-b's 8 gamma^2 is gone, so g^2 joins Y3's product as negated column terms
// (f29_mul_sqsub: 45 mads, no reduction of its own); the halving costs ~40 32-bit ops. 765
// mads per doubling against 810. In: X in N or N', Y in N' or N+-, Z in N. Out: X3 in N', Y3
// and Z3 in N (Y3 signed top, |Y3| < 2^258). Z = 0 maps to Z3 = 0.
SBFT_DEV void p29_dbl_h(jp29& r, const jp29& p) {
    f29 d, g, t0, t1, a1, al, b, x3, ng;
    f29_add(t0, p.y, p.y);           // 2Y < 2^30.2
    f29_sqr(d, p.z);                 // 2^29.2^2
    f29_sqr_d(g, p.y, t0);           // gamma (N)
    f29_mul(b, p.x, g);              // beta = X gamma (2^29.2 x 2^29)
    f29_sub(t1, p.x, d);             // |.| < 2^29.2
    f29_add(a1, p.x, d);             // < 2^30.1
    f29_mul(a1, t1, a1);             // a' (2^29.2 x 2^30.1)
    f29_triple_half(al, a1);         // alpha / 2 (limbs < 2^29 + 3, |.| < 2^258.1)
    f29_mul(r.z, p.y, p.z);          // Z3 = Y Z
    {
        const f29* const v[1] = {&b};
        const u32 c[1] = {f29_kconst(-2)};
        f29_mulsq_add<true, 1>(x3, al, al, v, c);  // X3 = (alpha/2)^2 - 2 beta: N'
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        t1.v[i] = b.v[i] - x3.v[i];  // (-2^29.2, 2^29 + 2^25)
        ng.v[i] = 0u - g.v[i];
        t0.v[i] = ng.v[i] << 1;      // -2 gamma
    }
    f29_mul_sqsub(r.y, al, t1, g, ng, t0);  // Y3 = (alpha/2)(beta - X3) - gamma^2: N
    r.x = x3;
}

#ifndef SBFT_F29_IL
#define SBFT_F29_IL 6
#endif
// SBFT_F29_IL bit 0/1/2: interleaved form of the doubling / Jacobian addition / mixed addition
#ifndef SBFT_DBL_FORM
#define SBFT_DBL_FORM 3  // 0: 6M + 2S (p29_dbl_s / _i), 1: 4M + 4S (p29_dbl_b), 2: p29_dbl_b fused (p29_dbl_f),
                         // 3: halved representative (p29_dbl_h)
#endif
SBFT_DEV void p29_dbl(jp29& r, const jp29& p) {
    if (SBFT_DBL_FORM == 3) p29_dbl_h(r, p);
    else if (SBFT_DBL_FORM == 2) p29_dbl_f(r, p);
    else if (SBFT_DBL_FORM == 1) p29_dbl_b(r, p);
    else if (SBFT_F29_IL & 1) p29_dbl_i(r, p);
    else p29_dbl_s(r, p);
}
SBFT_DEV void p29_add_jac_lean(jp29& acc, const jp29& b) {
    if (SBFT_F29_IL & 2) p29_add_jac_lean_i(acc, b);
    else p29_add_jac_lean_s(acc, b);
}
#ifndef SBFT_ADD_FUSED
#define SBFT_ADD_FUSED 1  // the mixed additions' X3 as a product with addends (p29_add_aff_lean_f)
#endif
// p29_add_aff_lean_i with X3 = r^2 - HHH - 2V as one product with two addends (f29_mulsq_add):
// no subtraction loop, no normalisation. HH rides with S2 (one interleaved pair) so r^2 can
// wait for HHH and V. |X3| < 2^256.1 + 2^256.6 + 2^257.6 < 2^258.5 before the fold: N'.
SBFT_DEV void p29_add_aff_lean_f(jp29& acc, const f29& x2, const f29& y2) {
    f29 z1z1, u2, s2, h, rr, hh, hhh, t, x3;
    f29_sqr(z1z1, acc.z);
    f29_mul2(u2, x2, z1z1, t, acc.z, z1z1);
    f29_sub(h, u2, acc.x);           // (-2^29.2, 2^29 + 2^25)
    {
        f29* const r[2] = {&s2, &hh};
        const f29* const a[2] = {&y2, &h};
        const f29* const b[2] = {&t, &h};
        f29_mulv<2, 2u>(r, a, b);    // S2 = y2 Z1^3 (2^29.2 x 2^29) | HH = H^2 (2^29.2^2)
    }
    f29_sub(rr, s2, acc.y);          // (-2^29.2, 2^29.2)
    f29_mul3(hhh, hh, h, u2, acc.x, hh, acc.z, acc.z, h);  // H^3, V = X1 H^2, Z3 = Z1 H
    {
        const f29* const v[2] = {&hhh, &u2};
        const u32 c[2] = {f29_kconst(-1), f29_kconst(-2)};
        f29_mulsq_add<true, 2>(x3, rr, rr, v, c);  // X3 = r^2 - HHH - 2V: N'
    }
    f29_sub(t, u2, x3);              // (-2^29.2, 2^29 + 2^25)
    f29_mul_sub(acc.y, rr, t, acc.y, hhh);  // rr t - Y1 H^3: N
    acc.x = x3;
}

SBFT_DEV void p29_add_aff_lean(jp29& acc, const f29& x2, const f29& y2) {
    if (SBFT_ADD_FUSED) p29_add_aff_lean_f(acc, x2, y2);
    else if (SBFT_F29_IL & 4) p29_add_aff_lean_i(acc, x2, y2);
    else p29_add_aff_lean_s(acc, x2, y2);
}

// ---------------------------------------------------------------- exceptional additions
// The lean mixed addition has no case analysis: for acc == +-P (H == 0) it returns Z3 = 0.
// In the verify ladders this can happen only at additions an attacker can aim at (the last
// addition of the u2 Q ladder, any comb addition of u1 G on top of u2 Q, see p256_verify.hip),
// and a crafted request must not cost more than an honest one (a rejected proposal triggers
// complain + sync, view.go:386-393). So after those additions:
//   hz = Z3 == 0 (exact; Z3 = Z1 H with Z1 != 0, so H == 0): then X3 = r^2, and r == 0 (the
//   addend equals acc: the result is 2P, a doubling of the affine addend) iff X3 == 0, else the
//   addend is -acc and the result is infinity (flag inf);
//   inf (acc was infinity): the result is the addend itself.
// The repair runs in a wave-uniform branch taken only when some lane of the wave needs it, so
// an honest batch pays the ~50-instruction zero test per addition. reload(x, y) re-materialises
// the addend (from the table or the comb in memory) instead of keeping it live across the
// addition; dbl(p) doubles in place (the kernel's doubling: one lane or a lane pair).
template <class Dbl, class Reload>
SBFT_DEV void add_aff_fix(jp29& acc, bool& inf, Dbl dbl, Reload reload) {
    const bool hz = !inf && f29_zero_mod_p(acc.z);
    if (__builtin_expect(__any(hz || inf), 0)) {
        f29 x2, y2;
        reload(x2, y2);
        const bool twice = hz && f29_zero_mod_p_any(acc.x);
        jp29 d;
        d.x = x2;
        d.y = y2;
        d.z = f29_const(C29_ONE);
        dbl(d);
        if (twice) acc = d;
        if (inf) {
            acc.x = x2;
            acc.y = y2;
            acc.z = f29_const(C29_ONE);
        }
        inf = hz && !twice;
    }
}

// ---------------------------------------------------------------- lane pairs (latency kernel)
// p256_verify_small_kernel<2> runs one verify on two adjacent lanes (2t, 2t+1). Both hold the
// same point; at each step the two lanes compute two independent products of the formula,
// each with its own operands (f29_pick), and f29_unpair hands both results to both lanes
// (two quad_perm DPP moves per limb). A doubling is 4 such steps instead of 8 products, a
// mixed addition 6 instead of 11: the per-lane instruction stream of a small batch, which is
// what its latency is, shrinks by ~40%.
//
// With one product per lane per step there is no second product to interleave with, and a
// product column is a chain of dependent 64-bit mads (a wait state each on gfx950). So the
// pair forms use f29_mul_ilp / f29_sqr_ilp: the 17 product columns are summed first as
// independent chains, then the Montgomery pass adds carry and reduction terms column by column
// (one extra 64-bit add per column, no wait states in the product part).
// SBFT_ILP_LA > 0: software-pipelined form. At one wave per SIMD (the latency kernels) nothing
// hides the Montgomery pass's serial chain (per column a 64-bit add and a 64-bit shift, each
// waiting on the last), and with every column summed first (SBFT_ILP_LA = 0) the chain runs
// after all 81 product mads with idle issue slots. Summing column k + LA while the chain is at
// column k gives the scheduler product mads to fill those slots with; the instructions are the
// same.
#ifndef SBFT_ILP_LA
#define SBFT_ILP_LA 4
#endif
template <bool SQ>
SBFT_DEV i64 f29_column(int k, const f29& a, const f29& b, const u32 (&d)[9], i64 c = 0) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int j = k - i;
        if (SQ) {
            if (j > i && j <= 8) c = smad(a.v[i], d[j], c);
            if (j == i) c = smad(a.v[i], a.v[i], c);
        } else {
            if (j >= 0 && j <= 8) c = smad(a.v[i], b.v[j], c);
        }
    }
    return c;
}
// Mont(a b) + sum_t c_t v_t with NA addends (see f29_mulsq_add; NA = 0: a plain product, v and
// c unused), the fold masked by hmask.
template <bool SQ, int NA>
SBFT_DEV void f29_mulsq_core(f29& r, const f29& a, const f29& b, const f29* const* v, const u32* c, u32 hmask) {
    const f29_red K = f29_red_consts();
    u32 d[9];
    if (SQ)
#pragma unroll
        for (int i = 0; i < 9; ++i) d[i] = a.v[i] << 1;
    i64 col[17];
    constexpr int LA = SBFT_ILP_LA > 0 ? SBFT_ILP_LA : 17;
#pragma unroll
    for (int k = 0; k < LA && k < 17; ++k) col[k] = f29_column<SQ>(k, a, b, d);
    // Reduction terms first (m[k-3..] are ready columns ahead), the carry last: the serial
    // chain is one 64-bit add and one shift per column.
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        if (k + LA < 17) col[k + LA] = f29_column<SQ>(k + LA, a, b, d);
        i64 x = col[k];
        if (k >= 3 && k - 3 <= 8) x = smad(m[k - 3], K.c9, x);
        if (k >= 6 && k - 6 <= 8) x = smad(m[k - 6], K.c18, x);
        if (k >= 7 && k - 7 <= 8) x = smad(m[k - 7], K.c7, x);
        if (k >= 8 && k - 8 <= 8) x = smad(m[k - 8], K.c8, x);
        if (k >= 9)
#pragma unroll
            for (int t = 0; t < NA; ++t) x = smad(v[t]->v[k - 9], c[t], x);
        acc = k == 0 ? x : x + acc;
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
    u32 top = (u32)acc;
    if (NA > 0) {
#pragma unroll
        for (int t = 0; t < NA; ++t) top += v[t]->v[8] * c[t];
        f29_fold_top(r, top, hmask);
    } else {
        r.v[8] = top;
    }
}
template <bool SQ>
SBFT_DEV void f29_mulsq_ilp(f29& r, const f29& a, const f29& b) {
    f29_mulsq_core<SQ, 0>(r, a, b, nullptr, nullptr, 0u);
}
template <bool SQ, int NA>
SBFT_DEV void f29_mulsq_add_ilp(f29& r, const f29& a, const f29& b, const f29* const (&v)[NA], const u32 (&c)[NA],
                                u32 hmask) {
    f29_mulsq_core<SQ, NA>(r, a, b, v, c, hmask);
}
// f29_mul_sub in the pipelined ILP form: Mont(a b + c nd) with nd = -d supplied by the caller
// (a lane that wants a plain product passes nd = 0). Each column is one mad chain over both
// products (the look-ahead columns fill its wait states), then the reduction terms and the carry
// as in f29_mulsq_core. f29_mul_sub's contract; output N.
SBFT_DEV void f29_mul_sub_ilp(f29& r, const f29& a, const f29& b, const f29& c, const f29& nd) {
    const f29_red K = f29_red_consts();
    const u32 unused[9] = {};
    i64 col[17];
    constexpr int LA = SBFT_ILP_LA > 0 ? SBFT_ILP_LA : 17;
#pragma unroll
    for (int k = 0; k < LA && k < 17; ++k)
        col[k] = f29_column<false>(k, c, nd, unused, f29_column<false>(k, a, b, unused));
    u32 m[9];
    i64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
        if (k + LA < 17)
            col[k + LA] = f29_column<false>(k + LA, c, nd, unused, f29_column<false>(k + LA, a, b, unused));
        i64 x = col[k];
        if (k >= 3 && k - 3 <= 8) x = smad(m[k - 3], K.c9, x);
        if (k >= 6 && k - 6 <= 8) x = smad(m[k - 6], K.c18, x);
        if (k >= 7 && k - 7 <= 8) x = smad(m[k - 7], K.c7, x);
        if (k >= 8 && k - 8 <= 8) x = smad(m[k - 8], K.c8, x);
        acc = k == 0 ? x : x + acc;
        if (k < 9) m[k] = lo29(acc);
        else r.v[k - 9] = lo29(acc);
        acc = sar29(acc);
    }
    r.v[8] = (u32)acc;
}
SBFT_DEV void f29_mul_ilp(f29& r, const f29& a, const f29& b) { f29_mulsq_ilp<false>(r, a, b); }
SBFT_DEV void f29_sqr_ilp(f29& r, const f29& a) { f29_mulsq_ilp<true>(r, a, a); }

// p29_add_aff_lean_f with the pipelined ILP products (one lane, no pairing): the same 8M + 3S,
// the same values limb for limb (the column sums are exact either way), but at one wave per SIMD
// the chain form's dependent mads leave most issue slots idle. For the latency kernels whose
// lanes each run their own additions (the registered-client comb, p256_verify_keyed_lanes_kernel).
SBFT_DEV void p29_add_aff_lean_ilp(jp29& acc, const f29& x2, const f29& y2) {
    f29 z1z1, u2, t, h, s2, hh, rr, hhh, v, x3, nd;
    f29_sqr_ilp(z1z1, acc.z);
    f29_mul_ilp(u2, x2, z1z1);
    f29_mul_ilp(t, acc.z, z1z1);
    f29_sub(h, u2, acc.x);           // (-2^29.2, 2^29 + 2^25)
    f29_mul_ilp(s2, y2, t);          // S2 = y2 Z1^3
    f29_sqr_ilp(hh, h);
    f29_sub(rr, s2, acc.y);          // (-2^29.2, 2^29.2)
    f29_mul_ilp(hhh, hh, h);
    f29_mul_ilp(v, acc.x, hh);       // V = X1 H^2
    f29_mul_ilp(acc.z, acc.z, h);    // Z3 = Z1 H
    {
        const f29* const va[2] = {&hhh, &v};
        const u32 c[2] = {(u32)-1, (u32)-2};
        f29_mulsq_add_ilp<true, 2>(x3, rr, rr, va, c, ~0u);  // X3 = r^2 - HHH - 2V: N'
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        t.v[i] = v.v[i] - x3.v[i];   // (-2^29.2, 2^29 + 2^25)
        nd.v[i] = 0u - hhh.v[i];
    }
    f29_mul_sub_ilp(acc.y, rr, t, acc.y, nd);  // r t - Y1 H^3: N
    acc.x = x3;
}

SBFT_DEV f29 f29_pick(bool odd, const f29& even_v, const f29& odd_v) {
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = odd ? odd_v.v[i] : even_v.v[i];
    return r;
}
// o = the even lane's value in the even lane, the odd lane's in the odd lane ->
// e = even lane's value, d = odd lane's value, in both lanes of the pair.
SBFT_DEV void f29_unpair(const f29& o, f29& e, f29& d) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        e.v[i] = (u32)__builtin_amdgcn_mov_dpp((int)o.v[i], 0xA0, 0xF, 0xF, false);  // quad_perm [0,0,2,2]
        d.v[i] = (u32)__builtin_amdgcn_mov_dpp((int)o.v[i], 0xF5, 0xF, 0xF, false);  // quad_perm [1,1,3,3]
    }
}

// p29_dbl_b on a lane pair (same products, same bounds):
//   1: d = Z^2 | g = Y^2     2: b2 = X (2g) | a' = (X - d)(X + d)
//   3: alpha^2 | gamma^2     4: alpha (2 b2 - X3) | Z3 = 2 Y Z
SBFT_DEV void p29_dbl_pair_b(jp29& r, const jp29& p, bool odd) {
    f29 o, d, g, t0, t1, a1, al, b2, m, l, x3, z3;
    f29_sqr_ilp(o, f29_pick(odd, p.z, p.y));                        // 2^29.2^2
    f29_unpair(o, d, g);
    f29_add(t0, g, g);                                          // 2g < 2^30
    f29_sub(t1, p.x, d);                                        // |.| < 2^29.2
    f29_add(a1, p.x, d);                                        // < 2^30.1
    f29_mul_ilp(o, f29_pick(odd, p.x, t1), f29_pick(odd, t0, a1));  // 2^29.2 x 2^30 | 2^29.2 x 2^30.1
    f29_unpair(o, b2, a1);
    f29_muls(al, a1, 3);                                        // 3a' < 2^30.6
    f29_normalize(al, al);                                      // alpha (N')
    f29_sqr_ilp(o, f29_pick(odd, al, g));                           // 2^29.2^2
    f29_unpair(o, m, l);
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = m.v[i] - (b2.v[i] << 2);  // (-2^31, 2^29)
    f29_normalize(x3, t1);                                      // X3 (N')
#pragma unroll
    for (int i = 0; i < 9; ++i) l.v[i] <<= 2;                  // 4L < 2^31
    f29_normalize(l, l);                                        // 4L (N')
#pragma unroll
    for (int i = 0; i < 9; ++i) t0.v[i] = (b2.v[i] << 1) - x3.v[i];  // (-2^29.2, 2^30 + 2^26)
    f29_add(t1, p.y, p.y);                                      // 2Y < 2^30.2
    f29_mul_ilp(o, f29_pick(odd, al, t1), f29_pick(odd, t0, p.z));  // 2^29.2 x 2^30.1 | 2^30.2 x 2^29.2
    f29_unpair(o, m, z3);
#pragma unroll
    for (int i = 0; i < 9; ++i) t1.v[i] = m.v[i] - (l.v[i] << 1);  // (-2^30.2, 2^29 + 2^27)
    f29_normalize(r.y, t1);                                     // Y3 (N')
    r.x = x3;
    r.z = z3;
}

// p29_add_aff_lean on a lane pair (same products, same bounds, no case analysis):
//   1: Z1^2 (both)          2: U2 = x2 Z1^2 | Z1^3     3: HH = H^2 | S2 = y2 Z1^3
//   4: V = X1 HH | HHH      5: r^2 | Z3 = Z1 H          6: r (V - X3) | Y1 HHH
SBFT_DEV void p29_add_aff_pair_b(jp29& acc, const f29& x2, const f29& y2, bool odd) {
    f29 o, z1z1, u2, s2, h, rr, hh, hhh, v, r2, z3, t, s;
    f29_sqr_ilp(z1z1, acc.z);
    f29_mul_ilp(o, f29_pick(odd, x2, acc.z), z1z1);
    f29_unpair(o, u2, s2);
    f29_sub(h, u2, acc.x);                                      // (-2^29.2, 2^29 + 2^26)
    f29_mul_ilp(o, f29_pick(odd, h, y2), f29_pick(odd, h, s2));
    f29_unpair(o, hh, s2);
    f29_sub(rr, s2, acc.y);                                     // (-2^29.2, 2^29.2)
    f29_mul_ilp(o, f29_pick(odd, acc.x, hh), f29_pick(odd, hh, h));
    f29_unpair(o, v, hhh);
    f29_mul_ilp(o, f29_pick(odd, rr, acc.z), f29_pick(odd, rr, h));
    f29_unpair(o, r2, z3);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = r2.v[i] - hhh.v[i] - (v.v[i] << 1);  // (-3 2^29, 2^29)
    f29_normalize(acc.x, t);
    f29_sub(t, v, acc.x);                                       // (-2^29.2, 2^29 + 2^26)
    f29_mul_ilp(o, f29_pick(odd, rr, acc.y), f29_pick(odd, t, hhh));
    f29_unpair(o, t, s);
    f29_sub(acc.y, t, s);                                       // N+-
    acc.z = z3;
}

// The pair forms with products with addends (f29_mulsq_add_ilp): the even lane's X3 and Y3
// come out of their products folded (N'), the odd lane's product takes c = 0. This takes the
// normalisations and subtraction loops off the pair's critical path.
#ifndef SBFT_PAIR_FUSED
#define SBFT_PAIR_FUSED 1
#endif
//   1: d = Z^2 | g = Y^2     2: b2 = X (2g) | a' = (X - d)(X + d)
//   3: X3 = alpha^2 - 4 b2 | L = gamma^2     4: Y3 = alpha (2 b2 - X3) - 8 L | Z3 = 2 Y Z
SBFT_DEV void p29_dbl_pair_f(jp29& r, const jp29& p, bool odd) {
    f29 o, d, g, t0, t1, a1, al, b2, l, x3, z3;
    f29_sqr_ilp(o, f29_pick(odd, p.z, p.y));                        // 2^29.2^2
    f29_unpair(o, d, g);
    f29_add(t0, g, g);                                          // 2g < 2^30
    f29_sub(t1, p.x, d);                                        // |.| < 2^29.2
    f29_add(a1, p.x, d);                                        // < 2^30.1
    f29_mul_ilp(o, f29_pick(odd, p.x, t1), f29_pick(odd, t0, a1));  // 2^29.2 x 2^30 | 2^29.2 x 2^30.1
    f29_unpair(o, b2, a1);
    if (SBFT_TRIPLE_CARRY) {
        f29_triple(al, a1);                                     // alpha (limbs < 2^29 + 2)
    } else {
        f29_muls(al, a1, 3);                                    // 3a' < 2^30.6
        f29_normalize(al, al);                                  // alpha (N')
    }
    {
        const f29* const v[1] = {&b2};
        const u32 c[1] = {odd ? 0u : (u32)-4};
        const f29 sq = f29_pick(odd, al, g);
        f29_mulsq_add_ilp<true, 1>(o, sq, sq, v, c, ~0u);       // alpha^2 - 4 b2 | gamma^2: N'
    }
    f29_unpair(o, x3, l);
#pragma unroll
    for (int i = 0; i < 9; ++i) t0.v[i] = (b2.v[i] << 1) - x3.v[i];  // (-2^29.2, 2^30 + 2^25)
    f29_add(t1, p.y, p.y);                                      // 2Y < 2^30.2
    {
        const f29* const v[1] = {&l};
        const u32 c[1] = {odd ? 0u : (u32)-8};
        f29_mulsq_add_ilp<false, 1>(o, f29_pick(odd, al, t1), f29_pick(odd, t0, p.z), v, c,
                                    odd ? 0u : ~0u);            // alpha t0 - 8 L: N' | 2YZ: N
    }
    f29_unpair(o, r.y, z3);
    r.x = x3;
    r.z = z3;
}

//   1: Z1^2 (both)          2: U2 = x2 Z1^2 | Z1^3     3: HH = H^2 | S2 = y2 Z1^3
//   4: V = X1 HH | HHH      5: X3 = r^2 - HHH - 2V | Z3 = Z1 H      6: r (V - X3) | Y1 HHH
SBFT_DEV void p29_add_aff_pair_f(jp29& acc, const f29& x2, const f29& y2, bool odd) {
    f29 o, z1z1, u2, s2, h, rr, hh, hhh, v, x3, z3, t, s;
    f29_sqr_ilp(z1z1, acc.z);
    f29_mul_ilp(o, f29_pick(odd, x2, acc.z), z1z1);
    f29_unpair(o, u2, s2);
    f29_sub(h, u2, acc.x);                                      // (-2^29.2, 2^29 + 2^26)
    f29_mul_ilp(o, f29_pick(odd, h, y2), f29_pick(odd, h, s2));
    f29_unpair(o, hh, s2);
    f29_sub(rr, s2, acc.y);                                     // (-2^29.2, 2^29.2)
    f29_mul_ilp(o, f29_pick(odd, acc.x, hh), f29_pick(odd, hh, h));
    f29_unpair(o, v, hhh);
    {
        const f29* const w[2] = {&hhh, &v};
        const u32 c[2] = {odd ? 0u : (u32)-1, odd ? 0u : (u32)-2};
        f29_mulsq_add_ilp<false, 2>(o, f29_pick(odd, rr, acc.z), f29_pick(odd, rr, h), w, c,
                                    odd ? 0u : ~0u);            // r^2 - HHH - 2V: N' | Z1 H: N
    }
    f29_unpair(o, x3, z3);
    f29_sub(t, v, x3);                                          // (-2^29.2, 2^29 + 2^25)
    f29_mul_ilp(o, f29_pick(odd, rr, acc.y), f29_pick(odd, t, hhh));
    f29_unpair(o, t, s);
    f29_sub(acc.y, t, s);                                       // N+-
    acc.x = x3;
    acc.z = z3;
}

SBFT_DEV void p29_dbl_pair(jp29& r, const jp29& p, bool odd) {
    if (SBFT_PAIR_FUSED) p29_dbl_pair_f(r, p, odd);
    else p29_dbl_pair_b(r, p, odd);
}
SBFT_DEV void p29_add_aff_pair(jp29& acc, const f29& x2, const f29& y2, bool odd) {
    if (SBFT_PAIR_FUSED) p29_add_aff_pair_f(acc, x2, y2, odd);
    else p29_add_aff_pair_b(acc, x2, y2, odd);
}

// ---------------------------------------------------------------- lane-local pair doubling
// A lane of the pair issues one instruction every ~4 cycles whatever it is (one wave per SIMD),
// so the pair's glue counts as much as its products. p29_dbl_pair keeps every value in both
// lanes: each step picks the two lanes' operands (18 v_cndmask) and hands both products to both
// lanes (18 DPP moves). The lane-local form keeps the point as
//   xb = X (both lanes), zy = Z (even lane) | Y (odd lane), zo = Z (odd lane),
// feeds each step from the lanes' own results, and moves across the pair (one quad_perm swap,
// 9 DPP) only the value the other lane needs: 159 glue instructions per doubling against 213.
// Same products, same bounds as p29_dbl_pair_f:
//   1: d = Z^2 | g = Y^2                     2: b2 = X (2g) | a' = (X - d)(X + d)
//   3: X3 = alpha^2 - 4 b2 | L = gamma^2     4: Y3 = alpha (2 b2 - X3) - 8 L | Z3 = 2 Y Z
struct pl29 {
    f29 xb, zy, zo;
};
// even lane's e, odd lane's o: one v_cndmask on the constant odd-lane mask. Written as asm so
// the compiler cannot turn a run of selects into a branch on the lane parity (it did: both
// sides then run one after the other, with exec-mask flips between them).
SBFT_DEV u32 sel_pair(u32 e, u32 o) {
    u32 r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(e), "v"(o), "s"(0xAAAAAAAAAAAAAAAAull));
    return r;
}
SBFT_DEV f29 f29_sel_pair(const f29& e, const f29& o) {
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = sel_pair(e.v[i], o.v[i]);
    return r;
}
SBFT_DEV f29 f29_swap_pair(const f29& a) {  // each lane gets its partner's value (quad_perm [1,0,3,2])
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = (u32)__builtin_amdgcn_mov_dpp((int)a.v[i], 0xB1, 0xF, 0xF, false);
    return r;
}
SBFT_DEV f29 f29_bcast_pair(const f29& a, bool from_odd) {  // the even (odd) lane's value in both lanes
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i)
        r.v[i] = from_odd ? (u32)__builtin_amdgcn_mov_dpp((int)a.v[i], 0xF5, 0xF, 0xF, false)
                          : (u32)__builtin_amdgcn_mov_dpp((int)a.v[i], 0xA0, 0xF, 0xF, false);
    return r;
}
SBFT_DEV pl29 pl29_from(const jp29& p, bool odd) {
    pl29 q;
    q.xb = p.x;
    q.zy = f29_sel_pair(p.z, p.y);
    q.zo = p.z;
    (void)odd;
    return q;
}
SBFT_DEV void pl29_to(jp29& p, const pl29& q) {
    p.x = q.xb;
    p.y = f29_bcast_pair(q.zy, true);
    p.z = f29_bcast_pair(q.zy, false);
}
SBFT_DEV void p29_dbl_pl(pl29& P, bool odd) {
    const u32 om = sel_pair(0u, ~0u);
    f29 o1, s1, a, b, o2, s2, al, o3, s3, o4;
    f29_sqr_ilp(o1, P.zy);                                      // d | g (2^29.2^2)
    s1 = f29_swap_pair(o1);                                     // g | d
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = P.xb.v[i] - (s1.v[i] & om);                    // X | X - d: |.| < 2^29.2
        b.v[i] = s1.v[i] + sel_pair(s1.v[i], P.xb.v[i]);        // 2g < 2^30 | X + d < 2^30.1
    }
    f29_mul_ilp(o2, a, b);                                      // b2 | a'
    s2 = f29_swap_pair(o2);                                     // a' | b2
    f29_triple(al, s2);                                         // alpha (even lane)
    {
        const f29 sq = f29_sel_pair(al, o1);
        const f29* const v[1] = {&o2};
        const u32 c[1] = {sel_pair((u32)-4, 0u)};
        f29_mulsq_add_ilp<true, 1>(o3, sq, sq, v, c, ~0u);     // X3 = alpha^2 - 4 b2 | L = gamma^2: N'
    }
    s3 = f29_swap_pair(o3);                                     // L | X3
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const u32 t0 = (o2.v[i] << 1) - o3.v[i];                // 2 b2 - X3: (-2^29.2, 2^30 + 2^25)
        const u32 y2 = P.zy.v[i] << 1;                          // 2Y < 2^30.2 (odd lane)
        a.v[i] = sel_pair(al.v[i], y2);
        b.v[i] = sel_pair(t0, P.zo.v[i]);
    }
    {
        const f29* const v[1] = {&s3};
        const u32 c[1] = {sel_pair((u32)-8, 0u)};
        f29_mulsq_add_ilp<false, 1>(o4, a, b, v, c, ~om);      // Y3 = alpha t0 - 8 L: N' | Z3 = 2YZ: N
    }
    P.xb = f29_sel_pair(o3, s3);                                // X3 in both lanes
    P.zy = f29_swap_pair(o4);                                   // Z3 | Y3
    P.zo = o4;                                                  // Z3 (odd lane)
    (void)odd;
}
// The mixed addition in the lane-local form (p29_add_aff_pair_f's products, same bounds):
//   1: Z1^2 (both)   2: U2 = x2 Z1^2 | Z1^3   3: HH = H^2 | S2 = y2 Z1^3   4: V = X1 HH | HHH
//   5: Z3 = Z1 H | X3 = r^2 - HHH - 2V        6: Y1 HHH | r (V - X3)
// (x2, y2) affine in both lanes. Out: X3 in N', Y3 in N+-, Z3 in N, as p29_add_aff_pair_f.
SBFT_DEV void p29_add_aff_pl(pl29& P, const f29& x2, const f29& y2) {
    f29 z1, o1, o2, s2, h, o3, s3, hh, o4, s4, r, o5, s5, szy, a, b, o6, s6;
    z1 = f29_sel_pair(P.zy, P.zo);                              // Z1 in both lanes
    f29_sqr_ilp(o1, z1);                                        // Z1^2
    f29_mul_ilp(o2, f29_sel_pair(x2, z1), o1);                  // U2 | Z1^3
    s2 = f29_swap_pair(o2);                                     // Z1^3 | U2
#pragma unroll
    for (int i = 0; i < 9; ++i) h.v[i] = sel_pair(o2.v[i], s2.v[i]) - P.xb.v[i];  // H: (-2^29.2, 2^29 + 2^25)
    f29_mul_ilp(o3, f29_sel_pair(h, y2), f29_sel_pair(h, o2));  // HH | S2
    s3 = f29_swap_pair(o3);                                     // S2 | HH
    hh = f29_sel_pair(o3, s3);                                  // HH in both lanes
    f29_mul_ilp(o4, f29_sel_pair(P.xb, h), hh);                 // V | HHH
    s4 = f29_swap_pair(o4);                                     // HHH | V
    f29_sub(r, o3, P.zy);                                       // r = S2 - Y1 (odd lane): |.| < 2^29.2
    {
        const f29* const v[2] = {&o4, &s4};
        const u32 c[2] = {sel_pair(0u, (u32)-1), sel_pair(0u, (u32)-2)};
        f29_mulsq_add_ilp<false, 2>(o5, f29_sel_pair(P.zy, r), f29_sel_pair(h, r), v, c,
                                    sel_pair(0u, ~0u));         // Z3 = Z1 H: N | X3 = r^2 - HHH - 2V: N'
    }
    szy = f29_swap_pair(P.zy);                                  // Y1 (even lane)
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = sel_pair(szy.v[i], r.v[i]);
        b.v[i] = sel_pair(s4.v[i], s4.v[i] - o5.v[i]);          // HHH | V - X3: (-2^29.2, 2^29 + 2^25)
    }
    f29_mul_ilp(o6, a, b);                                      // Y1 HHH | r (V - X3)
    s6 = f29_swap_pair(o6);
    s5 = f29_swap_pair(o5);                                     // X3 | Z3
    P.xb = f29_bcast_pair(o5, true);                            // X3 in both lanes
#pragma unroll
    for (int i = 0; i < 9; ++i) P.zy.v[i] = sel_pair(o5.v[i], o6.v[i] - s6.v[i]);  // Z3 | Y3 (N+-)
    P.zo = s5;                                                  // Z3 (odd lane)
}

#ifndef SBFT_PAIR_LANE_LOCAL
#define SBFT_PAIR_LANE_LOCAL 1
#endif

// ---------------------------------------------------------------- lane-local, W = c Z^2 carried
// The half kernel's two ladders (p256_verify_half_kernel) run the same instruction stream on two
// curves: pair A on the curve itself, pair B on E_c: y^2 = x^3 - 3c^2 x + b c^3 for c = r^3 - 3r
// + b, which (x, y) -> (c x, c y0 y) maps the curve onto when c = y0^2; R0 = (r, y0) lands on
// (c r, c^2), so pair B needs no square root. The doubling's a Z^4 term is then -3 (c Z^2)^2, so
// both pairs carry W = c Z^2 (c = 1 on pair A) and the step that squared Z computes (X - W)(X +
// W) directly (a general product instead of a square); W moves along as W3 = g W (doubling) and
// W HH (addition). The table entries are stored divided by c, so the addition's U2 = x2 Z1^2 is
// x2'' W and S2 = y2'' Z1 W. tests/test_f29_bounds.py (dbl_w, add_aff_w) checks every column,
// limb and contract, W = c Z^2 and X / W = x(k R0) on the curve.
// Halved representative as p29_dbl_h (X3 = h^2 - 2b, Y3 = h (b - X3) - g^2, Z3 = Y Z, h = 3a'/2):
//   1: a' = (X - W)(X + W) | g = Y^2      2: b = X g | W3 = W g
//   3: X3 = h^2 - 2b | L = g^2            4: Y3 = h (b - X3) - L | Z3 = Y Z
// In: X in N', Y in N' or N+-, Z, W in N. Out: X3, Y3 in N', Z3, W3 in N.
struct plw29 {
    f29 xb, zy, zo, w;  // X (both lanes), Z | Y, Z (odd lane), W (both lanes)
};
SBFT_DEV void p29_dbl_plw(plw29& P) {
    f29 a, b, o1, s1, o2, h, o3, s3, o4;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = sel_pair(P.xb.v[i] - P.w.v[i], P.zy.v[i]);   // X - W: |.| < 2^29.2 | Y
        b.v[i] = sel_pair(P.xb.v[i] + P.w.v[i], P.zy.v[i]);   // X + W < 2^30.1 | Y
    }
    f29_mul_ilp(o1, a, b);                                    // a' | g
    s1 = f29_swap_pair(o1);                                   // g | a'
    f29_mul_ilp(o2, f29_sel_pair(P.xb, P.w), f29_sel_pair(s1, o1));  // b = X g | W3 = W g
    f29_triple_half(h, o1);                                   // h = 3a'/2 (even lane; limbs < 2^29 + 3)
    {
        const f29 sq = f29_sel_pair(h, o1);
        const f29* const v[1] = {&o2};
        const u32 c[1] = {sel_pair((u32)-2, 0u)};
        f29_mulsq_add_ilp<true, 1>(o3, sq, sq, v, c, ~0u);   // X3 = h^2 - 2b | L = g^2: N'
    }
    s3 = f29_swap_pair(o3);                                   // L | X3
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = sel_pair(h.v[i], P.zy.v[i]);                 // h | Y
        b.v[i] = sel_pair(o2.v[i] - o3.v[i], P.zo.v[i]);      // b - X3: (-2^29.2, 2^29 + 2^25) | Z
    }
    {
        const f29* const v[1] = {&s3};
        const u32 c[1] = {sel_pair((u32)-1, 0u)};
        f29_mulsq_add_ilp<false, 1>(o4, a, b, v, c, sel_pair(~0u, 0u));  // Y3 = h (b - X3) - L: N' | Z3 = Y Z: N
    }
    P.xb = f29_sel_pair(o3, s3);                              // X3 in both lanes
    P.zy = f29_swap_pair(o4);                                 // Z3 | Y3
    P.zo = o4;                                                // Z3 (odd lane)
    P.w = f29_bcast_pair(o2, true);                           // W3 in both lanes
}
// The mixed addition with W (p29_add_aff_pl's steps 2-6, step 1 gone, W3 = W HH last):
//   1: U2 = x2'' W | T = Z1 W   2: HH = H^2 | S2 = y2'' T   3: V = X1 HH | HHH
//   4: Z3 = Z1 H | X3 = r^2 - HHH - 2V   5: Y1 HHH | r (V - X3)   6: W3 = W HH (both lanes)
// (x2'', y2'') = the entry divided by c, in both lanes (N, y2'' N+- when negated). Out: X3 in
// N', Y3 in N+-, Z3, W3 in N.
#ifndef SBFT_ADD_PLW5
#define SBFT_ADD_PLW5 1
#endif
// Five paired steps instead of six: W3 = W HH moves onto the even lane of the last step, whose
// odd lane computes Y3 = r (V - X3) - Y1 HHH in one f29_mul_sub_ilp (the even lane's second
// product is c 0). One reduction, the Y1 swap, the result swap and the Y3 subtraction fewer.
//   1: U2 = x2'' W | T = Z1 W   2: HH = H^2 | S2 = y2'' T   3: V = X1 HH | HHH
//   4: Z3 = Z1 H | X3 = r^2 - HHH - 2V   5: W3 = W HH | Y3 = r (V - X3) - Y1 HHH
// Out: X3 in N', Y3, Z3, W3 in N.
SBFT_DEV void p29_add_aff_plw5(plw29& P, const f29& x2, const f29& y2) {
    const u32 om = sel_pair(0u, ~0u);
    f29 o1, s1, h, o2, s2, hh, o3, s3, r, o4, a, b, nd, o5;
    f29_mul_ilp(o1, f29_sel_pair(x2, P.zo), P.w);             // U2 | T
    s1 = f29_swap_pair(o1);                                   // T | U2
#pragma unroll
    for (int i = 0; i < 9; ++i) h.v[i] = sel_pair(o1.v[i], s1.v[i]) - P.xb.v[i];  // H: (-2^29.2, 2^29 + 2^25)
    f29_mul_ilp(o2, f29_sel_pair(h, y2), f29_sel_pair(h, o1)); // HH | S2
    s2 = f29_swap_pair(o2);                                   // S2 | HH
    hh = f29_sel_pair(o2, s2);                                // HH in both lanes
    f29_mul_ilp(o3, f29_sel_pair(P.xb, h), hh);               // V | HHH
    s3 = f29_swap_pair(o3);                                   // HHH | V
    f29_sub(r, o2, P.zy);                                     // r = S2 - Y1 (odd lane): |.| < 2^29.2
    {
        const f29* const v[2] = {&o3, &s3};
        const u32 c[2] = {sel_pair(0u, (u32)-1), sel_pair(0u, (u32)-2)};
        f29_mulsq_add_ilp<false, 2>(o4, f29_sel_pair(P.zy, r), f29_sel_pair(h, r), v, c,
                                    sel_pair(0u, ~0u));       // Z3 = Z1 H: N | X3 = r^2 - HHH - 2V: N'
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = sel_pair(P.w.v[i], r.v[i]);                  // W | r
        b.v[i] = sel_pair(hh.v[i], s3.v[i] - o4.v[i]);        // HH | V - X3: (-2^29.2, 2^29 + 2^25)
        nd.v[i] = (0u - o3.v[i]) & om;                        // 0 | -HHH
    }
    f29_mul_sub_ilp(o5, a, b, P.zy, nd);                      // W3 | Y3 = r (V - X3) - Y1 HHH: N
    P.xb = f29_bcast_pair(o4, true);                          // X3 in both lanes
    P.zy = f29_sel_pair(o4, o5);                              // Z3 | Y3
    P.zo = f29_swap_pair(o4);                                 // Z3 (odd lane)
    P.w = f29_bcast_pair(o5, false);                          // W3 in both lanes
}
SBFT_DEV void p29_add_aff_plw(plw29& P, const f29& x2, const f29& y2) {
    if (SBFT_ADD_PLW5) {
        p29_add_aff_plw5(P, x2, y2);
        return;
    }
    f29 o1, s1, h, o2, s2, hh, o3, s3, r, o4, szy, a, b, o5, s5, s4, o6;
    f29_mul_ilp(o1, f29_sel_pair(x2, P.zo), P.w);             // U2 | T
    s1 = f29_swap_pair(o1);                                   // T | U2
#pragma unroll
    for (int i = 0; i < 9; ++i) h.v[i] = sel_pair(o1.v[i], s1.v[i]) - P.xb.v[i];  // H: (-2^29.2, 2^29 + 2^25)
    f29_mul_ilp(o2, f29_sel_pair(h, y2), f29_sel_pair(h, o1)); // HH | S2
    s2 = f29_swap_pair(o2);                                   // S2 | HH
    hh = f29_sel_pair(o2, s2);                                // HH in both lanes
    f29_mul_ilp(o6, P.w, hh);                                 // W3 = W HH (independent of steps 3-5)
    f29_mul_ilp(o3, f29_sel_pair(P.xb, h), hh);               // V | HHH
    s3 = f29_swap_pair(o3);                                   // HHH | V
    f29_sub(r, o2, P.zy);                                     // r = S2 - Y1 (odd lane): |.| < 2^29.2
    {
        const f29* const v[2] = {&o3, &s3};
        const u32 c[2] = {sel_pair(0u, (u32)-1), sel_pair(0u, (u32)-2)};
        f29_mulsq_add_ilp<false, 2>(o4, f29_sel_pair(P.zy, r), f29_sel_pair(h, r), v, c,
                                    sel_pair(0u, ~0u));       // Z3 = Z1 H: N | X3 = r^2 - HHH - 2V: N'
    }
    szy = f29_swap_pair(P.zy);                                // Y1 (even lane)
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = sel_pair(szy.v[i], r.v[i]);
        b.v[i] = sel_pair(s3.v[i], s3.v[i] - o4.v[i]);        // HHH | V - X3: (-2^29.2, 2^29 + 2^25)
    }
    f29_mul_ilp(o5, a, b);                                    // Y1 HHH | r (V - X3)
    s5 = f29_swap_pair(o5);
    s4 = f29_swap_pair(o4);                                   // X3 | Z3
    P.xb = f29_bcast_pair(o4, true);                          // X3 in both lanes
#pragma unroll
    for (int i = 0; i < 9; ++i) P.zy.v[i] = sel_pair(o4.v[i], o5.v[i] - s5.v[i]);  // Z3 | Y3 (N+-)
    P.zo = s4;                                                // Z3 (odd lane)
    P.w = o6;
}
SBFT_DEV void plw29_to(jp29& p, const plw29& q) {
    p.x = q.xb;
    p.y = f29_bcast_pair(q.zy, true);
    p.z = f29_bcast_pair(q.zy, false);
}

// ---------------------------------------------------------------- quads, W = c Z^2 carried
// The half kernel's wide form (p256_verify_half_kernel<FRAMED, true>: per-device shares of at
// most one workgroup per CU, e.g. a 10k proposal split over 2-8 GPUs) runs each 128-bit ladder on
// the four lanes of a quad instead of a pair. A step is still one product per lane in one
// instruction stream, so a step now carries four products. The doubling's depth is 3 (the Y
// chain: g = Y^2, then b and L, then Y3), the mixed addition's is 4, and its first step rides on
// the spare lanes of the doubling in front of it:
//   doubling:  1: a' = (X - W)(X + W) | g = Y^2 | Z3 = Y Z | (Y^2, unused)
//              2: h^2 | L = g^2 | b = X g | W3 = W g                 (h = 3a'/2, halved representative)
//              3: Y3 = h (3b - h^2) - L | X3 = h^2 - 2b [| U2 = x2'' W3 | T = Z3 W3]
//   addition:  2: - | HH = H^2 | Z3 = Z1 H | S2 = y2'' T              (H = U2 - X1)
//              3: V = X1 HH | HHH = H HH | W3 = W HH | r^2          (r = S2 - Y1)
//              4: r (V - X3) | Y1 HHH                                (X3 = r^2 - HHH - 2V: limb ops)
// (Y3 = h (b - X3) - L with b - X3 = 3b - h^2, so Y3 and X3 come out of the same step.) A 4-bit
// digit is 4 x 3 + 3 = 15 steps instead of the pair's 21. Every product is one the pair forms
// compute, with the same operand contracts except 3b - h^2 (limbs in (-2^29, 3 2^29): 9 column
// terms < 2^62.75, with the reduction terms < 2^62.8); tests/test_f29_bounds.py (dbl_q4,
// add_aff_q4) checks every column, limb and contract, W = c Z^2 and X / W = x(k R0).
// Lanes and registers (a value "@j" lives on lane j of its register):
//   doubling:  1: [a', g, Z3, a']       2: [h^2, L, W3, b]      3: [Y3, (U2), (T), X3]
//   addition:  2: [HH, HH, Z3, S2]      3: [V, HHH, W3, r^2]    4: [r (V - X3), Y1 HHH]
// a' runs on lanes 0 and 3, so h is on both lanes of step 3 without a move; the state is
// xy = [X, Y, Y, X] (one DPP of step 3's output), z = Z@2, w = W@2 (step 2's output) and
// wm = [W, 0, 0, W], so step 1's operands are xy - wm | xy + wm (lane 2: z) with one select.
// In: X in N', Y in N' or N+-, Z, W in N. Out: X3 in N', Y3 in N' (doubling) or N+- (addition),
// Z3, W3 in N.
struct q4w {
    f29 xy, z, w, wm;
};
constexpr u64 kQL0 = 0x1111111111111111ull, kQL1 = 0x2222222222222222ull, kQL2 = 0x4444444444444444ull,
              kQL3 = 0x8888888888888888ull;
template <u64 M>
SBFT_DEV u32 qsel(u32 a, u32 b) {  // b on the quad lanes of M, a elsewhere (one v_cndmask, as sel_pair)
    u32 r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(M));
    return r;
}
template <u64 M>
SBFT_DEV f29 f29_qsel(const f29& a, const f29& b) {
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = qsel<M>(a.v[i], b.v[i]);
    return r;
}
template <int CTRL>
SBFT_DEV f29 f29_qperm(const f29& a) {  // quad_perm DPP: lane j gets lane ((CTRL >> 2j) & 3)'s limbs
    f29 r;
#pragma unroll
    // (mov_dpp, not update_dpp(0, ..., bound_ctrl): with the latter ROCm 7.2's DPP combiner folds the
    // move into a consumer and the quad ladder came out wrong -- tools/isa/quad_unit.hip, round 6)
    for (int i = 0; i < 9; ++i) r.v[i] = (u32)__builtin_amdgcn_mov_dpp((int)a.v[i], CTRL, 0xF, 0xF, false);
    return r;
}
// b on the quad lanes of M, quad_perm CTRL of a elsewhere: one v_cndmask_b32_dpp per limb (the DPP
// applies to the select's src0), so a move and a select cost one instruction. The mask goes to VCC
// in the block; s_nop 1 covers the DPP read of a VGPR the instruction in front may have written.
#ifndef SBFT_QSELP_ASM
#define SBFT_QSELP_ASM 1
#endif
template <u64 M, int CTRL>
SBFT_DEV f29 f29_qselp(const f29& a, const f29& b) {
    f29 r;
    if (!SBFT_QSELP_ASM) {  // a move and a select per limb, scheduled limb by limb
        const f29 p = f29_qperm<CTRL>(a);
#pragma unroll
        for (int i = 0; i < 9; ++i) r.v[i] = qsel<M>(p.v[i], b.v[i]);
        return r;
    }
#define SBFT_QP "quad_perm:[%10,%11,%12,%13] row_mask:0xf bank_mask:0xf\n"
    asm("s_mov_b64 vcc, %9\n"
        "s_nop 1\n"
        "v_cndmask_b32_dpp %0, %14, %23, vcc " SBFT_QP
        "v_cndmask_b32_dpp %1, %15, %24, vcc " SBFT_QP
        "v_cndmask_b32_dpp %2, %16, %25, vcc " SBFT_QP
        "v_cndmask_b32_dpp %3, %17, %26, vcc " SBFT_QP
        "v_cndmask_b32_dpp %4, %18, %27, vcc " SBFT_QP
        "v_cndmask_b32_dpp %5, %19, %28, vcc " SBFT_QP
        "v_cndmask_b32_dpp %6, %20, %29, vcc " SBFT_QP
        "v_cndmask_b32_dpp %7, %21, %30, vcc " SBFT_QP
        "v_cndmask_b32_dpp %8, %22, %31, vcc " SBFT_QP
        : "=&v"(r.v[0]), "=&v"(r.v[1]), "=&v"(r.v[2]), "=&v"(r.v[3]), "=&v"(r.v[4]), "=&v"(r.v[5]), "=&v"(r.v[6]),
          "=&v"(r.v[7]), "=&v"(r.v[8])
        : "s"(M), "n"(CTRL & 3), "n"((CTRL >> 2) & 3), "n"((CTRL >> 4) & 3), "n"((CTRL >> 6) & 3), "v"(a.v[0]),
          "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]), "v"(a.v[6]), "v"(a.v[7]), "v"(a.v[8]),
          "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]), "v"(b.v[7]),
          "v"(b.v[8])
        : "vcc");
#undef SBFT_QP
    return r;
}
SBFT_DEV void q4w_set_w(q4w& P, const f29& w2) {  // W from lane 2 of w2
    P.w = w2;
    P.wm = f29_qselp<kQL1 | kQL2, 0xAA>(w2, f29{});
}
// The ladder's start: (x, y) on the curve (or E_c), Z = 1, W = c (every lane).
SBFT_DEV void q4w_init(q4w& P, const f29& x, const f29& y, const f29& one, const f29& c) {
    P.xy = f29_qsel<kQL1 | kQL2>(x, y);
    P.z = one;
    q4w_set_w(P, c);
}
// ADD: the next mixed addition's first step on lanes 1-2 of step 3 (U2 = x2 W3 | T = Z3 W3, in ut)
template <bool ADD>
SBFT_DEV void q4_dbl(q4w& P, const f29& x2, f29& ut) {
    f29 a, b, o1, h, o2, o3;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        a.v[i] = P.xy.v[i] - P.wm.v[i];                                  // X - W: |.| < 2^29.2 | Y | Y | X - W
        b.v[i] = qsel<kQL2>(P.xy.v[i] + P.wm.v[i], P.z.v[i]);            // X + W < 2^30.1 | Y | Z | X + W
    }
    f29_mul_ilp(o1, a, b);                   // a' | g | Z3 | a'
    f29_triple_half(h, o1);                  // h = 3a'/2 (lanes 0, 3; limbs < 2^29 + 3)
    b = f29_qselp<kQL0, 0x54>(o1, h);        // h | g | g | g (quad_perm [0,1,1,1])
#pragma unroll
    for (int i = 0; i < 9; ++i) a.v[i] = qsel<kQL2 | kQL3>(b.v[i], qsel<kQL3>(P.w.v[i], P.xy.v[i]));  // h | g | W | X
    f29_mul_ilp(o2, a, b);                   // h^2 | L | W3 | b
    const f29 bq = f29_qperm<0xFF>(o2);      // b (lane 0)
    const f29 v = f29_qperm<0xF5>(o2);       // quad_perm [1,1,3,3]: L (lane 0) | b (lane 3)
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const u32 t = bq.v[i] * 3u - o2.v[i];  // 3b - h^2 (lane 0): (-2^29, 3 2^29)
        b.v[i] = qsel<kQL3>(t, h.v[i]);        // 3b - h^2 | - | - | h
        a.v[i] = ADD ? qsel<kQL1>(qsel<kQL2>(h.v[i], o1.v[i]), x2.v[i]) : h.v[i];  // h | x2 | Z3 | h
    }
    if (ADD) b = f29_qselp<kQL0 | kQL3, 0xAA>(o2, b);  // 3b - h^2 | W3 | W3 | h
    {
        const f29* const vv[1] = {&v};
        const u32 c[1] = {qsel<kQL3>(qsel<kQL0>(0u, (u32)-1), (u32)-2)};
        f29_mulsq_add_ilp<false, 1>(o3, a, b, vv, c, qsel<kQL0 | kQL3>(0u, ~0u));  // Y3 | (U2 | T: N) | X3: N'
    }
    P.xy = f29_qperm<0xC3>(o3);  // quad_perm [3,0,0,3]: X3 | Y3 | Y3 | X3
    P.z = o1;                    // Z3 (lane 2)
    q4w_set_w(P, o2);            // W3 (lane 2)
    if (ADD) ut = o3;
}
// The mixed addition's steps 2-4 after q4_dbl<true> (ut = U2 | T on lanes 1 | 2), the entry
// (x2'', y2'') divided by c on every lane (y2'' N+- when negated). Y1 must be N' (a doubling's).
SBFT_DEV void q4_add_rest(q4w& P, const f29& y2, const f29& ut) {
    f29 h, a, b, o2, r, o3, t, x3, o4, y3;
    const f29 u = f29_qperm<0x95>(ut);    // quad_perm [1,1,1,2]: U2 | U2 | U2 | T
    const f29 xb = f29_qperm<0x00>(P.xy); // X1
    const f29 yb = f29_qperm<0x55>(P.xy); // Y1
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        h.v[i] = u.v[i] - xb.v[i];                                    // H = U2 - X1: (-2^29.2, 2^29 + 2^26)
        a.v[i] = qsel<kQL2>(qsel<kQL3>(h.v[i], y2.v[i]), P.z.v[i]);  // H | H | Z1 | y2
        b.v[i] = qsel<kQL3>(h.v[i], u.v[i]);                          // H | H | H | T
    }
    f29_mul_ilp(o2, a, b);                // HH | HH | Z3 | S2
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        r.v[i] = o2.v[i] - yb.v[i];  // r = S2 - Y1 (lane 3): |.| < 2^29.2
        a.v[i] = qsel<kQL1>(qsel<kQL2>(qsel<kQL3>(xb.v[i], r.v[i]), P.w.v[i]), h.v[i]);  // X1 | H | W | r
    }
    b = f29_qselp<kQL3, 0x00>(o2, r);     // HH | HH | HH | r
    f29_mul_ilp(o3, a, b);                // V | HHH | W3 | r^2
    const f29 vb = f29_qperm<0x00>(o3), hhh = f29_qperm<0x55>(o3), r2 = f29_qperm<0xFF>(o3);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = r2.v[i] - hhh.v[i] - (vb.v[i] << 1);  // r^2 - HHH - 2V: (-3 2^29, 2^29)
    f29_normalize(x3, t);                 // X3 (N')
    a = f29_qselp<kQL1, 0xFF>(r, yb);     // r | Y1
#pragma unroll
    for (int i = 0; i < 9; ++i) b.v[i] = qsel<kQL1>(vb.v[i] - x3.v[i], hhh.v[i]);  // V - X3: (-2^29.2, 2^29 + 2^26) | HHH
    f29_mul_ilp(o4, a, b);                // r (V - X3) | Y1 HHH
    const f29 p0 = f29_qperm<0x00>(o4), p1 = f29_qperm<0x55>(o4);
#pragma unroll
    for (int i = 0; i < 9; ++i) y3.v[i] = p0.v[i] - p1.v[i];  // Y3 (N+-)
    P.xy = f29_qsel<kQL1 | kQL2>(x3, y3);
    P.z = o2;  // Z3 (lane 2)
    q4w_set_w(P, o3);  // W3 (lane 2)
}
// A whole mixed addition (its first step on its own): Y1 brought to N' first, so any state qualifies.
SBFT_DEV void q4_add_full(q4w& P, const f29& x2, const f29& y2) {
    f29 ut;
    f29_normalize(P.xy, P.xy);
    f29_mul_ilp(ut, f29_qsel<kQL2>(x2, P.z), f29_qperm<0xAA>(P.w));  // U2 (lane 1) | T (lane 2)
    q4_add_rest(P, y2, ut);
}
// Jacobian (X, Y, Z) on every lane of the quad; Y in N'.
SBFT_DEV void q4w_to(jp29& p, const q4w& q) {
    p.x = f29_qperm<0x00>(q.xy);
    f29_normalize(p.y, f29_qperm<0x55>(q.xy));
    p.z = f29_qperm<0xAA>(q.z);
}
SBFT_DEV f29 q4w_w(const q4w& q) { return f29_qperm<0xAA>(q.w); }  // W on every lane

// ---------------------------------------------------------------- co-Z table building
// Odd multiples [1, 3, ..., 2^w - 1]Q with Meloni's co-Z additions (2007): every point of the
// chain shares the Z of the running 2Q, so an addition costs 4M + 2S and only the Z ratios
// h_k need keeping to make the table affine afterwards (one inversion per lane).
// N' = f29_normalize output (limbs in (-2^26, 2^29 + 2^26)).

// DBLU, a = -3, from affine P = (x, y) (N): D = 2P = (dx, dy) and P' = (px, py), both with
// Z = 2y (returned in z; limbs < 2^30). 2M + 4S. Outputs N'.
//   B = x^2, E = y^2, L = E^2, S = 4xE, M = 3(B - 1), X2 = M^2 - 2S, Y2 = M(S - X2) - 8L,
//   P' = (S, 8L)
SBFT_DEV void p29_dblu(const f29& x, const f29& y, f29& dx, f29& dy, f29& px, f29& py, f29& z) {
    f29 b, e, l, t, m, m2;
    f29_sqr(b, x);
    f29_sqr(e, y);
    f29_sqr(l, e);
    f29_mul(t, x, e);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] <<= 2;              // 4xE < 2^31
    f29_normalize(px, t);                                   // S (N')
    const f29 one = f29_const(C29_ONE);
#pragma unroll
    for (int i = 0; i < 9; ++i) m.v[i] = 3 * (b.v[i] - one.v[i]);  // |.| < 2^30.6
    f29_normalize(m, m);                                    // M (N')
    f29_sqr(m2, m);                                         // 2^29.2^2
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = m2.v[i] - (px.v[i] << 1);  // (-2^30.2, 2^29 + 2^27)
    f29_normalize(dx, t);                                   // X2 (N')
#pragma unroll
    for (int i = 0; i < 9; ++i) l.v[i] <<= 2;              // 4L < 2^31
    f29_normalize(l, l);
#pragma unroll
    for (int i = 0; i < 9; ++i) l.v[i] <<= 1;              // 8L, |.| < 2^30.2
    f29_normalize(py, l);                                   // 8L (N')
    f29_sub(t, px, dx);                                     // S - X2, |.| < 2^29.3
    f29_mul(m2, m, t);                                      // 2^29.2 x 2^29.3
    f29_sub(t, m2, py);                                     // (-2^29.2, 2^29)
    f29_normalize(dy, t);                                   // Y2 (N')
    f29_add(z, y, y);                                       // Z = 2y
}

// ZADDU: (dx, dy) = D and (tx, ty) = T share Z. T <- T + D and D <- D rescaled to the new
// Z = Z h, with h = X_D - X_T returned (4M + 2S). In: N or N'. Out: T in N', D in N, h with
// |limb| < 2^29.3. D == +-T (h = 0) cannot occur for the odd multiples of a point of prime
// order n: (2k+1)Q = +-2Q would need 2k+1 = +-2 mod n.
SBFT_DEV void p29_zaddu(f29& tx, f29& ty, f29& dx, f29& dy, f29& h) {
    f29 c, w1, w2, r, dd, a1, t;
    f29_sub(h, dx, tx);                                     // |.| < 2^29.3
    f29_sqr(c, h);
    f29_mul2(w1, dx, c, w2, tx, c);
    f29_sub(r, dy, ty);                                     // |.| < 2^29.3
    f29_sqr(dd, r);
    f29_sub(t, w1, w2);                                     // |.| < 2^29
    f29_mul(a1, dy, t);                                     // A1 = Y1 (W1 - W2)
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = dd.v[i] - w1.v[i] - w2.v[i];  // (-2^30, 2^29)
    f29_normalize(tx, t);                                   // X3 (N')
    f29_sub(t, w1, tx);                                     // |.| < 2^29.2
    f29_mul(c, r, t);                                       // 2^29.3 x 2^29.2
    f29_sub(t, c, a1);                                      // (-2^29, 2^29)
    f29_normalize(ty, t);                                   // Y3 (N')
    dx = w1;
    dy = a1;
}

// ---------------------------------------------------------------- conversions
// 8 x 32-bit limbs (a value < 2^256) -> 9 x 29-bit limbs (plain integer, not Montgomery).
SBFT_DEV f29 f29_from_u256(const fe& a) {
    f29 r;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        const u32 lo = a.v[w];
        const u32 hi = (w + 1 < 8) ? a.v[w + 1] : 0u;
        r.v[i] = __builtin_amdgcn_alignbit(hi, lo, s) & F29_MASK;
    }
    return r;
}
// x R mod p (8 x 32 Montgomery form, R = 2^256, canonical) -> the radix-2^29 Montgomery form
// x 2^261 mod p without a multiplication: the 9 limbs of 32 x R (< 2^261; limb i = bits
// [29 i - 5, 29 i + 24) of x R), then its 2^256 multiple q folded back with
// 2^256 = 2^224 - 2^192 - 2^96 + 1 (mod p): q << 21 at limb 7, -q << 18 at limb 6, -q << 9 at
// limb 3, +q at limb 0 (q < 32). Out: value in [0, 2^257), limbs 0..7 in (-2^23, 2^29 + 2^26),
// limb 8 in [0, 2^24) (within N').
SBFT_DEV f29 f29_from_mont256(const fe& a) {
    f29 r;
    r.v[0] = (a.v[0] << 5) & F29_MASK;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        const int bit = 29 * i - 5, w = bit >> 5, s = bit & 31;
        const u32 lo = a.v[w];
        const u32 hi = (w + 1 < 8) ? a.v[w + 1] : 0u;
        r.v[i] = __builtin_amdgcn_alignbit(hi, lo, s) & F29_MASK;
    }
    const u32 q = r.v[8] >> 24;
    r.v[8] &= 0x00FFFFFFu;
    r.v[7] += q << 21;
    r.v[6] -= q << 18;
    r.v[3] -= q << 9;
    r.v[0] += q;
    return r;
}

// Full normalisation to [0, 2^261) limbs-in-range form via a carry chain; |x| < 2^260 in,
// value x mod 2^261 out (callers add a multiple of p first when x may be negative).
SBFT_DEV void f29_norm_chain(f29& r, const f29& a) {
    i32 c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const i32 t = (i32)a.v[i] + c;
        r.v[i] = (u32)t & F29_MASK;
        c = t >> 29;
    }
    r.v[8] = a.v[8] + (u32)c;
}
// limbs in range (after f29_norm_chain, value in [0, 2^256+...)) -> 8 x 32-bit limbs (low 256 bits)
SBFT_DEV fe f29_to_u256(const f29& a) {
    fe r;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int bit = 32 * w, i = bit / 29, s = bit % 29;
        u64 x = (u64)a.v[i] >> s;
        x |= (u64)a.v[i + 1] << (29 - s);
        if (i + 2 < 9) x |= (u64)a.v[i + 2] << (58 - s);
        r.v[w] = (u32)x;
    }
    return r;
}

// Canonical plain value of a Montgomery f29 element: a * 2^-261 mod p in [0, p), as 8 x 32
// limbs. Once per verify (final comparison), so written for clarity, not speed.
SBFT_DEV fe f29_canon_plain(const f29& a) {
    f29 one;
#pragma unroll
    for (int i = 0; i < 9; ++i) one.v[i] = i == 0 ? 1u : 0u;
    f29 t;
    f29_mul(t, a, one);              // plain value, |t| < 2^256 + 2^1
    f29 p2 = f29_const(C29_2P);
    f29_add(t, t, p2);               // positive: (0, 2^258)
    f29_norm_chain(t, t);            // limbs 0..7 in [0, 2^29), limb 8 in [0, 2^26)
    // 8 low words + bits 256.. (top < 4), then subtract p while the value is >= p
    fe lo = f29_to_u256(t);
    u32 top = t.v[8] >> 24;
#pragma unroll 1
    for (int it = 0; it < 4; ++it) {
        fe d;
        u64 bw = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const u64 x = (u64)lo.v[k] - P256_P[k] - bw;
            d.v[k] = lo32(x);
            bw = x >> 63;
        }
        if (top >= (u32)bw) {  // value - p >= 0
            top -= (u32)bw;
            lo = d;
        }
    }
    return lo;
}

// Exceptional additions done in place (add_aff_careful below) leave R = infinity as the
// caller's flag; a lean addition that met one anyway leaves Z = 0 from there on, so
// Z == 0 (mod p) flags the tuple for the general path (exc). Otherwise x(R) mod n == r is
// checked projectively: X == r Z^2 or, when r + n < p, X == (r + n) Z^2. acc.z in normal form.
SBFT_DEV bool verify_final(const jp29& acc, const fe& rv, bool& exc) {
    exc = f29_zero_mod_p(acc.z);
    const f29 r2 = f29_const(C29_R2);
    f29 z2, lhs, rm, t;
    f29_sqr(z2, acc.z);
    f29_mul(rm, f29_from_u256(rv), r2);
    f29_mul(lhs, rm, z2);
    f29_sub(t, acc.x, lhs);  // X - r Z^2: |limb| < 2^30, |t| < 2^259
    bool accept = f29_zero_mod_p_any(t);
    // R.x in [n, p): compare with r + n as well when r + n < p
    fe rn;
    u64 c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c = (u64)rv.v[k] + P256_N[k] + c;
        rn.v[k] = lo32(c);
        c >>= 32;
    }
    if (c == 0 && fe_lt(rn, P256_P)) {
        f29_mul(rm, f29_from_u256(rn), r2);
        f29_mul(lhs, rm, z2);
        f29_sub(t, acc.x, lhs);
        accept = accept || f29_zero_mod_p_any(t);
    }
    return accept;
}

}  // namespace sbft
