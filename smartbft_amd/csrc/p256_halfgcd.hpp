// p256_halfgcd.hpp — half-size scalars for the latency verify kernel (p256_verify_half_kernel).
//
// Accelerated ECDSA verification (Antipa, Brown, Gallant, Lambert, Struik, Vanstone, "Accelerated
// verification of ECDSA signatures", SAC 2005). Go's check is x(u1 G + u2 Q) mod n == r. For
// r >= p - n the only candidate is R' = (r, +-y), and with v u2 = w (mod n):
//   v (u1 G + u2 Q) = (v u1) G + w Q,
// so R' = +-R0 (R0 = (r, sqrt(r^3 - 3r + b))) iff x((v u1) G + w Q) == x(v R0). With |v| and w
// below 2^128, the two variable-base multiplications are 128-bit ladders that run side by side
// on two lane pairs, instead of one 256-bit ladder.
//
// v, w come from the extended Euclidean algorithm on (n, u2), stopped at the first remainder
// w = r_i < 2^128; its cofactor t_i (r_i = t_i u2 mod n) has |t_i| <= n / r_{i-1} < 2^128. Each
// quotient q = floor(a / b) is estimated in double precision from the whole operands (relative
// error < 2^-49, so for q < 2^31 the estimate is off by at most one) and corrected once. A
// quotient >= 2^31 (an adversarial u2; honest ones never get near it), a second correction or
// an exhausted step budget clears `ok`: the kernel then verifies that tuple the classic way
// (v = 1, w = u2, a 256-bit ladder). The caller checks v u2 == +-w mod n before using a result.
//
// Header-only and free of HIP types (as p256_inv.hpp), so that tests/native/hgcd_test.cpp
// compiles the same code for the CPU and tests/test_native.py checks it against Python's exact
// Euclid.
#pragma once
#include <math.h>
#include <stdint.h>

#include "p256_inv.hpp"  // SBFT_HD, SBFT_UNROLL1

#ifndef SBFT_HGCD_LEHMER
#define SBFT_HGCD_LEHMER 1  // lehmer() batches (0: one step() per quotient, the round-4 form)
#endif

namespace sbft {
namespace hgcd {

// the group order n, little-endian 32-bit words
#define SBFT_HGCD_N {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu}

struct state {
    uint32_t a[8], b[8];   // remainders r_{i-1} > r_i
    uint32_t ta[5], tb[5]; // |t_{i-1}|, |t_i| (< 2^129 while b >= 2^128)
    bool neg;              // t_i < 0 (the signs alternate: t_1 = 1, t_2 = -q_1, ...)
    bool ok;
};

SBFT_HD void init(state& s, const uint32_t u[8]) {
    const uint32_t n[8] = SBFT_HGCD_N;
    for (int k = 0; k < 8; ++k) {
        s.a[k] = n[k];
        s.b[k] = u[k];
    }
    for (int k = 0; k < 5; ++k) {
        s.ta[k] = 0;
        s.tb[k] = 0;
    }
    s.tb[0] = 1;
    s.neg = false;
    s.ok = true;
}

// another step is due: b >= 2^128 (and no failure so far)
SBFT_HD bool more(const state& s) { return s.ok && (s.b[4] | s.b[5] | s.b[6] | s.b[7]) != 0; }

// nearest-ish double of a 256-bit value (8 roundings: relative error < 2^-49)
SBFT_HD double to_f64(const uint32_t x[8]) {
    double d = 0.0;
    for (int k = 7; k >= 0; --k) d = d * 4294967296.0 + (double)x[k];
    return d;
}

// One Euclid step: q = floor(a / b), (a, b) <- (b, a - q b), (ta, tb) <- (tb, ta + q tb).
SBFT_HD void step(state& s) {
    const double qd = floor(to_f64(s.a) / to_f64(s.b));
    if (!(qd < 2147483648.0) || !(qd >= 0.0)) {  // also NaN / inf (b == 0 cannot happen for u2 != 0)
        s.ok = false;
        return;
    }
    uint32_t q = (uint32_t)qd;
    // r = a - q b, with the bits at 2^256 and up in `top` (signed)
    uint32_t r[8];
    uint64_t pc = 0;
    int64_t bw = 0;
    for (int k = 0; k < 8; ++k) {
        const uint64_t pr = (uint64_t)q * s.b[k] + pc;
        pc = pr >> 32;
        const int64_t x = (int64_t)s.a[k] - (int64_t)(uint32_t)pr + bw;
        r[k] = (uint32_t)x;
        bw = x >> 32;  // 0 or -1
    }
    int64_t top = bw - (int64_t)pc;
    if (top < 0) {  // q one too large: r += b
        uint64_t c = 0;
        for (int k = 0; k < 8; ++k) {
            const uint64_t x = (uint64_t)r[k] + s.b[k] + c;
            r[k] = (uint32_t)x;
            c = x >> 32;
        }
        top += (int64_t)c;
        q -= 1;
    } else {  // q one too small (r >= b): r -= b
        int64_t d = 0;
        uint32_t t[8];
        for (int k = 0; k < 8; ++k) {
            const int64_t x = (int64_t)r[k] - (int64_t)s.b[k] + d;
            t[k] = (uint32_t)x;
            d = x >> 32;
        }
        if (d == 0) {  // r - b >= 0
            for (int k = 0; k < 8; ++k) r[k] = t[k];
            q += 1;
        }
    }
    // 0 <= r < b must hold now, else the estimate was off by more than one
    {
        int64_t d = 0;
        for (int k = 0; k < 8; ++k) d = ((int64_t)r[k] - (int64_t)s.b[k] + d) >> 32;
        if (top != 0 || d == 0) {
            s.ok = false;
            return;
        }
    }
    // tn = ta + q tb (magnitudes; |t_{i+1}| <= n / r_i <= 2^128 while b = r_i >= 2^128)
    uint32_t tn[5];
    uint64_t c = 0;
    for (int k = 0; k < 5; ++k) {
        const uint64_t x = (uint64_t)q * s.tb[k] + s.ta[k] + c;
        tn[k] = (uint32_t)x;
        c = x >> 32;
    }
    if (c != 0 || tn[4] > 1u) {
        s.ok = false;
        return;
    }
    for (int k = 0; k < 8; ++k) {
        s.a[k] = s.b[k];
        s.b[k] = r[k];
    }
    for (int k = 0; k < 5; ++k) {
        s.ta[k] = s.tb[k];
        s.tb[k] = tn[k];
    }
    s.neg = !s.neg;
}

// ---- Lehmer steps: many quotients from the leading 53 bits, one multi-word update ----
// Knuth's Algorithm L (TAOCP vol. 2, 4.5.2) on x = floor(a / 2^s), y = floor(b / 2^s), s = len(a)
// - 53, all exact in double precision. (A B; C D) is the cofactor matrix of the steps taken, so
// the true remainders are (A a + B b, C a + D b) and, scaled by 2^-s, lie within [x + min(A, B),
// x + max(A, B)] and [y + min(C, D), y + max(C, D)] (the entries of a row have opposite signs).
// A quotient is taken only when both corners give it -- floor((x + A) / (y + C)) ==
// floor((x + B) / (y + D)) -- so it is the true quotient; only while the true b is surely still
// >= 2^128 (y + min(C, D) >= 2^(128 - s)), so the reduction stops where step() would; and only
// while the new entries stay below 2^30 (signed 32-bit multipliers for the update). Every
// quotient estimate is within one of the truth (x, y < 2^53, rcp53) and the remainder x - q y,
// formed exactly by an FMA, corrects it. Returns false when no quotient could be taken (the caller then runs one step()).
SBFT_HD double hgcd_lead53(const uint32_t x[8], int ka, int sh) {
    // bits [32 ka + 32 - ... ] of x: the words ka, ka - 1, ka - 2 (ka >= 4), shifted right by sh
    uint32_t w2 = 0, w1 = 0, w0 = 0;
SBFT_UNROLL
    for (int k = 2; k < 8; ++k) {
        if (k == ka) w2 = x[k];
        if (k == ka - 1) w1 = x[k];
        if (k == ka - 2) w0 = x[k];
    }
    // (w2 w1 w0) >> sh, sh in [12, 43]: the result has at most 53 bits
    const uint64_t hi = ((uint64_t)w2 << 32) | w1;
    uint64_t v;
    if (sh >= 32) v = hi >> (sh - 32);
    else v = (hi << (32 - sh)) | (w0 >> sh);
    return (double)v;
}

// 1 / y: v_rcp_f64 and one Newton step on the device (the IEEE division is a ten-instruction
// dependent chain); the host build starts from a float reciprocal (2 steps), so that
// tests/test_native.py exercises the same correction with a rough first estimate. With q below
// 2^31 (the cofactor cap) floor(x1 / y1) is then off by at most one either way and the remainder
// fixes it; a worse estimate fails the remainder test and only ends the round.
SBFT_HD double rcp53(double y) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double r = __builtin_amdgcn_rcp(y);
    return fma(fma(-y, r, 1.0), r, r);
#else
    double r = (double)(float)(1.0 / y);
    r = fma(fma(-y, r, 1.0), r, r);
    return fma(fma(-y, r, 1.0), r, r);
#endif
}

// The quotient batch of a Lehmer round: the cofactor matrix (A B; C D) of the k quotients taken.
struct lmat {
    double A, B, C, D;
    int k;
};
SBFT_HD lmat lehmer_quotients(const state& s) {
    int ka = 7;
SBFT_UNROLL
    for (int k = 4; k < 8; ++k)
        if (s.a[k] != 0) ka = k;  // a >= b >= 2^128: the top word is at 4..7
    uint32_t top = 0;
SBFT_UNROLL
    for (int k = 4; k < 8; ++k)
        if (k == ka) top = s.a[k];
    const int len = 32 * ka + 32 - __builtin_clz(top);  // bit length of a, >= 129
    const int sft = len - 53;                            // >= 76
    const int sh = sft - 32 * (ka - 2);                  // in [12, 43]
    double x = hgcd_lead53(s.a, ka, sh), y = hgcd_lead53(s.b, ka, sh);
    const double thr = ldexp(1.0, 128 - sft);  // 2^128 / 2^s
    double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
    int k = 0;
    const double cap = 1073741824.0;  // 2^30
SBFT_UNROLL1
    for (; k < 64; ++k) {
        // every condition from independent values, one exit test: the per-step dependent chain
        // is y1 -> rcp -> q -> remainder -> (x, y) (a branch per test cost more than the test)
        const double y1 = y + C, y2 = y + D, x1 = x + A, x2 = x + B;
        double q = floor(x1 * rcp53(y1));
        const double rm = fma(-q, y1, x1);  // exact: |x1 - q y1| < 2^53
        q = rm < 0.0 ? q - 1.0 : (rm >= y1 ? q + 1.0 : q);
        const double rq = fma(-q, y1, x1), r2 = fma(-q, y2, x2);
        const double nc = fma(-q, C, A), nd = fma(-q, D, B);
        const bool ok = (y + fmin(C, D) >= thr) & (y1 > 0.0) & (y2 > 0.0) & (rq >= 0.0) & (rq < y1) &
                        (r2 >= 0.0) & (r2 < y2) & (fabs(nc) < cap) & (fabs(nd) < cap);
        // refused: the true b may be below 2^128, the corners disagree (or the estimate was off by
        // more than one), or an entry would reach 2^30
        if (!ok) break;
        const double ny = fma(-q, y, x);
        A = C;
        B = D;
        C = nc;
        D = nd;
        x = y;
        y = ny;
    }
    return lmat{A, B, C, D, k};
}

// The same quotient batch with exactly K candidate steps and no branch: a step's conditions go
// through one chain of minima into one comparison (every value is an integer below 2^53, so
// a >= b is a - b + 1/2 > 0), and a refused step freezes the lane for the rest of the batch.
// One wavefront runs K steps per round whatever its lanes do (the variable loop ran its slowest
// lane's count plus the exit tests: VALU compares into SGPR masks, scalar ANDs, exec updates).
template <int K>
SBFT_HD lmat lehmer_quotients_k(const state& s) {
    int ka = 7;
SBFT_UNROLL
    for (int k = 4; k < 8; ++k)
        if (s.a[k] != 0) ka = k;
    uint32_t top = 0;
SBFT_UNROLL
    for (int k = 4; k < 8; ++k)
        if (k == ka) top = s.a[k];
    const int len = 32 * ka + 32 - __builtin_clz(top);
    const int sft = len - 53;
    const int sh = sft - 32 * (ka - 2);
    double x = hgcd_lead53(s.a, ka, sh), y = hgcd_lead53(s.b, ka, sh);
    const double thr = ceil(ldexp(1.0, 128 - sft)) - 0.5;  // y + min(C, D) >= 2^(128-s), integers
    const double cap = 1073741824.0;                       // 2^30
    double A = 1.0, B = 0.0, C = 0.0, D = 1.0, kk = 0.0;
    bool live = true;
SBFT_UNROLL
    for (int j = 0; j < K; ++j) {
        const double y1 = y + C, y2 = y + D, x1 = x + A, x2 = x + B;
        double q = floor(x1 * rcp53(y1));
        const double rm = fma(-q, y1, x1);
        q = rm < 0.0 ? q - 1.0 : (rm >= y1 ? q + 1.0 : q);
        const double rq = fma(-q, y1, x1), r2 = fma(-q, y2, x2);
        const double nc = fma(-q, C, A), nd = fma(-q, D, B);
        const double m1 = fmin(fmin(y + fmin(C, D) - thr, fmin(y1, y2)), fmin(rq + 0.5, y1 - rq));
        const double m2 = fmin(fmin(r2 + 0.5, y2 - r2), cap - fmax(fabs(nc), fabs(nd)));
        live = live && fmin(m1, m2) > 0.0;
        const double ny = fma(-q, y, x);
        A = live ? C : A;
        B = live ? D : B;
        C = live ? nc : C;
        D = live ? nd : D;
        x = live ? y : x;
        y = live ? ny : y;
        kk += live ? 1.0 : 0.0;
    }
    return lmat{A, B, C, D, (int)kk};
}

#ifndef SBFT_HGCD_K
#define SBFT_HGCD_K 16  // candidate steps per Lehmer round (0: the variable-length loop)
#endif
SBFT_HD bool lehmer(state& s) {
    const lmat m = SBFT_HGCD_K ? lehmer_quotients_k<SBFT_HGCD_K ? SBFT_HGCD_K : 1>(s) : lehmer_quotients(s);
    const int k = m.k;
    if (k == 0) return false;
    const int32_t iA = (int32_t)m.A, iB = (int32_t)m.B, iC = (int32_t)m.C, iD = (int32_t)m.D;
    uint32_t na[8], nb[8];
    int64_t ca = 0, cb = 0;
SBFT_UNROLL
    for (int j = 0; j < 8; ++j) {  // (A a + B b, C a + D b): both exact remainders, >= 0
        ca += (int64_t)iA * (int64_t)s.a[j] + (int64_t)iB * (int64_t)s.b[j];
        cb += (int64_t)iC * (int64_t)s.a[j] + (int64_t)iD * (int64_t)s.b[j];
        na[j] = (uint32_t)ca;
        nb[j] = (uint32_t)cb;
        ca >>= 32;
        cb >>= 32;
    }
    // cofactor magnitudes: the signs alternate along the sequence and across each matrix row,
    // so |A t_a + B t_b| = |A| |t_a| + |B| |t_b|
    const uint32_t mA = (uint32_t)(iA < 0 ? -iA : iA), mB = (uint32_t)(iB < 0 ? -iB : iB);
    const uint32_t mC = (uint32_t)(iC < 0 ? -iC : iC), mD = (uint32_t)(iD < 0 ? -iD : iD);
    uint32_t nta[5], ntb[5];
    uint64_t ua = 0, ub = 0;  // products < 2^62 each: a limb's sum stays below 2^64
SBFT_UNROLL
    for (int j = 0; j < 5; ++j) {
        ua += (uint64_t)mA * s.ta[j] + (uint64_t)mB * s.tb[j];
        ub += (uint64_t)mC * s.ta[j] + (uint64_t)mD * s.tb[j];
        nta[j] = (uint32_t)ua;
        ntb[j] = (uint32_t)ub;
        ua >>= 32;
        ub >>= 32;
    }
    if (ca != 0 || cb != 0 || ua != 0 || ub != 0 || ntb[4] > 1u) {  // cannot happen; the caller's
        s.ok = false;                                                // relation check is the net
        return true;
    }
SBFT_UNROLL
    for (int j = 0; j < 8; ++j) {
        s.a[j] = na[j];
        s.b[j] = nb[j];
    }
SBFT_UNROLL
    for (int j = 0; j < 5; ++j) {
        s.ta[j] = nta[j];
        s.tb[j] = ntb[j];
    }
    if (k & 1) s.neg = !s.neg;
    return true;
}

// Outputs of a finished state: w = r_i (< 2^128), |v| = |t_i| (<= 2^128), v < 0.
SBFT_HD void result(const state& s, uint32_t w[8], uint32_t v[8], bool& vneg) {
    for (int k = 0; k < 8; ++k) {
        w[k] = s.b[k];
        v[k] = k < 5 ? s.tb[k] : 0u;
    }
    vneg = s.neg;
}

// The whole reduction for one u2 (host form; the kernel runs step() under a wave-wide loop).
SBFT_HD bool half_gcd(const uint32_t u[8], uint32_t w[8], uint32_t v[8], bool& vneg) {
    state s;
    init(s, u);
    for (int it = 0; it < 400 && more(s); ++it)
        if (!SBFT_HGCD_LEHMER || !lehmer(s)) step(s);
    if (more(s)) s.ok = false;
    result(s, w, v, vneg);
    return s.ok;
}

}  // namespace hgcd
}  // namespace sbft
