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
    for (int it = 0; it < 400 && more(s); ++it) step(s);
    if (more(s)) s.ok = false;
    result(s, w, v, vneg);
    return s.ok;
}

}  // namespace hgcd
}  // namespace sbft
