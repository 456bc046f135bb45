// sinv_host.hpp — s^-1 for a batch of signatures on the host, in the Montgomery form mod n the
// keyed wavefront kernel's products take (gpuverify.cpp enqueue_keyed: small zero-copy batches
// skip the kernel's own divstep table and safegcd, ~15 us of its ~45). Header-only and free of
// HIP types: tests/native/sinv_test.cpp checks it against Python's pow(s, -1, n).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <array>
#include <vector>

#include "modn_host.hpp"
#include "p256_inv.hpp"

namespace sbft {
namespace modn {

// w_i = s_i^-1 R mod n (R = 2^256: the Montgomery form the keyed kernel's fn_ products take)
// for n big-endian s values, as 8 little-endian words each, by Montgomery's trick: the
// Montgomery forms' prefix products, ONE safegcd (p256_inv.hpp, the kernels' own inversion, here
// on the host) of the last with c = R^2 mod n, which gives M(p^-1) = R^2 / M(p), then two products
// per element going back. An s outside [1, n) stands in as 1 (its verdict is false whatever w
// is: the kernel checks r and s itself). ~4 products of ~20 ns per signature + ~1.7 us.
inline void sinv_batch_mont(const uint8_t* s_be, size_t n, uint32_t* w_out) {
    static const uint32_t kDivstep5[SBFT_DIVSTEP5_WORDS] = SBFT_DIVSTEP5_TABLE;
    if (n == 0) return;
    std::vector<std::array<u64, 4>> sm(n), pre(n);
    for (size_t i = 0; i < n; ++i) {
        u64 v[4];
        for (int k = 0; k < 4; ++k) {
            u64 x = 0;
            for (int j = 0; j < 8; ++j) x = (x << 8) | s_be[32 * i + 8 * (3 - k) + j];
            v[k] = x;
        }
        if ((v[0] | v[1] | v[2] | v[3]) == 0 || geq_n(v)) v[0] = 1, v[1] = v[2] = v[3] = 0;
        mont_mul(sm[i].data(), v, R2);  // M(s_i)
        if (i == 0) pre[0] = sm[0];
        else mont_mul(pre[i].data(), pre[i - 1].data(), sm[i].data());  // M(s_0 ... s_i)
    }
    uint32_t x[8], c[8], o[8];
    for (int k = 0; k < 4; ++k) {
        x[2 * k] = (uint32_t)pre[n - 1][k];
        x[2 * k + 1] = (uint32_t)(pre[n - 1][k] >> 32);
        c[2 * k] = (uint32_t)R2[k];
        c[2 * k + 1] = (uint32_t)(R2[k] >> 32);
    }
    inv::inv_mod(o, x, kDivstep5, false, c);  // R^2 / M(p) = M(p^-1)
    u64 acc[4];
    for (int k = 0; k < 4; ++k) acc[k] = (u64)o[2 * k] | ((u64)o[2 * k + 1] << 32);
    auto put = [&](size_t i, const u64* w) {
        for (int k = 0; k < 4; ++k) {
            w_out[8 * i + 2 * k] = (uint32_t)w[k];
            w_out[8 * i + 2 * k + 1] = (uint32_t)(w[k] >> 32);
        }
    };
    for (size_t i = n - 1; i > 0; --i) {
        u64 w[4], t[4];
        mont_mul(w, acc, pre[i - 1].data());  // M(s_i^-1)
        put(i, w);
        mont_mul(t, acc, sm[i].data());  // M((s_0 ... s_{i-1})^-1)
        for (int k = 0; k < 4; ++k) acc[k] = t[k];
    }
    put(0, acc);
}

}  // namespace modn
}  // namespace sbft
