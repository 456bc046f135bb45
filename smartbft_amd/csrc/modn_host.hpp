// modn_host.hpp — host-side arithmetic mod the P-256 group order n, for the pre-signature
// signer (verifier.cpp, sbft_signer_presign): the online half of a pooled signature is
// s = A e + B (mod n), one product and one addition; the GPU computed A = k^-1 and B = k^-1 r d
// with k G. Four 64-bit limbs, little-endian, Montgomery multiplication (CIOS) with R = 2^256.
// Header-only and free of HIP types so tests/native/modn_test.cpp checks it against Python.
#pragma once
#include <stdint.h>

namespace sbft {
namespace modn {

typedef uint64_t u64;
typedef unsigned __int128 u128;

static const u64 N[4] = {0xf3b9cac2fc632551ull, 0xbce6faada7179e84ull, 0xffffffffffffffffull,
                         0xffffffff00000000ull};
static const u64 N0INV = 0xccd1c8aaee00bc4full;  // -n^-1 mod 2^64
static const u64 R2[4] = {0x83244c95be79eea2ull, 0x4699799c49bd6fa6ull, 0x2845b2392b6bec59ull,
                          0x66e12d94f3d95620ull};  // 2^512 mod n

// a >= n ? (a < 2^256)
inline bool geq_n(const u64 a[4]) {
    for (int i = 3; i >= 0; --i)
        if (a[i] != N[i]) return a[i] > N[i];
    return true;
}
// a -= n (a >= n, or a carry out of 2^256 pending: the wrap is the right value then)
inline void sub_n(u64 a[4]) {
    u64 b = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 d = (u128)a[i] - N[i] - b;
        a[i] = (u64)d;
        b = (u64)(d >> 64) & 1u;
    }
}

// r = a b 2^-256 mod n for a, b < n
inline void mont_mul(u64 r[4], const u64 a[4], const u64 b[4]) {
    u64 t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a[j] * b[i] + t[j];
            t[j] = (u64)c;
            c >>= 64;
        }
        c += t[4];
        t[4] = (u64)c;
        t[5] = (u64)(c >> 64);
        const u64 m = t[0] * N0INV;
        c = (u128)m * N[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; ++j) {
            c += (u128)m * N[j] + t[j];
            t[j - 1] = (u64)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (u64)c;
        t[4] = t[5] + (u64)(c >> 64);
    }
    for (int i = 0; i < 4; ++i) r[i] = t[i];
    if (t[4] || geq_n(r)) sub_n(r);
}

// r = a b mod n for a, b < n
inline void mul_mod(u64 r[4], const u64 a[4], const u64 b[4]) {
    u64 t[4];
    mont_mul(t, a, b);  // a b 2^-256
    mont_mul(r, t, R2);  // a b
}

// r = a + b mod n for a, b < n
inline void add_mod(u64 r[4], const u64 a[4], const u64 b[4]) {
    u64 c = 0;
    for (int i = 0; i < 4; ++i) {
        const u128 s = (u128)a[i] + b[i] + c;
        r[i] = (u64)s;
        c = (u64)(s >> 64);
    }
    if (c || geq_n(r)) sub_n(r);
}

// 32 big-endian bytes <-> limbs; from_be32 reduces once (any 256-bit value < 2n)
inline void from_be32(u64 r[4], const uint8_t b[32]) {
    for (int i = 0; i < 4; ++i) {
        u64 w = 0;
        for (int k = 0; k < 8; ++k) w = (w << 8) | b[8 * (3 - i) + k];
        r[i] = w;
    }
    if (geq_n(r)) sub_n(r);
}
inline void to_be32(uint8_t b[32], const u64 a[4]) {
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 8; ++k) b[8 * (3 - i) + k] = (uint8_t)(a[i] >> (56 - 8 * k));
}
inline bool is_zero(const u64 a[4]) { return (a[0] | a[1] | a[2] | a[3]) == 0; }

}  // namespace modn
}  // namespace sbft
