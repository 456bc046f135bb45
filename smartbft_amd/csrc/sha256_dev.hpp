// sha256_dev.hpp — SHA-256 (FIPS 180-4) device routines shared by the batched hashing kernel
// (sha256.hip) and the keyed consenter-signature kernel (p256_keyed.hip), which hashes each
// signature message inside the verify launch. One message per lane; arbitrary byte
// alignment via v_alignbyte funnel shifts; the caller's blob is readable >= 68 bytes past
// its last message.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sbft {

__device__ __constant__ static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// x ^ y ^ z in one v_bitop3_b32 (truth table 0x96); the compiler emits two v_xor_b32 otherwise
__device__ __forceinline__ uint32_t xor3(uint32_t x, uint32_t y, uint32_t z) {
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
}

__device__ __forceinline__ void compress(uint32_t h[8], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // (e & f) | (~e & g)
        const uint32_t t1 = hh + S1 + ch + K256[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t maj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
        const uint32_t t2 = S0 + maj;
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
}

// M independent compressions interleaved round by round: the M dependency chains give the
// scheduler M x the instruction-level parallelism of one (SHA-256's rounds are a serial chain).
// live[m] false: the state of message m is left unchanged.
template <int M>
__device__ __forceinline__ void compress_multi(uint32_t (&h)[M][8], uint32_t (&w)[M][16], const bool (&live)[M]) {
    uint32_t a[M], b[M], c[M], d[M], e[M], f[M], g[M], hh[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        a[m] = h[m][0]; b[m] = h[m][1]; c[m] = h[m][2]; d[m] = h[m][3];
        e[m] = h[m][4]; f[m] = h[m][5]; g[m] = h[m][6]; hh[m] = h[m][7];
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            uint32_t wi;
            if (i < 16) {
                wi = w[m][i];
            } else {
                const uint32_t w15 = w[m][(i + 1) & 15], w2 = w[m][(i + 14) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                wi = w[m][i & 15] + s0 + w[m][(i + 9) & 15] + s1;
                w[m][i & 15] = wi;
            }
            const uint32_t S1 = xor3(rotr(e[m], 6), rotr(e[m], 11), rotr(e[m], 25));
            const uint32_t ch = __builtin_amdgcn_bitop3_b32(e[m], f[m], g[m], 0xCA);
            const uint32_t t1 = hh[m] + S1 + ch + K256[i] + wi;
            const uint32_t S0 = xor3(rotr(a[m], 2), rotr(a[m], 13), rotr(a[m], 22));
            const uint32_t maj = __builtin_amdgcn_bitop3_b32(a[m], b[m], c[m], 0xE8);
            hh[m] = g[m];
            g[m] = f[m];
            f[m] = e[m];
            e[m] = d[m] + t1;
            d[m] = c[m];
            c[m] = b[m];
            b[m] = a[m];
            a[m] = t1 + S0 + maj;
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        if (live[m]) {
            h[m][0] += a[m]; h[m][1] += b[m]; h[m][2] += c[m]; h[m][3] += d[m];
            h[m][4] += e[m]; h[m][5] += f[m]; h[m][6] += g[m]; h[m][7] += hh[m];
        }
    }
}

// Message words of the block starting at byte address p (any alignment), big-endian.
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t w[16]) {
    typedef const __attribute__((address_space(1))) uint32_t gu32;  // global, not flat, loads
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    gu32* base = (gu32*)(addr & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(addr & 3);
    uint32_t raw[17];
#pragma unroll
    for (int i = 0; i < 17; ++i) raw[i] = base[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t v = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
        w[i] = __builtin_bswap32(v);
    }
}

__device__ __forceinline__ void sha256_one(const uint8_t* msg, uint32_t len, uint32_t h[8]) {
    h[0] = 0x6a09e667;
    h[1] = 0xbb67ae85;
    h[2] = 0x3c6ef372;
    h[3] = 0xa54ff53a;
    h[4] = 0x510e527f;
    h[5] = 0x9b05688c;
    h[6] = 0x1f83d9ab;
    h[7] = 0x5be0cd19;
    const uint32_t full = len >> 6;
    uint32_t w[16];
    for (uint32_t blk = 0; blk < full; ++blk) {
        load_block(msg + 64ull * blk, w);
        compress(h, w);
    }
    // tail: rem bytes of data, 0x80, zeros, 64-bit bit length (one or two blocks)
    const uint32_t rem = len & 63;
    const uint8_t* tail = msg + 64ull * full;
    load_block(tail, w);  // reads within the padded blob
    const uint64_t bits = (uint64_t)len * 8;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t b0 = 4 * i;  // first byte index of this word
        uint32_t v = w[i];
        // keep bytes < rem, byte == rem becomes 0x80, the rest 0
        uint32_t keep_mask;
        if (b0 + 4 <= rem) keep_mask = 0xffffffffu;
        else if (b0 >= rem) keep_mask = 0;
        else keep_mask = 0xffffffffu << (8 * (4 - (rem - b0)));
        v &= keep_mask;
        if (rem >= b0 && rem < b0 + 4) v |= 0x80u << (8 * (3 - (rem - b0)));
        w[i] = v;
    }
    if (rem < 56) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(h, w);
    } else {
        compress(h, w);
#pragma unroll
        for (int i = 0; i < 14; ++i) w[i] = 0;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(h, w);
    }
}

// Block b (0-based) of the FIPS 180-4 padded message (msg, len): data blocks, then the tail
// block(s) with 0x80, zeros and the 64-bit bit length. The tail masking runs under a
// wave-uniform branch, so lanes of one wavefront may sit at different blocks of different
// messages (sha256_stream_kernel) without diverging.
__device__ __forceinline__ uint32_t sha256_nblocks(uint32_t len) { return (len >> 6) + ((len & 63) < 56 ? 1 : 2); }
__device__ __forceinline__ void sha256_block_at(const uint8_t* msg, uint32_t len, uint32_t b, uint32_t w[16]) {
    const uint32_t full = len >> 6;
    const bool tail = b >= full;
    load_block(msg + 64ull * (tail ? full : b), w);  // the blob is padded past its last message
    if (__builtin_expect(__any(tail), 0)) {
        if (tail) {
            const uint32_t rem = len & 63;
            const bool first = b == full;
            const uint32_t krem = first ? rem : 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t b0 = 4 * i;
                uint32_t keep_mask;
                if (b0 + 4 <= krem) keep_mask = 0xffffffffu;
                else if (b0 >= krem) keep_mask = 0;
                else keep_mask = 0xffffffffu << (8 * (4 - (krem - b0)));
                uint32_t v = w[i] & keep_mask;
                if (first && rem >= b0 && rem < b0 + 4) v |= 0x80u << (8 * (3 - (rem - b0)));
                w[i] = v;
            }
            if (b + 1 == sha256_nblocks(len)) {
                const uint64_t bits = (uint64_t)len * 8;
                w[14] = (uint32_t)(bits >> 32);
                w[15] = (uint32_t)bits;
            }
        }
    }
}

}  // namespace sbft
