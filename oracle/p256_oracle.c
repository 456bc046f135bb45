/*
 * p256_oracle.c — plain-C restatement of Go 1.24.1 crypto/ecdsa.Verify (P-256)
 * and crypto/sha256. TEST INFRASTRUCTURE ONLY (see oracle.h for the provenance,
 * the pinning story and who may load this). Parity unpinned by the reference (it
 * holds no vectors for this path and Go is absent); cross-checked against OpenSSL
 * 3.0.2 and Node crypto on every committed fixture.
 *
 * Deliberately simple and independent of the GPU kernels: 4x64-bit limbs,
 * generic CIOS Montgomery multiplication for both p and n, Jacobian points with
 * explicit branches for every exceptional case, bit-by-bit Shamir ladder, an
 * affine conversion by Fermat inversion before the final x comparison. None of
 * the GPU kernel's tricks (special-prime reduction, windows, LDS tables, batched
 * inversion, projective compare) appear here, so an error in one is not
 * mirrored in the other.
 */
#include "oracle.h"

#include <pthread.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } u256; /* little-endian 64-bit limbs */

/* ------------------------------------------------------------------ u256 */
static u256 u256_from_be(const uint8_t b[32]) {
    u256 r;
    for (int i = 0; i < 4; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
        r.v[i] = w;
    }
    return r;
}
static void u256_to_be(const u256* a, uint8_t b[32]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256* a, const u256* b) {
    for (int i = 3; i >= 0; --i) {
        if (a->v[i] < b->v[i]) return -1;
        if (a->v[i] > b->v[i]) return 1;
    }
    return 0;
}
static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (u128)a->v[i] + b->v[i];
        r->v[i] = (uint64_t)c;
        c >>= 64;
    }
    return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->v[i] - b->v[i] - borrow;
        r->v[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 64) & 1;
    }
    return borrow;
}
static int u256_bit(const u256* a, int i) { return (int)((a->v[i >> 6] >> (i & 63)) & 1); }

/* ------------------------------------------------- Montgomery arithmetic */
typedef struct {
    u256 m;      /* modulus */
    uint64_t m0; /* -m^-1 mod 2^64 */
    u256 r2;     /* 2^512 mod m */
    u256 one;    /* 2^256 mod m (Montgomery 1) */
} mont_ctx;

static void mod_add(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
    u256 t, t2;
    uint64_t carry = u256_add(&t, a, b);
    uint64_t borrow = u256_sub(&t2, &t, &c->m);
    *r = (carry || !borrow) ? t2 : t;
}
static void mod_sub(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
    u256 t;
    if (u256_sub(&t, a, b)) u256_add(&t, &t, &c->m);
    *r = t;
}
/* CIOS Montgomery product: a*b*2^-256 mod m, inputs < m. */
static void mont_mul(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        u128 carry = 0;
        for (int j = 0; j < 4; ++j) {
            carry += (u128)a->v[j] * b->v[i] + t[j];
            t[j] = (uint64_t)carry;
            carry >>= 64;
        }
        carry += t[4];
        t[4] = (uint64_t)carry;
        t[5] = (uint64_t)(carry >> 64);
        uint64_t mq = t[0] * c->m0;
        carry = ((u128)mq * c->m.v[0] + t[0]) >> 64;
        for (int j = 1; j < 4; ++j) {
            carry += (u128)mq * c->m.v[j] + t[j];
            t[j - 1] = (uint64_t)carry;
            carry >>= 64;
        }
        carry += t[4];
        t[3] = (uint64_t)carry;
        t[4] = t[5] + (uint64_t)(carry >> 64);
    }
    u256 res = {{t[0], t[1], t[2], t[3]}}, red;
    uint64_t borrow = u256_sub(&red, &res, &c->m);
    *r = (t[4] || !borrow) ? red : res;
}
static void to_mont(const mont_ctx* c, u256* r, const u256* a) { mont_mul(c, r, a, &c->r2); }
static void from_mont(const mont_ctx* c, u256* r, const u256* a) {
    u256 one = {{1, 0, 0, 0}};
    mont_mul(c, r, a, &one);
}
/* a^e (Montgomery domain), plain square-and-multiply over the 256 bits of e. */
static void mont_pow(const mont_ctx* c, u256* r, const u256* a, const u256* e) {
    u256 acc = c->one;
    for (int i = 255; i >= 0; --i) {
        mont_mul(c, &acc, &acc, &acc);
        if (u256_bit(e, i)) mont_mul(c, &acc, &acc, a);
    }
    *r = acc;
}
/* Fermat inverse a^(m-2); a != 0. */
static void mont_inv(const mont_ctx* c, u256* r, const u256* a) {
    u256 e, two = {{2, 0, 0, 0}};
    u256_sub(&e, &c->m, &two);
    mont_pow(c, r, a, &e);
}

static void mont_init(mont_ctx* c, const u256* m) {
    c->m = *m;
    uint64_t inv = 1; /* Newton iteration for m^-1 mod 2^64 */
    for (int i = 0; i < 7; ++i) inv *= 2 - m->v[0] * inv;
    c->m0 = (uint64_t)0 - inv;
    /* one = 2^256 mod m = (2^256 - m) mod m since m > 2^255 for both P-256 moduli */
    u256 zero = {{0, 0, 0, 0}};
    u256_sub(&c->one, &zero, m);
    /* r2 = 2^512 mod m by 256 modular doublings of one */
    u256 x = c->one;
    for (int i = 0; i < 256; ++i) mod_add(c, &x, &x, &x);
    c->r2 = x;
}

/* ------------------------------------------------------- P-256 constants
 * SEC 2 v2 / FIPS 186-5 D.1.2.3 (same constants as Go's nistec p256). */
static const uint8_t P_BE[32] = {0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01, 0x00, 0x00, 0x00,
                                 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0xff, 0xff,
                                 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
static const uint8_t N_BE[32] = {0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x00, 0xff, 0xff, 0xff,
                                 0xff, 0xff, 0xff, 0xff, 0xff, 0xbc, 0xe6, 0xfa, 0xad, 0xa7, 0x17,
                                 0x9e, 0x84, 0xf3, 0xb9, 0xca, 0xc2, 0xfc, 0x63, 0x25, 0x51};
static const uint8_t B_BE[32] = {0x5a, 0xc6, 0x35, 0xd8, 0xaa, 0x3a, 0x93, 0xe7, 0xb3, 0xeb, 0xbd,
                                 0x55, 0x76, 0x98, 0x86, 0xbc, 0x65, 0x1d, 0x06, 0xb0, 0xcc, 0x53,
                                 0xb0, 0xf6, 0x3b, 0xce, 0x3c, 0x3e, 0x27, 0xd2, 0x60, 0x4b};
static const uint8_t GX_BE[32] = {0x6b, 0x17, 0xd1, 0xf2, 0xe1, 0x2c, 0x42, 0x47, 0xf8, 0xbc, 0xe6,
                                  0xe5, 0x63, 0xa4, 0x40, 0xf2, 0x77, 0x03, 0x7d, 0x81, 0x2d, 0xeb,
                                  0x33, 0xa0, 0xf4, 0xa1, 0x39, 0x45, 0xd8, 0x98, 0xc2, 0x96};
static const uint8_t GY_BE[32] = {0x4f, 0xe3, 0x42, 0xe2, 0xfe, 0x1a, 0x7f, 0x9b, 0x8e, 0xe7, 0xeb,
                                  0x4a, 0x7c, 0x0f, 0x9e, 0x16, 0x2b, 0xce, 0x33, 0x57, 0x6b, 0x31,
                                  0x5e, 0xce, 0xcb, 0xb6, 0x40, 0x68, 0x37, 0xbf, 0x51, 0xf5};

static mont_ctx FP, FN;
static u256 B_M, THREE_M; /* b and 3 in Montgomery form mod p */
typedef struct { u256 x, y, z; } jpoint; /* Jacobian, Montgomery coords; z == 0 <=> infinity */
static jpoint G_J;
static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void init_consts(void) {
    u256 p = u256_from_be(P_BE), n = u256_from_be(N_BE);
    mont_init(&FP, &p);
    mont_init(&FN, &n);
    u256 b = u256_from_be(B_BE), three = {{3, 0, 0, 0}};
    to_mont(&FP, &B_M, &b);
    to_mont(&FP, &THREE_M, &three);
    u256 gx = u256_from_be(GX_BE), gy = u256_from_be(GY_BE);
    to_mont(&FP, &G_J.x, &gx);
    to_mont(&FP, &G_J.y, &gy);
    G_J.z = FP.one;
}
static void ensure_init(void) { pthread_once(&init_once, init_consts); }

/* ------------------------------------------------------ point arithmetic */
static int jp_is_inf(const jpoint* a) { return u256_is_zero(&a->z); }

/* Doubling, textbook Jacobian (y^2 = x^3 + a x + b, a = -3):
 * S = 4XY^2, M = 3X^2 + aZ^4, X' = M^2 - 2S, Y' = M(S - X') - 8Y^4, Z' = 2YZ. */
static void jp_double(jpoint* r, const jpoint* a) {
    if (jp_is_inf(a) || u256_is_zero(&a->y)) {
        memset(r, 0, sizeof *r);
        return;
    }
    u256 xx, yy, yyyy, zz, zzzz, s, m, t, x3, y3, z3;
    mont_mul(&FP, &xx, &a->x, &a->x);
    mont_mul(&FP, &yy, &a->y, &a->y);
    mont_mul(&FP, &yyyy, &yy, &yy);
    mont_mul(&FP, &zz, &a->z, &a->z);
    mont_mul(&FP, &zzzz, &zz, &zz);
    mont_mul(&FP, &s, &a->x, &yy);
    mod_add(&FP, &s, &s, &s);
    mod_add(&FP, &s, &s, &s);             /* S = 4 X Y^2 */
    mont_mul(&FP, &m, &THREE_M, &xx);     /* 3X^2 */
    mont_mul(&FP, &t, &THREE_M, &zzzz);   /* 3Z^4 */
    mod_sub(&FP, &m, &m, &t);             /* M = 3X^2 - 3Z^4 */
    mont_mul(&FP, &x3, &m, &m);
    mod_sub(&FP, &x3, &x3, &s);
    mod_sub(&FP, &x3, &x3, &s);           /* X' = M^2 - 2S */
    mod_sub(&FP, &t, &s, &x3);
    mont_mul(&FP, &y3, &m, &t);
    u256 y8 = yyyy;
    mod_add(&FP, &y8, &y8, &y8);
    mod_add(&FP, &y8, &y8, &y8);
    mod_add(&FP, &y8, &y8, &y8);          /* 8Y^4 */
    mod_sub(&FP, &y3, &y3, &y8);
    mont_mul(&FP, &z3, &a->y, &a->z);
    mod_add(&FP, &z3, &z3, &z3);          /* Z' = 2YZ */
    r->x = x3;
    r->y = y3;
    r->z = z3;
}

/* General addition with every exceptional case branched explicitly. */
static void jp_add(jpoint* r, const jpoint* a, const jpoint* b) {
    if (jp_is_inf(a)) { *r = *b; return; }
    if (jp_is_inf(b)) { *r = *a; return; }
    u256 z1z1, z2z2, u1, u2, s1, s2, t;
    mont_mul(&FP, &z1z1, &a->z, &a->z);
    mont_mul(&FP, &z2z2, &b->z, &b->z);
    mont_mul(&FP, &u1, &a->x, &z2z2);
    mont_mul(&FP, &u2, &b->x, &z1z1);
    mont_mul(&FP, &t, &b->z, &z2z2);
    mont_mul(&FP, &s1, &a->y, &t);
    mont_mul(&FP, &t, &a->z, &z1z1);
    mont_mul(&FP, &s2, &b->y, &t);
    if (u256_cmp(&u1, &u2) == 0) {
        if (u256_cmp(&s1, &s2) == 0) { jp_double(r, a); return; }
        memset(r, 0, sizeof *r); /* P + (-P) */
        return;
    }
    u256 h, rr, hh, hhh, v, x3, y3, z3;
    mod_sub(&FP, &h, &u2, &u1);
    mod_sub(&FP, &rr, &s2, &s1);
    mont_mul(&FP, &hh, &h, &h);
    mont_mul(&FP, &hhh, &hh, &h);
    mont_mul(&FP, &v, &u1, &hh);
    mont_mul(&FP, &x3, &rr, &rr);
    mod_sub(&FP, &x3, &x3, &hhh);
    mod_sub(&FP, &x3, &x3, &v);
    mod_sub(&FP, &x3, &x3, &v);           /* X3 = R^2 - H^3 - 2 U1 H^2 */
    mod_sub(&FP, &t, &v, &x3);
    mont_mul(&FP, &y3, &rr, &t);
    mont_mul(&FP, &t, &s1, &hhh);
    mod_sub(&FP, &y3, &y3, &t);           /* Y3 = R (U1 H^2 - X3) - S1 H^3 */
    mont_mul(&FP, &z3, &a->z, &b->z);
    mont_mul(&FP, &z3, &z3, &h);          /* Z3 = Z1 Z2 H */
    r->x = x3;
    r->y = y3;
    r->z = z3;
}

/* a*G + b*Q by a joint left-to-right binary ladder over {G, Q, G+Q}. */
static void jp_double_mul(jpoint* r, const u256* a, const jpoint* q, const u256* b) {
    jpoint gq, acc;
    jp_add(&gq, &G_J, q);
    memset(&acc, 0, sizeof acc);
    for (int i = 255; i >= 0; --i) {
        jp_double(&acc, &acc);
        int ba = u256_bit(a, i), bb = u256_bit(b, i);
        if (ba && bb) jp_add(&acc, &acc, &gq);
        else if (ba) jp_add(&acc, &acc, &G_J);
        else if (bb) jp_add(&acc, &acc, q);
    }
    *r = acc;
}

/* Affine (plain, non-Montgomery) coordinates of a finite point. */
static void jp_to_affine(const jpoint* a, u256* x, u256* y) {
    u256 zi, zi2, zi3, t;
    mont_inv(&FP, &zi, &a->z);
    mont_mul(&FP, &zi2, &zi, &zi);
    mont_mul(&FP, &zi3, &zi2, &zi);
    mont_mul(&FP, &t, &a->x, &zi2);
    from_mont(&FP, x, &t);
    if (y) {
        mont_mul(&FP, &t, &a->y, &zi3);
        from_mont(&FP, y, &t);
    }
}

/* nistec P256Point.SetBytes for the uncompressed encoding: canonical coordinates
 * (x, y < p) and on the curve y^2 = x^3 - 3x + b. */
static int load_pubkey(const uint8_t qx[32], const uint8_t qy[32], jpoint* out) {
    u256 x = u256_from_be(qx), y = u256_from_be(qy);
    if (u256_cmp(&x, &FP.m) >= 0 || u256_cmp(&y, &FP.m) >= 0) return 0;
    u256 xm, ym, lhs, rhs, t;
    to_mont(&FP, &xm, &x);
    to_mont(&FP, &ym, &y);
    mont_mul(&FP, &lhs, &ym, &ym);
    mont_mul(&FP, &rhs, &xm, &xm);
    mont_mul(&FP, &rhs, &rhs, &xm);
    mont_mul(&FP, &t, &THREE_M, &xm);
    mod_sub(&FP, &rhs, &rhs, &t);
    mod_add(&FP, &rhs, &rhs, &B_M);
    if (u256_cmp(&lhs, &rhs) != 0) return 0;
    out->x = xm;
    out->y = ym;
    out->z = FP.one;
    return 1;
}

/* ------------------------------------------------------------- ECDSA API */
void oracle_normalize_hash(const uint8_t* hash, size_t len, uint8_t out32[32]) {
    /* hashToNat for a 256-bit order: keep the first N.Size()=32 bytes; the
     * excess-bit shift is zero for P-256; a shorter hash is a smaller integer. */
    memset(out32, 0, 32);
    if (len >= 32) memcpy(out32, hash, 32);
    else if (len) memcpy(out32 + (32 - len), hash, len);
}

int oracle_verify_p256(const uint8_t digest[32], const uint8_t rb[32], const uint8_t sb[32],
                       const uint8_t qx[32], const uint8_t qy[32]) {
    ensure_init();
    jpoint q;
    if (!load_pubkey(qx, qy, &q)) return 0; /* ecdsa.NewPublicKey / SetBytes error */
    u256 r = u256_from_be(rb), s = u256_from_be(sb);
    /* bigmod.SetBytes(sig.R, c.N) errors for r >= n; IsZero rejects 0. Same for s. */
    if (u256_is_zero(&r) || u256_cmp(&r, &FN.m) >= 0) return 0;
    if (u256_is_zero(&s) || u256_cmp(&s, &FN.m) >= 0) return 0;
    /* e = SetOverflowingBytes(hash[:32]) -> reduced mod n (one conditional subtraction
     * suffices: 2^256 < 2n). */
    u256 e = u256_from_be(digest), t;
    if (!u256_sub(&t, &e, &FN.m)) e = t;
    u256 sm, w, em, rm, u1m, u2m, u1, u2;
    to_mont(&FN, &sm, &s);
    mont_inv(&FN, &w, &sm);
    to_mont(&FN, &em, &e);
    to_mont(&FN, &rm, &r);
    mont_mul(&FN, &u1m, &em, &w);
    mont_mul(&FN, &u2m, &rm, &w);
    from_mont(&FN, &u1, &u1m);
    from_mont(&FN, &u2, &u2m);
    jpoint R;
    jp_double_mul(&R, &u1, &q, &u2);
    if (jp_is_inf(&R)) return 0; /* BytesX errors on the point at infinity */
    u256 x;
    jp_to_affine(&R, &x, NULL);
    /* v = SetOverflowingBytes(Rx, N): x < p < 2n, so one conditional subtraction. */
    if (!u256_sub(&t, &x, &FN.m)) x = t;
    return u256_cmp(&x, &r) == 0;
}

/* ------------------------------------------------------------- SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void oracle_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                     0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t full = len / 64;
    for (size_t i = 0; i < full; ++i) sha256_block(h, msg + 64 * i);
    uint8_t tail[128];
    size_t rem = len - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, msg + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tlen = (rem < 56) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; ++i) tail[tlen - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_block(h, tail);
    if (tlen == 128) sha256_block(h, tail + 64);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

/* ------------------------------------------------------------ batches */
typedef struct {
    int kind; /* 0 verify, 1 sha */
    const uint8_t *digest, *r, *s, *qx, *qy, *blob;
    const uint64_t* off;
    const uint32_t* len;
    uint8_t* out;
    size_t begin, end;
} job_t;

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    for (size_t i = j->begin; i < j->end; ++i) {
        if (j->kind == 0)
            j->out[i] = (uint8_t)oracle_verify_p256(j->digest + 32 * i, j->r + 32 * i, j->s + 32 * i,
                                                    j->qx + 32 * i, j->qy + 32 * i);
        else
            oracle_sha256(j->blob + j->off[i], j->len[i], j->out + 32 * i);
    }
    return NULL;
}

static void run_parallel(job_t proto, size_t n, int nthreads) {
    ensure_init();
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    job_t jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = proto;
        jobs[t].begin = n * t / nthreads;
        jobs[t].end = n * (t + 1) / nthreads;
        if (nthreads == 1) run_job(&jobs[t]);
        else pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void oracle_verify_p256_batch(const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                              const uint8_t* qx, const uint8_t* qy, size_t n, uint8_t* ok_out,
                              int nthreads) {
    job_t p = {0};
    p.kind = 0; p.digest = digest; p.r = r; p.s = s; p.qx = qx; p.qy = qy; p.out = ok_out;
    run_parallel(p, n, nthreads);
}

void oracle_sha256_batch(const uint8_t* blob, const uint64_t* off, const uint32_t* len, size_t n,
                         uint8_t* dig_out, int nthreads) {
    job_t p = {0};
    p.kind = 1; p.blob = blob; p.off = off; p.len = len; p.out = dig_out;
    run_parallel(p, n, nthreads);
}

/* ------------------------------------------- fixture-construction helpers */
int oracle_pubkey(const uint8_t db[32], uint8_t qx[32], uint8_t qy[32]) {
    ensure_init();
    u256 d = u256_from_be(db), zero = {{0, 0, 0, 0}};
    if (u256_is_zero(&d) || u256_cmp(&d, &FN.m) >= 0) return 0;
    jpoint R, inf;
    memset(&inf, 0, sizeof inf);
    jp_double_mul(&R, &d, &inf, &zero);
    if (jp_is_inf(&R)) return 0;
    u256 x, y;
    jp_to_affine(&R, &x, &y);
    u256_to_be(&x, qx);
    u256_to_be(&y, qy);
    return 1;
}

int oracle_sign(const uint8_t db[32], const uint8_t kb[32], const uint8_t digest[32], uint8_t rb[32],
                uint8_t sb[32]) {
    ensure_init();
    u256 d = u256_from_be(db), k = u256_from_be(kb), zero = {{0, 0, 0, 0}}, t;
    if (u256_is_zero(&d) || u256_cmp(&d, &FN.m) >= 0) return 0;
    if (u256_is_zero(&k) || u256_cmp(&k, &FN.m) >= 0) return 0;
    jpoint R, inf;
    memset(&inf, 0, sizeof inf);
    jp_double_mul(&R, &k, &inf, &zero);
    u256 x;
    jp_to_affine(&R, &x, NULL);
    if (!u256_sub(&t, &x, &FN.m)) x = t;
    if (u256_is_zero(&x)) return 0;
    u256 e = u256_from_be(digest);
    if (!u256_sub(&t, &e, &FN.m)) e = t;
    u256 km, kinv, dm, rm, em, acc, s;
    to_mont(&FN, &km, &k);
    mont_inv(&FN, &kinv, &km);
    to_mont(&FN, &dm, &d);
    to_mont(&FN, &rm, &x);
    to_mont(&FN, &em, &e);
    mont_mul(&FN, &acc, &rm, &dm);
    mod_add(&FN, &acc, &acc, &em);
    mont_mul(&FN, &acc, &acc, &kinv);
    from_mont(&FN, &s, &acc);
    if (u256_is_zero(&s)) return 0;
    u256_to_be(&x, rb);
    u256_to_be(&s, sb);
    return 1;
}

int oracle_double_mul(const uint8_t ab[32], const uint8_t bb[32], const uint8_t qx[32],
                      const uint8_t qy[32], uint8_t ox[32], uint8_t oy[32]) {
    ensure_init();
    jpoint q, R;
    if (!load_pubkey(qx, qy, &q)) return 0;
    u256 a = u256_from_be(ab), b = u256_from_be(bb);
    jp_double_mul(&R, &a, &q, &b);
    if (jp_is_inf(&R)) return 0;
    u256 x, y;
    jp_to_affine(&R, &x, &y);
    u256_to_be(&x, ox);
    u256_to_be(&y, oy);
    return 1;
}

int oracle_lift_x(const uint8_t xb[32], int odd, uint8_t yb[32]) {
    ensure_init();
    u256 x = u256_from_be(xb);
    if (u256_cmp(&x, &FP.m) >= 0) return 0;
    u256 xm, rhs, t, y, chk, e, one = {{1, 0, 0, 0}};
    to_mont(&FP, &xm, &x);
    mont_mul(&FP, &rhs, &xm, &xm);
    mont_mul(&FP, &rhs, &rhs, &xm);
    mont_mul(&FP, &t, &THREE_M, &xm);
    mod_sub(&FP, &rhs, &rhs, &t);
    mod_add(&FP, &rhs, &rhs, &B_M);
    /* p = 3 mod 4: sqrt = rhs^((p+1)/4) */
    u256_add(&e, &FP.m, &one);
    for (int i = 0; i < 2; ++i) { /* e >>= 1, twice (p+1 does not overflow 2^256) */
        for (int l = 0; l < 4; ++l) e.v[l] = (e.v[l] >> 1) | (l < 3 ? e.v[l + 1] << 63 : 0);
    }
    mont_pow(&FP, &y, &rhs, &e);
    mont_mul(&FP, &chk, &y, &y);
    if (u256_cmp(&chk, &rhs) != 0) return 0;
    u256 yp;
    from_mont(&FP, &yp, &y);
    if ((int)(yp.v[0] & 1) != (odd ? 1 : 0) && !u256_is_zero(&yp)) u256_sub(&yp, &FP.m, &yp);
    u256_to_be(&yp, yb);
    return 1;
}

static void mod_op(const mont_ctx* c, int op, const uint8_t ab[32], const uint8_t bb[32],
                   uint8_t out[32]) {
    ensure_init();
    u256 a = u256_from_be(ab), b = bb ? u256_from_be(bb) : (u256){{0, 0, 0, 0}}, t, r;
    if (!u256_sub(&t, &a, &c->m)) a = t;
    if (!u256_sub(&t, &b, &c->m)) b = t;
    u256 am, bm, rm;
    switch (op) {
    case 0: mod_add(c, &r, &a, &b); break;
    case 1: mod_sub(c, &r, &a, &b); break;
    case 2:
        to_mont(c, &am, &a);
        to_mont(c, &bm, &b);
        mont_mul(c, &rm, &am, &bm);
        from_mont(c, &r, &rm);
        break;
    case 3:
        to_mont(c, &am, &a);
        mont_inv(c, &rm, &am);
        from_mont(c, &r, &rm);
        break;
    default: {
        u256 zero = {{0, 0, 0, 0}};
        mod_sub(c, &r, &zero, &a);
    }
    }
    u256_to_be(&r, out);
}
void oracle_modn(int op, const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    ensure_init();
    mod_op(&FN, op, a, b, out);
}
void oracle_modp(int op, const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
    ensure_init();
    mod_op(&FP, op, a, b, out);
}
