// p256_keyed.hip — P-256 verification against REGISTERED public keys (consenter keys), gfx950.
//
// SmartBFT's consenter signatures (VerifyConsenterSig at internal/bft/view.go:631 and :834,
// viewchanger.go:718; VerifySignature at viewchanger.go:598) are always checked against one of
// the n consenter keys of the configuration. Those keys are known before any signature
// arrives, so the engine precomputes a fixed-base comb table per key when it is registered
// (the plugin's key registry, include/sbft_verifier.h sbft_verifier_add_consenter), exactly
// as every P-256 implementation does for the generator G:
//
//   table[w][j] = j * 2^(8w) * Q   (w = 0..31, j = 1..255), affine, Montgomery form mod p
//
// 32 windows x 256 entries x 64 B = 512 KiB per key in HBM (100 consenters = 51 MiB; the
// generator's table is key slot 0). Then u1*G + u2*Q = sum_w table_G[w][byte_w(u1)] +
// sum_w table_Q[w][byte_w(u2)]: 64 table points and NO doublings.
//
// p256_verify_keyed_wave_kernel (latency path, one workgroup of two wavefronts per signature):
//   wave 1: w = s^-1 R mod n (lane-parallel scaled safegcd, p256_inv.hpp inv_mod_wave)
//   wave 0: [SHA-256 of the message] ; then u = e w (lanes < 32) or r w (lanes >= 32)
//   lane l: loads ONE table point (l < 32: G window l of u1; l >= 32: Q window l-32 of u2)
//   6-level butterfly over the wave in radix 2^29 with lean additions (quad-cooperative
//   products, DPP broadcasts); Z = 0 at the end marks an exceptional addition, and only then
//   the wave re-runs the butterfly with the exact 8 x 32 additions (infinity, doubling,
//   cancellation); accept iff R != infinity and x(R) = r (mod n), projectively (r and r + n).
// The dependent chain is ~6 point additions + one inversion instead of 256 doublings: a
// 67-signature commit quorum is one ~42 us kernel (the phase timeline).
// Large batches take p256_verify.hip's four-lane kernel over the same tables.
//
// Verdicts are bit-exact with Go crypto/ecdsa.Verify (same semantics as p256_verify.hip;
// oracle/p256_oracle.c is the parity reference). An unregistered/invalid key id verifies false.
#include "p256_f29.hpp"
#include "p256_inv.hpp"
#include "p256_point.hpp"
#include "sbft_kernels.h"
#include "sha256_dev.hpp"

namespace sbft {

// Phase marks for tools/keyed_phases.hip (which defines the macro before including this file)
#ifndef SBFT_KEYED_MARK
#define SBFT_KEYED_MARK(i) ((void)0)
#endif

// comb table layout (COMB_*): p256_point.hpp

SBFT_DEV void to_affine_mont(fe& x, fe& y, const jp& p) {
    fe zi, zi2, zi3;
    fp_inv(zi, p.z);
    fp_sqr(zi2, zi);
    fp_mul(zi3, zi2, zi);
    fp_mul(x, p.x, zi2);
    fp_mul(y, p.y, zi3);
    fp_canon(x, x);
    fp_canon(y, y);
}

// One lane per table entry (key, w, j): j * 2^(8w) * Q_key, for nk keys whose tables lie
// contiguously from `tables` (COMB_KEY_U4 uint4 each). status[key] = 1 iff Q_key is a valid key
// (canonical coordinates on the curve); the table is written either way (zeros if invalid).
__global__ __launch_bounds__(256) void p256_comb_build_kernel(const uint8_t* __restrict__ qxs,
                                                              const uint8_t* __restrict__ qys,
                                                              uint4* __restrict__ tables,
                                                              uint32_t* __restrict__ status, uint32_t nk) {
    const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t key = (uint32_t)(gt / (COMB_WINDOWS * COMB_ENTRIES));
    if (key >= nk) return;
    const uint32_t t = (uint32_t)(gt % (COMB_WINDOWS * COMB_ENTRIES));
    const uint32_t w = t / COMB_ENTRIES, j = t % COMB_ENTRIES;
    const fe qx = load_be32(qxs + 32ull * key), qy = load_be32(qys + 32ull * key);
    bool valid = fe_lt(qx, P256_P) && fe_lt(qy, P256_P);
    const fe r2p = fe_const(C_R2P);
    jp base;
    fp_mul(base.x, qx, r2p);
    fp_mul(base.y, qy, r2p);
    base.z = fe_const(C_ONEP);
    {
        fe lhs, rhs, tt;
        fp_sqr(lhs, base.y);
        fp_sqr(rhs, base.x);
        fp_mul(rhs, rhs, base.x);
        fp_add(tt, base.x, base.x);
        fp_add(tt, tt, base.x);
        fp_sub(rhs, rhs, tt);
        fp_add(rhs, rhs, fe_const(C_BM));
        fp_canon(lhs, lhs);
        fp_canon(rhs, rhs);
        valid = valid && fe_eq(lhs, rhs);
    }
    if (t == 0) status[key] = valid ? 1u : 0u;
    uint4* out = tables + (size_t)key * COMB_KEY_U4 + (size_t)t * COMB_ENTRY_U4;
    if (!valid || j == 0) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        out[0] = z;
        out[1] = z;
        out[2] = z;
        out[3] = z;
        return;
    }
#pragma unroll 1
    for (uint32_t i = 0; i < 8 * w; ++i) pt_dbl(base, base);  // 2^(8w) Q (never infinity: n is prime)
    jp acc;
    bool inf = true;
    acc = base;
#pragma unroll 1
    for (int b = 7; b >= 0; --b) {
        if (!inf) pt_dbl(acc, acc);
        pt_add_jac(acc, inf, base, ((j >> b) & 1u) != 0);
    }
    fe x, y;
    to_affine_mont(x, y, acc);  // j < n, so j 2^(8w) Q is never infinity
    out[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    out[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
    out[2] = make_uint4(y.v[0], y.v[1], y.v[2], y.v[3]);
    out[3] = make_uint4(y.v[4], y.v[5], y.v[6], y.v[7]);
}

SBFT_DEV u32 shfl_xor_u32(u32 v, int mask) { return (u32)__shfl_xor((int)v, mask, 64); }
SBFT_DEV void shfl_xor_fe(fe& o, const fe& a, int mask) {
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = shfl_xor_u32(a.v[k], mask);
}



// ---- cooperative point additions (latency path) ----
// In the butterfly, every lane of an aligned group holds the same pair of points, so the
// group splits ONE addition's independent field multiplications over its lanes (lane & 3 in
// quads, lane & 1 in pairs) and re-broadcasts the products with DPP quad permutes: the
// dependent chain of a Jacobian addition drops from 16 multiplications to 5.
template <int CTRL>
SBFT_DEV fe dpp_fe(const fe& a) {
    fe o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)a.v[k], CTRL, 0xf, 0xf, false);
    return o;
}
#define QB(J) ((J) * 0x55)               // quad_perm [J,J,J,J]
#define PB0 0xA0                         // quad_perm [0,0,2,2]
#define PB1 0xF5                         // quad_perm [1,1,3,3]
// Two levels of two-way selects on the bits of j (v_cndmask): written as a j == 0/1/2 chain,
// the selects over whole structs were lowered to a scratch array indexed by j.
SBFT_DEV u32 pick4(bool b0, bool b1, u32 a0, u32 a1, u32 a2, u32 a3) {
    const u32 lo = b0 ? a1 : a0, hi = b0 ? a3 : a2;
    return b1 ? hi : lo;
}
SBFT_DEV fe sel4(u32 j, const fe& a0, const fe& a1, const fe& a2, const fe& a3) {
    const bool b0 = (j & 1u) != 0, b1 = (j & 2u) != 0;
    fe o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = pick4(b0, b1, a0.v[k], a1.v[k], a2.v[k], a3.v[k]);
    return o;
}
SBFT_DEV fe sel2(u32 j, const fe& a0, const fe& a1) {
    fe o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.v[k] = j == 0 ? a0.v[k] : a1.v[k];
    return o;
}

// Resolve the special cases of P1 + P2 given the generic result (x3, y3, z3) computed from
// H = U2 - U1 and R = S2 - S1: infinity operands, P1 = P2 (doubling), P1 = -P2 (infinity).
SBFT_DEV void finish_add(jp& acc, bool& inf, const jp& p1, bool i1, const jp& p2, bool i2, const fe& H,
                         const fe& R, const fe& x3, const fe& y3, const fe& z3) {
    const bool hz = fp_is_zero(H), rz = fp_is_zero(R);
    const bool both = !i1 && !i2;
    jp out;
    out.x = x3;
    out.y = y3;
    out.z = z3;
    bool oinf = hz && !rz;
    const bool need_dbl = both && hz && rz;
    if (__builtin_expect(__any(need_dbl), 0)) {
        jp d;
        pt_dbl(d, p1);
        jp_sel(out, need_dbl, d);
        if (need_dbl) oinf = false;
    }
    jp_sel(out, i1, p2);
    jp_sel(out, i2 && !i1, p1);
    acc = out;
    inf = both ? oinf : (i1 && i2);
}

// Level 0: P1, P2 affine (Z = 1), lane pairs (2m, 2m+1); P1 is the even lane's point.
SBFT_DEV void coop_add_affine_pair(jp& acc, bool& inf, u32 lane) {
    jp o;
    o.x = dpp_fe<0xB1>(acc.x);  // quad_perm [1,0,3,2]: the partner lane
    o.y = dpp_fe<0xB1>(acc.y);
    const bool oinf = __builtin_amdgcn_mov_dpp(inf ? 1 : 0, 0xB1, 0xf, 0xf, false) != 0;
    const u32 j = lane & 1u;
    jp p1, p2;
    p1.x = sel2(j, acc.x, o.x);
    p1.y = sel2(j, acc.y, o.y);
    p2.x = sel2(j, o.x, acc.x);
    p2.y = sel2(j, o.y, acc.y);
    p1.z = p2.z = fe_const(C_ONEP);
    const bool i1 = j ? oinf : inf, i2 = j ? inf : oinf;
    fe H, R, t;
    fp_sub(H, p2.x, p1.x);
    fp_sub(R, p2.y, p1.y);
    // S1: HH = H^2 (j0), RR = R^2 (j1)
    {
        const fe a = sel2(j, H, R);
        fp_mul(t, a, a);
    }
    const fe HH = dpp_fe<PB0>(t), RR = dpp_fe<PB1>(t);
    // S2: HHH = H HH (j0), V = X1 HH (j1)
    fp_mul(t, sel2(j, H, p1.x), HH);
    const fe HHH = dpp_fe<PB0>(t), V = dpp_fe<PB1>(t);
    fe X3, VX;
    fp_sub(X3, RR, HHH);
    fp_sub(X3, X3, V);
    fp_sub(X3, X3, V);
    fp_sub(VX, V, X3);
    // S3: Y1 HHH (j0), R (V - X3) (j1)
    fp_mul(t, sel2(j, p1.y, R), sel2(j, HHH, VX));
    fe Y3;
    fp_sub(Y3, dpp_fe<PB1>(t), dpp_fe<PB0>(t));
    finish_add(acc, inf, p1, i1, p2, i2, H, R, X3, Y3, H);
}

// Level lvl >= 1: Jacobian P1 (lower half-group) + P2 (upper), computed by each quad.
SBFT_DEV void coop_add_jac_quad(jp& acc, bool& inf, u32 lane, int lvl) {
    const int m = 1 << lvl;
    jp o;
    shfl_xor_fe(o.x, acc.x, m);
    shfl_xor_fe(o.y, acc.y, m);
    shfl_xor_fe(o.z, acc.z, m);
    const bool oinf = shfl_xor_u32(inf ? 1u : 0u, m) != 0;
    const bool hi = ((lane >> lvl) & 1u) != 0;
    jp p1, p2;
    p1.x = sel2(hi, acc.x, o.x);
    p1.y = sel2(hi, acc.y, o.y);
    p1.z = sel2(hi, acc.z, o.z);
    p2.x = sel2(hi, o.x, acc.x);
    p2.y = sel2(hi, o.y, acc.y);
    p2.z = sel2(hi, o.z, acc.z);
    const bool i1 = hi ? oinf : inf, i2 = hi ? inf : oinf;
    const u32 j = lane & 3u;
    fe t;
    // S1: A = Z1^2 (j0), B = Z2^2 (j1), C = Z1 Z2 (j2)
    fp_mul(t, sel4(j, p1.z, p2.z, p1.z, p1.z), sel4(j, p1.z, p2.z, p2.z, p1.z));
    const fe A = dpp_fe<QB(0)>(t), B = dpp_fe<QB(1)>(t), C = dpp_fe<QB(2)>(t);
    // S2: U1 = X1 B (j0), U2 = X2 A (j1), T1 = Z1 A (j2), T2 = Z2 B (j3)
    fp_mul(t, sel4(j, p1.x, p2.x, p1.z, p2.z), sel4(j, B, A, A, B));
    const fe U1 = dpp_fe<QB(0)>(t), U2 = dpp_fe<QB(1)>(t), T1 = dpp_fe<QB(2)>(t), T2 = dpp_fe<QB(3)>(t);
    fe H;
    fp_sub(H, U2, U1);
    // S3: S1 = Y1 T2 (j0), S2 = Y2 T1 (j1), Z3 = C H (j2), HH = H^2 (j3)
    fp_mul(t, sel4(j, p1.y, p2.y, C, H), sel4(j, T2, T1, H, H));
    const fe S1 = dpp_fe<QB(0)>(t), S2 = dpp_fe<QB(1)>(t), Z3 = dpp_fe<QB(2)>(t), HH = dpp_fe<QB(3)>(t);
    fe R;
    fp_sub(R, S2, S1);
    // S4: RR = R^2 (j0), HHH = H HH (j1), V = U1 HH (j2)
    fp_mul(t, sel4(j, R, H, U1, R), sel4(j, R, HH, HH, R));
    const fe RR = dpp_fe<QB(0)>(t), HHH = dpp_fe<QB(1)>(t), V = dpp_fe<QB(2)>(t);
    fe X3, VX;
    fp_sub(X3, RR, HHH);
    fp_sub(X3, X3, V);
    fp_sub(X3, X3, V);
    fp_sub(VX, V, X3);
    // S5: S1 HHH (j0), R (V - X3) (j1)
    fp_mul(t, sel2(j & 1u, S1, R), sel2(j & 1u, HHH, VX));
    fe Y3;
    fp_sub(Y3, dpp_fe<QB(1)>(t), dpp_fe<QB(0)>(t));
    finish_add(acc, inf, p1, i1, p2, i2, H, R, X3, Y3, Z3);
}


// ---- the same butterfly in radix-2^29 arithmetic (p256_f29.hpp), lean additions ----
// A field product here is f29_mul_ilp: its 17 column sums are independent chains, so one
// wavefront issues them back to back, where the 8 x 32 product above is one long carry chain
// (~2,800 cycles per cooperative step against ~1,000). The additions have no case analysis
// beyond infinity operands (digit-0 entries, selected around): P1 = +-P2 gives H = 0, hence
// Z3 = 0, which every later level keeps; the kernel then re-runs the tuple on the exact
// butterfly above. Limb bounds as in p29_add_jac_lean_i (p256_f29.hpp).
#ifndef SBFT_KEYED_F29
#define SBFT_KEYED_F29 1
#endif

template <int CTRL>
SBFT_DEV f29 dpp29(const f29& a) {
    f29 o;
#pragma unroll
    for (int k = 0; k < 9; ++k) o.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)a.v[k], CTRL, 0xf, 0xf, false);
    return o;
}
SBFT_DEV f29 sel2_29(bool j, const f29& a0, const f29& a1) {
    f29 o;
#pragma unroll
    for (int k = 0; k < 9; ++k) o.v[k] = j ? a1.v[k] : a0.v[k];
    return o;
}
SBFT_DEV f29 sel4_29(u32 j, const f29& a0, const f29& a1, const f29& a2, const f29& a3) {
    const bool b0 = (j & 1u) != 0, b1 = (j & 2u) != 0;
    f29 o;
#pragma unroll
    for (int k = 0; k < 9; ++k) o.v[k] = pick4(b0, b1, a0.v[k], a1.v[k], a2.v[k], a3.v[k]);
    return o;
}
SBFT_DEV f29 shfl_xor29(const f29& a, int mask) {
    f29 o;
#pragma unroll
    for (int k = 0; k < 9; ++k) o.v[k] = shfl_xor_u32(a.v[k], mask);
    return o;
}
SBFT_DEV void jp29_sel(jp29& out, bool c, const jp29& a) {
    out.x = sel2_29(c, out.x, a.x);
    out.y = sel2_29(c, out.y, a.y);
    out.z = sel2_29(c, out.z, a.z);
}

// table entry (8 x 32 Montgomery, R = 2^256, canonical) -> affine f29 Montgomery (R = 2^261)
SBFT_DEV void entry_to_f29(const fe& x, const fe& y, jp29& p) {
    p.x = f29_from_mont256(x);
    p.y = f29_from_mont256(y);
    p.z = f29_const(C29_ONE);
}

// Level 0: affine P1 (even lane) + affine P2 (odd lane) on lane pairs, three product steps.
SBFT_DEV void coop29_add_affine_pair(jp29& acc, bool& inf, u32 lane) {
    const f29 ox = dpp29<0xB1>(acc.x), oy = dpp29<0xB1>(acc.y);  // quad_perm [1,0,3,2]
    const bool oinf = __builtin_amdgcn_mov_dpp(inf ? 1 : 0, 0xB1, 0xf, 0xf, false) != 0;
    const bool j = (lane & 1u) != 0;
    jp29 p1, p2;
    p1.x = sel2_29(j, acc.x, ox);
    p1.y = sel2_29(j, acc.y, oy);
    p2.x = sel2_29(j, ox, acc.x);
    p2.y = sel2_29(j, oy, acc.y);
    p1.z = p2.z = acc.z;  // ONE on every lane
    const bool i1 = j ? oinf : inf, i2 = j ? inf : oinf;
    f29 H, R, t, X3, VX, Y3;
    f29_sub(H, p2.x, p1.x);  // |limb| < 2^29
    f29_sub(R, p2.y, p1.y);
    {
        const f29 a = sel2_29(j, H, R);
        f29_mul_ilp(t, a, a);  // HH | RR
    }
    const f29 HH = dpp29<PB0>(t), RR = dpp29<PB1>(t);
    f29_mul_ilp(t, sel2_29(j, H, p1.x), HH);  // HHH | V = X1 HH
    const f29 HHH = dpp29<PB0>(t), V = dpp29<PB1>(t);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = RR.v[i] - HHH.v[i] - (V.v[i] << 1);  // (-3 2^29, 2^29)
    f29_normalize(X3, t);
    f29_sub(VX, V, X3);                                             // (-2^29.2, 2^29 + 2^26)
    f29_mul_ilp(t, sel2_29(j, p1.y, R), sel2_29(j, HHH, VX));       // Y1 HHH | R (V - X3)
    f29_sub(Y3, dpp29<PB1>(t), dpp29<PB0>(t));                      // N+-
    jp29 out;
    out.x = X3;
    out.y = Y3;
    out.z = H;
    jp29_sel(out, i2, p1);
    jp29_sel(out, i1, p2);
    acc = out;
    inf = i1 && i2;
}

// Levels >= 1: Jacobian P1 (lower half-group) + P2 (upper) on each quad, five product steps.
SBFT_DEV void coop29_add_jac_quad(jp29& acc, bool& inf, u32 lane, int lvl) {
    const int m = 1 << lvl;
    jp29 o;
    o.x = shfl_xor29(acc.x, m);
    o.y = shfl_xor29(acc.y, m);
    o.z = shfl_xor29(acc.z, m);
    const bool oinf = shfl_xor_u32(inf ? 1u : 0u, m) != 0;
    const bool hi = ((lane >> lvl) & 1u) != 0;
    jp29 p1 = acc, p2 = o;
    jp29_sel(p1, hi, o);
    jp29_sel(p2, hi, acc);
    const bool i1 = hi ? oinf : inf, i2 = hi ? inf : oinf;
    const u32 j = lane & 3u;
    f29 t, H, R, X3, VX, Y3;
    // S1: A = Z1^2 (j0), B = Z2^2 (j1), C = Z1 Z2 (j2)
    f29_mul_ilp(t, sel4_29(j, p1.z, p2.z, p1.z, p1.z), sel4_29(j, p1.z, p2.z, p2.z, p1.z));
    const f29 A = dpp29<QB(0)>(t), B = dpp29<QB(1)>(t), C = dpp29<QB(2)>(t);
    // S2: U1 = X1 B (j0), U2 = X2 A (j1), T1 = Z1 A (j2), T2 = Z2 B (j3)
    f29_mul_ilp(t, sel4_29(j, p1.x, p2.x, p1.z, p2.z), sel4_29(j, B, A, A, B));
    const f29 U1 = dpp29<QB(0)>(t), U2 = dpp29<QB(1)>(t), T1 = dpp29<QB(2)>(t), T2 = dpp29<QB(3)>(t);
    f29_sub(H, U2, U1);  // N+-
    // S3: S1 = Y1 T2 (j0), S2 = Y2 T1 (j1), Z3 = C H (j2), HH = H^2 (j3)
    f29_mul_ilp(t, sel4_29(j, p1.y, p2.y, C, H), sel4_29(j, T2, T1, H, H));
    const f29 S1 = dpp29<QB(0)>(t), S2 = dpp29<QB(1)>(t), Z3 = dpp29<QB(2)>(t), HH = dpp29<QB(3)>(t);
    f29_sub(R, S2, S1);  // N+-
    // S4: RR = R^2 (j0), HHH = H HH (j1), V = U1 HH (j2)
    f29_mul_ilp(t, sel4_29(j, R, H, U1, R), sel4_29(j, R, HH, HH, R));
    const f29 RR = dpp29<QB(0)>(t), HHH = dpp29<QB(1)>(t), V = dpp29<QB(2)>(t);
#pragma unroll
    for (int i = 0; i < 9; ++i) t.v[i] = RR.v[i] - HHH.v[i] - (V.v[i] << 1);  // (-3 2^29, 2^29)
    f29_normalize(X3, t);
    f29_sub(VX, V, X3);  // (-2^29.2, 2^29 + 2^26)
    // S5: S1 HHH (j0), R (V - X3) (j1)
    f29_mul_ilp(t, sel2_29((j & 1u) != 0, S1, R), sel2_29((j & 1u) != 0, HHH, VX));
    f29_sub(Y3, dpp29<QB(1)>(t), dpp29<QB(0)>(t));  // N+-
    jp29 out;
    out.x = X3;
    out.y = Y3;
    out.z = Z3;
    jp29_sel(out, i2, p1);
    jp29_sel(out, i1, p2);
    acc = out;
    inf = i1 && i2;
}

__device__ __constant__ static const u32 C29_P1[9] = P256_F29_P;
__device__ __constant__ static const u32 C29_P3[9] = P256_F29_3P;

// t == 0 (mod p) for an f29 product output (|t| < 2^256 + 2): t + 2p is one of p, 2p, 3p.
SBFT_DEV bool f29_small_is_zero_modp(const f29& t) {
    f29 u;
    f29_add(u, t, f29_const(C29_2P));
    f29_norm_chain(u, u);
    bool e1 = true, e2 = true, e3 = true;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        e1 = e1 && u.v[k] == C29_P1[k];
        e2 = e2 && u.v[k] == C29_2P[k];
        e3 = e3 && u.v[k] == C29_P3[k];
    }
    return e1 || e2 || e3;
}

// The final check of the lean butterfly, spread over each quad (every lane holds R = acc):
//   1: Z^2 | r R2 | (r + n) R2 | Z 1        2: r Z^2 | (r + n) Z^2 (Montgomery)
//   3: (X - r Z^2) 1 | (X - (r + n) Z^2) 1, then each lane tests its value for 0 mod p.
// exc: Z == 0 (an exceptional addition happened); the verdict: X == r Z^2, or X == (r + n) Z^2
// when r + n < p. Both wave-uniform.
SBFT_DEV bool keyed29_final(const jp29& acc, const fe& rv, u32 lane, bool& exc) {
    fe rn;
    u64 c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        c = (u64)rv.v[k] + P256_N[k] + c;
        rn.v[k] = lo32(c);
        c >>= 32;
    }
    const bool rn_ok = c == 0 && fe_lt(rn, P256_P);
    const u32 j = lane & 3u;
    const f29 r2 = f29_const(C29_R2);
    f29 one;
#pragma unroll
    for (int i = 0; i < 9; ++i) one.v[i] = i == 0 ? 1u : 0u;
    f29 t;
    f29_mul_ilp(t, sel4_29(j, acc.z, f29_from_u256(rv), f29_from_u256(rn), acc.z), sel4_29(j, acc.z, r2, r2, one));
    const f29 z2 = dpp29<QB(0)>(t), rma = dpp29<QB(1)>(t), rmb = dpp29<QB(2)>(t), zt = dpp29<QB(3)>(t);
    const bool odd = (j & 1u) != 0;
    f29_mul_ilp(t, sel2_29(odd, rma, rmb), z2);  // r Z^2 | (r + n) Z^2
    f29 d;
    f29_sub(d, acc.x, t);                        // (-2^29 - 2^26, 2^29 + 2^26)
    f29_mul_ilp(t, d, one);
    const bool z = f29_small_is_zero_modp(t);
    const bool za = __builtin_amdgcn_readlane(z ? 1 : 0, 0) != 0, zb = __builtin_amdgcn_readlane(z ? 1 : 0, 1) != 0;
    exc = f29_small_is_zero_modp(zt);
    return za || (rn_ok && zb);
}

// One wavefront per tuple. Digests come either precomputed (digest != null) or as messages
// blob[off[t] .. +len[t]) hashed here (digest == null). key[t] indexes keytab (slot 0 is G's
// table, so registered keys are 1 .. nkeys-1).
// Two wavefronts per signature: wave 1 inverts s (safegcd, wave-uniform: the compiler runs it
// on the scalar unit, ~37k cycles) while wave 0 hashes the message; they meet at one barrier
// and wave 0 carries on alone. The two dependent chains overlapped instead of following each
// other.
__global__ __launch_bounds__(128) void p256_verify_keyed_wave_kernel(
    const uint8_t* __restrict__ digest, const uint8_t* __restrict__ blob, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint8_t* __restrict__ rr, const uint8_t* __restrict__ ss,
    const uint32_t* __restrict__ key, const uint4* const* __restrict__ keytab, uint32_t nkeys,
    uint8_t* __restrict__ ok, uint32_t n, uint8_t mark, const uint32_t* __restrict__ winv) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    __shared__ u32 w_lds[8];
    SBFT_KEYED_MARK(0);
    if (!winv) inv::stage_divstep_table(dtab);  // (kernel-uniform: winv is an argument)
    SBFT_KEYED_MARK(1);
    const uint32_t t = blockIdx.x;
    const u32 lane = threadIdx.x & 63u;
    const u32 wave = threadIdx.x >> 6;
    if (t >= n) return;  // uniform per workgroup

    const fe r = load_be32(rr + 32ull * t);
    const fe s = load_be32(ss + 32ull * t);
    const uint32_t kid = key[t];
    // an invalid registered key has a null table pointer
    const bool valid = !fe_is_zero_raw(r) && fe_lt(r, P256_N) && !fe_is_zero_raw(s) && fe_lt(s, P256_N) &&
                       kid >= 1 && kid < nkeys && keytab[kid] != nullptr;
    fe e_raw;
    if (wave == 1 && winv) {  // s^-1 R mod n from the host (host_sinv_batch, gpuverify.cpp)
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 8; ++k) w_lds[k] = winv[8ull * t + k];
    } else if (wave == 1) {
        // w = s^-1 (plain)
        fe sv = s, w;
        if (!valid) {
            sv = fe_zero();
            sv.v[0] = 1;
        }
        const fe rn = fe_const(C_ONEN);  // 2^256 mod n: w comes out in Montgomery form
        inv::inv_mod_wave(w.v, sv.v, dtab, false, rn.v);
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 8; ++k) w_lds[k] = w.v[k];
    } else if (digest) {
        e_raw = load_be32(digest + 32ull * t);
    } else {
        uint32_t h[8];
        sha256_one(blob + off[t], len[t], h);
#pragma unroll
        for (int k = 0; k < 8; ++k) e_raw.v[k] = h[7 - k];
    }
    __syncthreads();
    SBFT_KEYED_MARK(2);
    if (wave == 1) return;
    fe wm;  // s^-1 R mod n
#pragma unroll
    for (int k = 0; k < 8; ++k) wm.v[k] = w_lds[k];
    // lanes 0-31 take the G windows of u1 = e s^-1, lanes 32-63 the Q windows of u2 = r s^-1:
    // each lane needs one of the two products
    fe e, u;
    fn_canon(e, e_raw);
    fn_mul(u, lane < 32 ? e : r, wm);
    fn_canon(u, u);
    SBFT_KEYED_MARK(3);

    // this lane's table point
    const u32 win = lane & 31u;
    const u32 digit = byte_of(u, win);
    const uint4* tab = keytab[lane < 32 ? 0u : (valid ? kid : 0u)];
    const uint4* ent = tab + (size_t)(win * COMB_ENTRIES + digit) * COMB_ENTRY_U4;
    jp acc;
    bool inf = digit == 0;
    {
        const uint4 a = ent[0], b = ent[1], c = ent[2], d = ent[3];
        acc.x = {{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
        acc.y = {{c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w}};
        acc.z = fe_const(C_ONEP);
    }
    SBFT_KEYED_MARK(4);
    // butterfly: after level k every lane holds the sum of its aligned group of 2^(k+1) points
    // (the same representation on every lane of the group: the additions are cooperative)
    bool exact = !SBFT_KEYED_F29;
    if (SBFT_KEYED_F29) {
        jp29 a29;
        entry_to_f29(acc.x, acc.y, a29);
        bool inf29 = inf;
        coop29_add_affine_pair(a29, inf29, lane);
        SBFT_KEYED_MARK(5);
#pragma unroll 1
        for (int lvl = 1; lvl < 6; ++lvl) coop29_add_jac_quad(a29, inf29, lane, lvl);
        SBFT_KEYED_MARK(6);
        bool exc = false;
        const bool accept = keyed29_final(a29, r, lane, exc) && !inf29;
        // every lane holds the same point: exc is wave-uniform
        exact = __builtin_amdgcn_readfirstlane((!inf29 && exc) ? 1 : 0) != 0;
        if (!exact && lane == 0) ok[t] = ((valid && accept) ? 1 : 0) | mark;
    }
    if (exact) {  // rare: an exceptional addition in the lean butterfly (or SBFT_KEYED_F29 0)
        coop_add_affine_pair(acc, inf, lane);
        SBFT_KEYED_MARK(5);
#pragma unroll 1
        for (int lvl = 1; lvl < 6; ++lvl) coop_add_jac_quad(acc, inf, lane, lvl);
        SBFT_KEYED_MARK(6);
        if (lane == 0) ok[t] = ((valid && !inf && x_matches_r(acc, r)) ? 1 : 0) | mark;
    }
    SBFT_KEYED_MARK(7);
}

// ---- latency-path signing (api.Signer: SignProposal at view.go:481, Sign at viewchanger.go:445)
// Two wavefronts per signature over G's comb table (keytab slot 0). Wave 1 inverts k (mod n,
// scaled to Montgomery form) while wave 0 computes R = k G from 32 table points with the lean
// radix-2^29 butterfly above and makes it affine (one wave-wide inversion mod p); they meet at
// one barrier for s = k^-1 (e + r d). Q = d G (same butterfly, a second inversion) only when
// the caller asks for it (qx_out != null): a signer derives its key once. The lean additions
// never meet an exceptional case here: every partial sum of the butterfly is a multiple
// 0 < m < k < n of G over disjoint windows, so two of them never coincide or cancel (a Z = 0
// would only mark the signature failed, which the caller retries with another nonce). Same
// outputs and status as p256_sign_kernel (one signature per lane, bench workload generation).

// k G on the whole wavefront (lanes < 32: window `lane` of k; lanes >= 32 add nothing)
SBFT_DEV void wave29_mul_g(jp29& acc, bool& inf, const fe& k, const uint4* gtab, u32 lane) {
    const u32 win = lane & 31u;
    const u32 digit = lane < 32 ? byte_of(k, win) : 0u;
    const uint4* ent = gtab + (size_t)(win * COMB_ENTRIES + digit) * COMB_ENTRY_U4;
    inf = digit == 0;
    const uint4 a = ent[0], b = ent[1], c = ent[2], d = ent[3];
    const fe x = {{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
    const fe y = {{c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w}};
    entry_to_f29(x, y, acc);
    coop29_add_affine_pair(acc, inf, lane);
#pragma unroll 1
    for (int lvl = 1; lvl < 6; ++lvl) coop29_add_jac_quad(acc, inf, lane, lvl);
}

// Affine coordinates (plain, canonical) of a Jacobian f29 point; bad when Z == 0.
SBFT_DEV void affine29(const jp29& p, fe& x, fe* y, bool& bad, const uint32_t* dtab) {
    const fe zc = f29_canon_plain(p.z);
    bad = fe_is_zero_raw(zc);
    fe zi;
    inv::inv_mod_wave(zi.v, zc.v, dtab, true);  // plain Z^-1 (0 for Z == 0)
    f29 zm, z2, t;
    f29_mul_ilp(zm, f29_from_u256(zi), f29_const(C29_R2));  // Montgomery form
    f29_mul_ilp(z2, zm, zm);
    f29_mul_ilp(t, p.x, z2);
    x = f29_canon_plain(t);
    if (y) {
        f29 z3;
        f29_mul_ilp(z3, z2, zm);
        f29_mul_ilp(t, p.y, z3);
        *y = f29_canon_plain(t);
    }
}

__global__ __launch_bounds__(128) void p256_sign_wave_kernel(const uint8_t* __restrict__ dd, const uint8_t* __restrict__ kk,
                                                             const uint8_t* __restrict__ ee, const uint4* const* __restrict__ keytab,
                                                             uint8_t* __restrict__ qx_out, uint8_t* __restrict__ qy_out,
                                                             uint8_t* __restrict__ r_out, uint8_t* __restrict__ s_out,
                                                             uint8_t* __restrict__ status, uint32_t n) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    __shared__ u32 kinv_lds[8];
    inv::stage_divstep_table(dtab);
    const uint32_t t = blockIdx.x;
    const u32 lane = threadIdx.x & 63u;
    const u32 wave = threadIdx.x >> 6;
    if (t >= n) return;  // uniform per workgroup
    const fe d = load_be32(dd + 32ull * t), k = load_be32(kk + 32ull * t);
    bool ok = !fe_is_zero_raw(d) && fe_lt(d, P256_N) && !fe_is_zero_raw(k) && fe_lt(k, P256_N);
    fe r;
    if (wave == 1) {
        fe kv = k;
        if (!ok) {
            kv = fe_zero();
            kv.v[0] = 1;
        }
        const fe rn = fe_const(C_ONEN);
        fe kinv;
        inv::inv_mod_wave(kinv.v, kv.v, dtab, false, rn.v);  // k^-1 R mod n
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < 8; ++i) kinv_lds[i] = kinv.v[i];
    } else {
        const uint4* gtab = keytab[0];
        jp29 P;
        bool inf, bad;
        fe x;
        if (qx_out) {  // Q = d G (the public key)
            fe y;
            wave29_mul_g(P, inf, d, gtab, lane);
            affine29(P, x, &y, bad, dtab);
            if (lane == 0) {
                store_be32(qx_out + 32ull * t, x);
                store_be32(qy_out + 32ull * t, y);
            }
        }
        wave29_mul_g(P, inf, k, gtab, lane);  // R = k G
        affine29(P, x, nullptr, bad, dtab);
        ok = ok && !inf && !bad;
        fn_canon(r, x);  // x < p < 2n
    }
    __syncthreads();
    if (wave == 1) return;
    fe kinv;
#pragma unroll
    for (int i = 0; i < 8; ++i) kinv.v[i] = kinv_lds[i];
    const fe e_raw = load_be32(ee + 32ull * t);
    fe e, dm, rd, sum, sv;
    fn_canon(e, e_raw);
    fn_mul(dm, d, fe_const(C_R2N));  // d R
    fn_mul(rd, r, dm);               // r d (plain, lazily reduced)
    fn_canon(rd, rd);
    fn_add(sum, e, rd);              // e + r d mod n
    fn_mul(sv, sum, kinv);           // (e + r d) k^-1 (plain)
    fn_canon(sv, sv);
    ok = ok && !fe_is_zero_raw(r) && !fe_is_zero_raw(sv);
    if (lane == 0) {
        store_be32(r_out + 32ull * t, r);
        store_be32(s_out + 32ull * t, sv);
        status[t] = ok ? 1 : 0;
    }
}

}  // namespace sbft

extern "C" int sbft_launch_p256_sign_wave(const uint8_t* d_d, const uint8_t* d_k, const uint8_t* d_e,
                                          const void* const* d_keytab, uint8_t* d_qx, uint8_t* d_qy, uint8_t* d_r,
                                          uint8_t* d_s, uint8_t* d_status, uint32_t n, hipStream_t stream) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    hipLaunchKernelGGL(sbft::p256_sign_wave_kernel, dim3(n), dim3(128), 0, stream, d_d, d_k, d_e,
                       (const uint4* const*)d_keytab, d_qx, d_qy, d_r, d_s, d_status, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sbft_launch_comb_build(const uint8_t* d_qx, const uint8_t* d_qy, void* d_tables,
                                      uint32_t* d_status, uint32_t nk, hipStream_t stream) {
    if (nk == 0) return 0;
    const unsigned threads = 256;
    const uint64_t total = (uint64_t)nk * COMB_WINDOWS * COMB_ENTRIES;
    hipLaunchKernelGGL(sbft::p256_comb_build_kernel, dim3((unsigned)(total / threads)), dim3(threads), 0, stream,
                       d_qx, d_qy, (uint4*)d_tables, d_status, nk);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" size_t sbft_comb_table_bytes(void) { return (size_t)COMB_KEY_U4 * 16; }

extern "C" int sbft_launch_p256_verify_keyed(const uint8_t* d_digest, const uint8_t* d_blob, const uint64_t* d_off,
                                             const uint32_t* d_len, const uint8_t* d_r, const uint8_t* d_s,
                                             const uint32_t* d_key, const void* const* d_keytab, uint32_t nkeys,
                                             uint8_t* d_ok, uint32_t n, uint8_t mark, const uint32_t* d_winv,
                                             hipStream_t stream) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    if (!d_digest && (!d_blob || !d_off || !d_len)) return -1;
    hipLaunchKernelGGL(sbft::p256_verify_keyed_wave_kernel, dim3(n), dim3(128), 0, stream, d_digest, d_blob, d_off,
                       d_len, d_r, d_s, d_key, (const uint4* const*)d_keytab, nkeys, d_ok, n, mark, d_winv);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
