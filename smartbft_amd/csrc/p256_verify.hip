// p256_verify.hip — batched ECDSA P-256 verification for gfx950.
//
// One verify per lane. Per lane (Go 1.24.1 crypto/ecdsa.Verify semantics, restated in
// oracle/p256_oracle.c, which the parity tests hold this kernel to bit for bit):
//   1. range checks r, s in [1, n-1]; Qx, Qy < p; Q on y^2 = x^3 - 3x + b
//   2. e = digest mod n; w = s^-1 mod n (batched over the launch: Montgomery's trick in
//      1,024-tuple groups, one safegcd inversion of the product of the group totals)
//   3. u1 = e*w, u2 = r*w
//   4. R = u2*Q + u1*G. u2*Q: 256 doublings with radix-16 regular signed-odd digits (never
//      zero, so every addition is live and select-free) over [1,3,..,15]Q, built per lane with
//      co-Z additions and made affine with one safegcd inversion mod p (scratch; 64 mixed
//      additions). u1*G: K + 1 mixed additions from a fixed-base comb table of K W-bit windows
//      in HBM (built once per device), after the ladder
//   5. R = infinity -> reject; accept iff X == r*Z^2 or (r+n < p and X == (r+n)*Z^2)
// Exceptional additions (P + P, P + (-P), infinity) leave Z = 0; such lanes are re-verified by
// the fully case-split p256_verify_fixup_kernel, so adversarial inputs cost only themselves.
//
// Inputs: SoA, 32-byte big-endian fields. Output: one verdict byte per tuple.
#include <cstdio>
#include <cstdlib>

#include "p256_f29.hpp"
#include "p256_halfgcd.hpp"
#include "p256_inv.hpp"
#include "p256_point.hpp"
#include "sbft_kernels.h"
#include "sha256_dev.hpp"

namespace sbft {

// Inclusive product scan mod n (Montgomery form) over the 256 lanes of the workgroup
// (Hillis-Steele, 8 steps through LDS). suffix = true scans from lane 255 down. On return
// buf[k][lane] holds every lane's inclusive value. Called by all 256 threads.
template <int W>
SBFT_DEV void block_scan_mul_n(fe& x, u32 (*buf)[W], int tid, bool suffix) {
#pragma unroll 1
    for (int off = 1; off < W; off <<= 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) buf[k][tid] = x.v[k];
        __syncthreads();
        const int src = suffix ? tid + off : tid - off;
        if (suffix ? (src < W) : (src >= 0)) {
            fe y;
#pragma unroll
            for (int k = 0; k < 8; ++k) y.v[k] = buf[k][src];
            fn_mul(x, x, y);
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) buf[k][tid] = x.v[k];
    __syncthreads();
}

// ------------------------------------------------------------ general path
// The fully case-split verify (Booth radix-16 digits including zero, explicit infinity and
// doubling branches in every addition). It runs only for tuples the lean kernel flagged:
// adversarial inputs whose Shamir ladder hits P + P, P + (-P) or infinity.
// Inlined into its one caller, the fixup kernel. As a __noinline__ function (rounds 1-4) it was
// over 128 KiB of code, so its branches needed long-branch expansion, and from round 4's build on
// the compiler used s[30:31] -- the function's return address -- as the long branches' scratch
// pair: the return jumped into the function's own body and the fixup kernel faulted on its first
// flagged tuple (tools/scan_retaddr.py, run on every CPU test pass, refuses a build
// with such a function). A kernel has no return address to lose.
SBFT_DEV bool verify_general(const fe& e_raw, const fe& r, const fe& s, const fe& qx,
                                            const fe& qy, const u32* gtab) {
    // 1. range checks
    bool valid = !fe_is_zero_raw(r) && fe_lt(r, P256_N) && !fe_is_zero_raw(s) && fe_lt(s, P256_N) &&
                 fe_lt(qx, P256_P) && fe_lt(qy, P256_P);

    // Q to Montgomery form and on-curve check y^2 == x^3 - 3x + b
    const fe r2p = fe_const(C_R2P);
    jp q;
    fp_mul(q.x, qx, r2p);
    fp_mul(q.y, qy, r2p);
    q.z = fe_const(C_ONEP);
    {
        fe lhs, rhs, t;
        fp_sqr(lhs, q.y);
        fp_sqr(rhs, q.x);
        fp_mul(rhs, rhs, q.x);
        fp_add(t, q.x, q.x);
        fp_add(t, t, q.x);
        fp_sub(rhs, rhs, t);
        fp_add(rhs, rhs, fe_const(C_BM));
        fp_canon(lhs, lhs);
        fp_canon(rhs, rhs);
        valid = valid && fe_eq(lhs, rhs);
    }

    // 2-3. scalars
    fe e;
    fn_canon(e, e_raw);
    fe sm, w, u1, u2;
    fn_mul(sm, s, fe_const(C_R2N));  // s*R mod n
    fn_inv(w, sm);                    // s^-1 * R
    fn_mul(u1, e, w);                 // e*s^-1 (plain)
    fn_mul(u2, r, w);                 // r*s^-1 (plain)

    // 4. [1..8]Q in Jacobian form (scratch)
    jp tq[8];
    tq[0] = q;
    pt_dbl(tq[1], q);
#pragma unroll 1
    for (int k = 2; k < 8; ++k) {
        jp t = tq[k - 1];
        bool tinf = false;
        pt_add_jac(t, tinf, q, true);
        tq[k] = t;
    }

    jp acc;
    bool inf = true;
    acc.x = fe_zero();
    acc.y = fe_zero();
    acc.z = fe_zero();
    // window 64: the digit is bit 255
    {
        const bool b2 = (u2.v[7] >> 31) != 0;
        const bool b1 = (u1.v[7] >> 31) != 0;
        pt_add_jac(acc, inf, q, b2);
        fe gx, gy;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            gx.v[k] = gtab[k];
            gy.v[k] = gtab[8 + k];
        }
        pt_add_aff(acc, inf, gx, gy, b1);
    }
    fe k1 = u1, k2 = u2;
#pragma unroll 1
    for (int limb = 7; limb >= 0; --limb) {
        const u32 cur1 = k1.v[7], below1 = k1.v[6];
        const u32 cur2 = k2.v[7], below2 = k2.v[6];
#pragma unroll
        for (int k = 7; k > 0; --k) {
            k1.v[k] = k1.v[k - 1];
            k2.v[k] = k2.v[k - 1];
        }
        k1.v[0] = 0;
        k2.v[0] = 0;
        const u64 w1 = ((u64)cur1 << 1) | (below1 >> 31);
        const u64 w2 = ((u64)cur2 << 1) | (below2 >> 31);
#pragma unroll 1
        for (int nib = 7; nib >= 0; --nib) {
#pragma unroll 1
            for (int d = 0; d < 4; ++d) pt_dbl(acc, acc);
            const int d2 = booth((u32)(w2 >> (4 * nib)) & 31u);
            const int d1 = booth((u32)(w1 >> (4 * nib)) & 31u);
            // Q digit
            {
                const int m = d2 < 0 ? -d2 : d2;
                jp t = tq[m > 0 ? m - 1 : 0];
                if (d2 < 0) {
                    fe ny;
                    fp_sub(ny, fe_zero(), t.y);
                    t.y = ny;
                }
                pt_add_jac(acc, inf, t, d2 != 0);
            }
            // G digit
            {
                const int m = d1 < 0 ? -d1 : d1;
                const int base = (m > 0 ? m - 1 : 0) * 16;
                fe gx, gy;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    gx.v[k] = gtab[base + k];
                    gy.v[k] = gtab[base + 8 + k];
                }
                if (d1 < 0) {
                    fe ny;
                    fp_sub(ny, fe_zero(), gy);
                    gy = ny;
                }
                pt_add_aff(acc, inf, gx, gy, d1 != 0);
            }
        }
    }

    // 5. x(R) mod n == r, projectively
    bool accept = false;
    if (!inf) {
        fe z2, lhs, xc, rm;
        fp_sqr(z2, acc.z);
        fp_canon(xc, acc.x);
        fp_mul(rm, r, r2p);
        fp_mul(lhs, rm, z2);
        fp_canon(lhs, lhs);
        accept = fe_eq(lhs, xc);
        // r + n < p ?
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
    }
    return valid && accept;
}

__global__ __launch_bounds__(256) void p256_verify_fixup_kernel(const uint8_t* __restrict__ digest,
                                                                const uint8_t* __restrict__ rr,
                                                                const uint8_t* __restrict__ ss,
                                                                const uint8_t* __restrict__ qxx,
                                                                const uint8_t* __restrict__ qyy,
                                                                uint8_t* __restrict__ ok,
                                                                const uint32_t* __restrict__ work) {
    __shared__ u32 gtab[2 * 8 * P256_GTAB4_ENTRIES];
    const uint32_t count = work[0];
    if (blockIdx.x * blockDim.x >= count) return;  // block-uniform: the grid is sized for the worst case
    for (int i = threadIdx.x; i < 2 * 8 * P256_GTAB4_ENTRIES; i += blockDim.x) gtab[i] = C_GTAB[i];
    __syncthreads();
    const uint32_t* list = work + 1;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
        const uint32_t idx = list[j];
        const bool v = verify_general(load_be32(digest + 32ull * idx), load_be32(rr + 32ull * idx),
                                      load_be32(ss + 32ull * idx), load_be32(qxx + 32ull * idx),
                                      load_be32(qyy + 32ull * idx), gtab);
        ok[idx] = v ? 1 : 0;
    }
}

// lanes = 0 (sbft_launch_p256_verify): every tuple through the fixup kernel -- the count and
// the list 0 .. n-1 written on the device, so the whole launch stays on the stream
__global__ __launch_bounds__(256) void p256_fixup_all_kernel(uint32_t* __restrict__ work, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) work[0] = n;
    if (i < n) work[1 + i] = i;
}

// ------------------------------------------------------------ batched s^-1
// Montgomery's trick over the whole launch: s_i^-1 = G^-1 * E_g * F_g * pre_{i-1} * suf_{i+1},
// with G the product of all s, E_g / F_g the products of the group totals before / after
// group g (groups of SBFT_SINV_GROUP = 1,024 tuples), and pre / suf the inclusive products
// inside group g. One safegcd inversion (p256_inv.hpp) per launch replaces one per lane.
//   prep kernel   : per group, prefix/suffix scans of s*R -> pre, suf, tot[g]
//   totals kernel : one workgroup: scans of tot, G^-1, K_g = G^-1 E_g F_g -> kb[g]
//   main kernel   : w_i = K_g * pre_{i-1} * suf_{i+1}
// Lanes with s outside [1, n-1] (or past n) contribute 1, so every product is invertible.
struct sinv_ws {
    uint4* pre;  // n x 32 B (Montgomery limbs, little-endian)
    uint4* suf;  // n x 32 B
    uint4* tot;  // nb x 32 B
    uint4* kb;   // nb x 32 B
    uint4* qtab; // n x SBFT_VERIFY_QTAB_BYTES: per-lane Q tables (SBFT_QTAB_GLOBAL)
};
#ifdef SBFT_DEBUG_BOUNDS
#define SBFT_CHECK(cond, what, a, b)                                                              \
    do {                                                                                          \
        if (!(cond)) {                                                                            \
            printf("SBFT bounds: %s (%llu vs %llu) block %u thread %u\n", what,                    \
                   (unsigned long long)(a), (unsigned long long)(b), blockIdx.x, threadIdx.x);   \
            return;                                                                               \
        }                                                                                         \
    } while (0)
#else
#define SBFT_CHECK(cond, what, a, b) \
    do {                             \
    } while (0)
#endif
SBFT_DEV void st_fe(uint4* p, const fe& a) {
    p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    p[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
SBFT_DEV fe ld_fe(const uint4* p) {
    const uint4 a = p[0], b = p[1];
    fe r = {{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
    return r;
}

// s^-1 groups of SBFT_SINV_GROUP tuples (1,024): each group gets inclusive pre / suf
// products and a total tot[g]; the totals kernel turns the totals into kb[g] = 1 / tot[g].
// One 128-lane workgroup per group, eight consecutive tuples per lane: serial prefix /
// suffix over the lane's eight, a 128-lane scan of the lane products, then each lane
// applies its exclusive neighbour product (~5.9 products per tuple; padding tuples are 1).
#define SBFT_SINV_GROUP_LOG2 10
#define SBFT_SINV_GROUP (1u << SBFT_SINV_GROUP_LOG2)
__global__ __launch_bounds__(128) void p256_sinv_prep_kernel(const uint8_t* __restrict__ ss, uint32_t n,
                                                             sinv_ws ws) {
    constexpr int L = 128, T = SBFT_SINV_GROUP / L;
    __shared__ u32 buf[8][L];
    const int lane = threadIdx.x;
    SBFT_CHECK(blockDim.x == L, "prep geometry", blockDim.x, L);
    const uint32_t g0 = blockIdx.x * SBFT_SINV_GROUP + lane * T;
    const fe one = fe_const(C_ONEN);
    fe x[T];
#pragma unroll
    for (int j = 0; j < T; ++j) {
        x[j] = one;
        if (g0 + j < n) {
            const fe s = load_be32(ss + 32ull * (g0 + j));
            if (!fe_is_zero_raw(s) && fe_lt(s, P256_N)) fn_mul(x[j], s, fe_const(C_R2N));
        }
    }
    {
        // prefix: p_j = x_0..x_j inside the lane, scanned across lanes
        fe p[T];
        p[0] = x[0];
#pragma unroll
        for (int j = 1; j < T; ++j) fn_mul(p[j], p[j - 1], x[j]);
        fe c = p[T - 1];
        block_scan_mul_n(c, buf, lane, false);  // inclusive over lanes; buf holds every lane's value
        if (lane == L - 1) st_fe(ws.tot + 2ull * blockIdx.x, c);
        if (lane > 0) {
            fe e;
#pragma unroll
            for (int k = 0; k < 8; ++k) e.v[k] = buf[k][lane - 1];
#pragma unroll
            for (int j = 0; j < T; ++j) fn_mul(p[j], p[j], e);
        }
#pragma unroll
        for (int j = 0; j < T; ++j)
            if (g0 + j < n) st_fe(ws.pre + 2ull * (g0 + j), p[j]);
    }
    __syncthreads();  // buf is reused by the suffix scan
    // suffix: q_j = x_j..x_{T-1} inside the lane, scanned across lanes from the last lane down
    fe q[T];
    q[T - 1] = x[T - 1];
#pragma unroll
    for (int j = T - 2; j >= 0; --j) fn_mul(q[j], x[j], q[j + 1]);
    fe c = q[0];
    block_scan_mul_n(c, buf, lane, true);
    if (lane < L - 1) {
        fe e;
#pragma unroll
        for (int k = 0; k < 8; ++k) e.v[k] = buf[k][lane + 1];
#pragma unroll
        for (int j = 0; j < T; ++j) fn_mul(q[j], q[j], e);
    }
#pragma unroll
    for (int j = 0; j < T; ++j)
        if (g0 + j < n) st_fe(ws.suf + 2ull * (g0 + j), q[j]);
}

__global__ __launch_bounds__(256) void p256_sinv_totals_kernel(uint32_t nb, sinv_ws ws) {
    SBFT_CHECK(gridDim.x == 1 && blockDim.x == 256, "totals geometry", gridDim.x, blockDim.x);
    __shared__ u32 buf[8][256];
    __shared__ u32 pre_c[8][256];
    __shared__ u32 ginv[8];
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    inv::stage_divstep_table(dtab);  // ends with a barrier
    const int tid = threadIdx.x;
    const uint32_t chunk = (nb + 255) / 256;
    const uint32_t b0 = tid * chunk, b1 = min(nb, b0 + chunk);
    const fe one = fe_const(C_ONEN);
    fe c = one;
    for (uint32_t b = b0; b < b1; ++b) {
        SBFT_CHECK(b < nb, "totals tot idx", b, nb);
        fn_mul(c, c, ld_fe(ws.tot + 2ull * b));
    }
    fe cp = c, cs = c;
    block_scan_mul_n(cp, pre_c, tid, false);  // inclusive prefix of chunk products
    block_scan_mul_n(cs, buf, tid, true);     // inclusive suffix
    if (tid < 64) {
        // G^-1 in Montgomery form: the safegcd inverse of G's Montgomery representative M
        // is M^-1 = g^-1 R^-1, and two multiplications by R^2 (mod n) give g^-1 R. One
        // wavefront, ~0.03 ms (a Fermat chain here was ~0.3 ms of dependent multiplications).
        fe g, gi, m, mi;
#pragma unroll
        for (int k = 0; k < 8; ++k) g.v[k] = pre_c[k][255];
        fn_canon(m, g);
        inv::inv_mod_n(mi.v, m.v, dtab);
        const fe r2n = fe_const(C_R2N);
        fn_mul(gi, mi, r2n);
        fn_mul(gi, gi, r2n);
        if (tid == 0)
#pragma unroll
            for (int k = 0; k < 8; ++k) ginv[k] = gi.v[k];
    }
    __syncthreads();
    fe gi, e, f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        gi.v[k] = ginv[k];
        e.v[k] = tid > 0 ? pre_c[k][tid - 1] : one.v[k];
        f.v[k] = tid < 255 ? buf[k][tid + 1] : one.v[k];
    }
    // forward: kb[b] = G^-1 * E_b ; backward: kb[b] *= F_b
    fe run;
    fn_mul(run, gi, e);
    for (uint32_t b = b0; b < b1; ++b) {
        st_fe(ws.kb + 2ull * b, run);
        fn_mul(run, run, ld_fe(ws.tot + 2ull * b));
    }
    run = f;
    for (uint32_t b = b1; b > b0; --b) {
        fe k = ld_fe(ws.kb + 2ull * (b - 1));
        fn_mul(k, k, run);
        st_fe(ws.kb + 2ull * (b - 1), k);
        fn_mul(run, run, ld_fe(ws.tot + 2ull * (b - 1)));
    }
}

// ------------------------------------------------------------ fixed-base comb for u1*G
// u1*G is summed from a comb table in HBM after the Q ladder (K + 1 mixed additions, no
// doublings): W-bit windows, K = ceil(256 / W) of them, 2^(W-1) odd multiples each. The 33
// radix-256 additions of an LDS table inside the ladder it replaced were 1.6 M instructions per
// 1,000 verifies more. Wider windows trade HBM for additions (entries are gathered, never
// scanned): W = 16: 17 additions, 42 MB; W = 20: 14, 0.55 GB; W = 22: 13, 2.0 GB (the default
// since round 3, built at init in ~0.44 s: once the products with addends had made the
// doublings cheaper, the 4 additions saved were worth 0.9% of the throughput kernel,
// profiles/r03u_gcomb22_ab.txt); W = 24: 12, 7.4 GB.
#ifndef SBFT_GCOMB_W
#define SBFT_GCOMB_W 22
#endif
#define SBFT_GCOMB_WINDOWS ((256 + SBFT_GCOMB_W - 1) / SBFT_GCOMB_W)
#define SBFT_GCOMB_ENTRIES (1u << (SBFT_GCOMB_W - 1))  // odd digits 1, 3, ..., 2^W - 1
// entry = 20 words (80 B, five 16-B loads): x limbs 0..8, pad, y limbs 0..8, pad (f29 Montgomery)
#define SBFT_GCOMB_BYTES ((size_t)(SBFT_GCOMB_WINDOWS * (size_t)SBFT_GCOMB_ENTRIES + 1) * 80)
static_assert(SBFT_GCOMB_W >= 8 && SBFT_GCOMB_W <= 26, "window bits: digits are read from one 32-bit word");
constexpr int kGWin = SBFT_GCOMB_W;
constexpr int kGK = SBFT_GCOMB_WINDOWS;  // windows; entry kGK of the table is 2^(W K) G
constexpr u32 kGMask = (1u << SBFT_GCOMB_W) - 1u;

// affine (x, y) of P as canonical plain integers (8 x 32 domain; one Fermat inversion)
SBFT_DEV void comb_affine(fe& x, fe& y, const jp& p) {
    fe zi, zi2, zi3, t;
    fp_inv(zi, p.z);
    fp_sqr(zi2, zi);
    fp_mul(zi3, zi2, zi);
    const fe one_plain = {{1, 0, 0, 0, 0, 0, 0, 0}};
    fp_mul(t, p.x, zi2);
    fp_mul(t, t, one_plain);
    fp_canon(x, t);
    fp_mul(t, p.y, zi3);
    fp_mul(t, t, one_plain);
    fp_canon(y, t);
}

// 2^e mod n (e <= 280) by modular doubling
SBFT_DEV fe pow2_mod_n(uint32_t e) {
    fe x = fe_zero();
    x.v[0] = 1;
#pragma unroll 1
    for (uint32_t i = 0; i < e; ++i) {
        fe t, d;
        u32 c = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            t.v[k] = (x.v[k] << 1) | c;
            c = x.v[k] >> 31;
        }
        u64 bw = 0;  // 2x < 2n: subtract n once if 2x >= n
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const u64 v = (u64)t.v[k] - P256_N[k] - bw;
            d.v[k] = lo32(v);
            bw = v >> 63;
        }
        const bool ge = c || !bw;
#pragma unroll
        for (int k = 0; k < 8; ++k) x.v[k] = ge ? d.v[k] : t.v[k];
    }
    return x;
}

// table[w][j] = (2j+1) 2^(W w) G for w < K, j < 2^(W-1); table[K][0] = 2^(W K) G. One point per
// thread through the (case-split) fixed-base multiplication of the signer; built once per
// device.
__global__ __launch_bounds__(256) void p256_gcomb_build_kernel(uint4* __restrict__ table) {
    __shared__ u32 gtab4[2 * 8 * P256_GTAB4_ENTRIES];
    for (int i = threadIdx.x; i < 2 * 8 * P256_GTAB4_ENTRIES; i += blockDim.x) gtab4[i] = C_GTAB[i];
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t total = SBFT_GCOMB_WINDOWS * SBFT_GCOMB_ENTRIES + 1;
    if (gid >= total) return;
    // scalar (2j + 1) 2^(W w) mod n: 2^(W w) mod n into Montgomery form, times the odd digit
    const uint32_t w = gid / SBFT_GCOMB_ENTRIES, j = gid % SBFT_GCOMB_ENTRIES;
    fe d = pow2_mod_n((uint32_t)kGWin * w);
    if (w < (uint32_t)kGK) {
        fe odd = fe_zero();
        odd.v[0] = 2 * j + 1;
        fn_mul(d, d, fe_const(C_R2N));  // 2^(W w) R
        fn_mul(d, d, odd);              // (2j + 1) 2^(W w)
        fn_canon(d, d);
    }
    jp P;
    bool inf;
    pt_mul_base(P, inf, d, gtab4);
    fe x, y;
    comb_affine(x, y, P);
    const f29 r2 = f29_const(C29_R2);
    f29 mx, my;
    f29_mul(mx, f29_from_u256(x), r2);
    f29_mul(my, f29_from_u256(y), r2);
    uint4* e = table + (size_t)gid * 5;
    e[0] = make_uint4(mx.v[0], mx.v[1], mx.v[2], mx.v[3]);
    e[1] = make_uint4(mx.v[4], mx.v[5], mx.v[6], mx.v[7]);
    e[2] = make_uint4(mx.v[8], 0u, my.v[0], my.v[1]);
    e[3] = make_uint4(my.v[2], my.v[3], my.v[4], my.v[5]);
    e[4] = make_uint4(my.v[6], my.v[7], my.v[8], 0u);
}

// an affine point as a 20-word entry (the comb's layout): x limbs 0..8, pad, y limbs 0..8, pad
SBFT_DEV void pack_entry(const f29& x, const f29& y, uint4 (&e)[5]) {
    e[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    e[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
    e[2] = make_uint4(x.v[8], 0u, y.v[0], y.v[1]);
    e[3] = make_uint4(y.v[2], y.v[3], y.v[4], y.v[5]);
    e[4] = make_uint4(y.v[6], y.v[7], y.v[8], 0u);
}

// ------------------------------------------------------------ the kernels
// The throughput kernel's Q table: 1 = each lane's 8 entries contiguous in the workspace (640 B
// per tuple, 5 x 16-B loads per digit); 0 = a private array (lane-interleaved scratch, A/B only).
// Same-box A/B (profiles/r03i_qtab_mulsub_ab.txt): 14.75 -> 14.04 ms per 1M, HBM traffic 21.7 ->
// 7.9 KB per verify.
#ifndef SBFT_QTAB_GLOBAL
#define SBFT_QTAB_GLOBAL 1
#endif
#ifndef SBFT_DBL_UNROLL
#define SBFT_DBL_UNROLL 1
#endif
constexpr int kDblUnroll = SBFT_DBL_UNROLL;  // doublings per iteration of the w-doubling loop
#ifndef SBFT_QWIN
#define SBFT_QWIN 4
#endif
constexpr int kQWin = SBFT_QWIN;                    // u2 in radix 2^w (latency kernels)
constexpr int kQTab = 1 << (kQWin - 1);             // [1, 3, ..., 2^w - 1]Q
constexpr int kQDigits = (255 + kQWin - 1) / kQWin; // windows over u2 >> 1 (< 2^255)
// the throughput kernel's window (SBFT_TQWIN): its Q table lives in the workspace
// (SBFT_VERIFY_QTAB_BYTES per tuple), the latency kernels' in LDS
constexpr int kTWin = SBFT_TQWIN;
constexpr int kTTab = 1 << (kTWin - 1);
constexpr int kTDigits = (255 + kTWin - 1) / kTWin;
static_assert(kTTab * 80 == SBFT_VERIFY_QTAB_BYTES, "workspace Q-table stride (sbft_kernels.h)");
#ifndef SBFT_VERIFY_WAVES
#define SBFT_VERIFY_WAVES 4
#endif

// 1. range checks and the on-curve check y^2 == x^3 - 3x + b (8 x 32 Montgomery domain)
// The range part of verify_inputs_valid: r, s in [1, n), Qx, Qy in [0, p).
SBFT_DEV bool verify_inputs_in_range(const fe& r, const fe& s, const fe& qx, const fe& qy) {
    return !fe_is_zero_raw(r) && fe_lt(r, P256_N) && !fe_is_zero_raw(s) && fe_lt(s, P256_N) && fe_lt(qx, P256_P) &&
           fe_lt(qy, P256_P);
}
SBFT_DEV bool verify_inputs_valid(const fe& r, const fe& s, const fe& qx, const fe& qy) {
    bool valid = !fe_is_zero_raw(r) && fe_lt(r, P256_N) && !fe_is_zero_raw(s) && fe_lt(s, P256_N) &&
                 fe_lt(qx, P256_P) && fe_lt(qy, P256_P);
    const fe r2p = fe_const(C_R2P);
    fe x, y, lhs, rhs, t;
    fp_mul(x, qx, r2p);
    fp_mul(y, qy, r2p);
    fp_sqr(lhs, y);
    fp_sqr(rhs, x);
    fp_mul(rhs, rhs, x);
    fp_add(t, x, x);
    fp_add(t, t, x);
    fp_sub(rhs, rhs, t);
    fp_add(rhs, rhs, fe_const(C_BM));
    fp_canon(lhs, lhs);
    fp_canon(rhs, rhs);
    return valid && fe_eq(lhs, rhs);
}

// The odd multiples [1,3,...,2^w - 1]Q in the radix-2^29 Montgomery domain of the ladder
// (p256_f29.hpp), affine. Invalid lanes run a harmless stand-in (Q = 2G); their verdict is
// masked by `valid` at the end. Built with co-Z additions (DBLU, then ZADDU of the running 2Q:
// 4M + 2S each), then made affine with ONE inversion per lane (safegcd mod p of the final Z;
// the earlier Z's follow from the recorded ratios h_k).
// inv_p(z) returns z^-1 mod p (plain 8 x 32 limbs) for the plain canonical z.
template <int TAB, class InvP>
SBFT_DEV void build_q_table(f29 (&tx)[TAB], f29 (&ty)[TAB], const fe& qx, const fe& qy, bool valid,
                            InvP inv_p) {
    const f29 r2 = f29_const(C29_R2);
    f29 qxm, qym;
    f29_mul(qxm, f29_from_u256(qx), r2);
    f29_mul(qym, f29_from_u256(qy), r2);
    if (!valid) {
        qxm = f29_const(C29_G2X);
        qym = f29_const(C29_G2Y);
    }
    tx[0] = qxm;
    ty[0] = qym;
    f29 dx, dy, cx, cy, z;  // D = 2Q and the current odd multiple, co-Z (Z = z)
    p29_dblu(qxm, qym, dx, dy, cx, cy, z);
    f29 hs[TAB - 1];      // Z ratios: Z(T_k) = Z(T_{k-1}) h_k
#pragma unroll 1
    for (int k = 1; k < TAB; ++k) {
        f29 h;
        p29_zaddu(cx, cy, dx, dy, h);  // T_k = T_{k-1} + 2Q
        tx[k] = cx;
        ty[k] = cy;
        hs[k - 1] = h;
        f29_mul(z, z, h);              // 2^30 (first) x 2^29.3
    }
    f29 inv;  // 1 / Z(T_last), Montgomery form
    {
        const fe zi = inv_p(f29_canon_plain(z));
        f29_mul(inv, f29_from_u256(zi), r2);
    }
#pragma unroll 1
    for (int k = TAB - 1; k >= 1; --k) {
        f29 zi2, zi3;
        f29_sqr(zi2, inv);
        f29_mul(zi3, zi2, inv);
        f29_mul(tx[k], tx[k], zi2);
        f29_mul(ty[k], ty[k], zi3);
        f29_mul(inv, inv, hs[k - 1]);  // 1 / Z(T_{k-1})
    }
}

// build_q_table on a lane pair (p256_verify_small_kernel<2>): the same products and bounds, two
// per step (see p29_dbl_pair). Conversion 1 step instead of 2, DBLU 4 instead of 6, each ZADDU
// 3 instead of 6, the product of the Z ratios a 4-step tree instead of a 7-product chain, and
// each affine conversion 3 steps instead of 5.
// The pair build from the point already in the radix-2^29 Montgomery domain (qxm, qym in N).
template <class InvP>
SBFT_DEV void build_q_table_pair_m(f29 (&tx)[kQTab], f29 (&ty)[kQTab], const f29& qxm, const f29& qym, bool odd,
                                   InvP inv_p);
template <class InvP>
SBFT_DEV void build_q_table_pair(f29 (&tx)[kQTab], f29 (&ty)[kQTab], const fe& qx, const fe& qy, bool valid,
                                 bool odd, InvP inv_p) {
    const f29 r2 = f29_const(C29_R2);
    f29 qxm, qym, o;
    f29_mul_ilp(o, f29_pick(odd, f29_from_u256(qx), f29_from_u256(qy)), r2);
    f29_unpair(o, qxm, qym);
    if (!valid) {
        qxm = f29_const(C29_G2X);
        qym = f29_const(C29_G2Y);
    }
    build_q_table_pair_m(tx, ty, qxm, qym, odd, inv_p);
}
template <class InvP>
SBFT_DEV void build_q_table_pair_m(f29 (&tx)[kQTab], f29 (&ty)[kQTab], const f29& qxm, const f29& qym, bool odd,
                                   InvP inv_p) {
    static_assert(kQTab == 8, "the Z-ratio product tree below is written for 7 ratios");
    // e = a0 b0 (even lane's product), d = a1 b1 (odd lane's), both in both lanes
    auto pmul = [odd](f29& e, f29& d, const f29& a0, const f29& b0, const f29& a1, const f29& b1) {
        f29 o;
        f29_mul_ilp(o, f29_pick(odd, a0, a1), f29_pick(odd, b0, b1));
        f29_unpair(o, e, d);
    };
    const f29 r2 = f29_const(C29_R2);
    tx[0] = qxm;
    ty[0] = qym;
    f29 dx, dy, cx, cy, z;  // D = 2Q and the current odd multiple, co-Z (Z = z)
    {                        // DBLU (p29_dblu): B = x^2 | E = y^2, L = E^2 | x E, M^2, M (S - X2)
        f29 b, e, l, t, m, m2;
        pmul(b, e, qxm, qxm, qym, qym);
        pmul(l, t, e, e, qxm, e);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] <<= 2;  // 4xE < 2^31
        f29_normalize(cx, t);                       // S (N')
        const f29 one = f29_const(C29_ONE);
#pragma unroll
        for (int i = 0; i < 9; ++i) m.v[i] = 3 * (b.v[i] - one.v[i]);  // |.| < 2^30.6
        f29_normalize(m, m);                        // M (N')
        f29_mul_ilp(m2, m, m);                      // 2^29.2^2
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] = m2.v[i] - (cx.v[i] << 1);
        f29_normalize(dx, t);                       // X2 (N')
#pragma unroll
        for (int i = 0; i < 9; ++i) l.v[i] <<= 2;  // 4L < 2^31
        f29_normalize(l, l);
#pragma unroll
        for (int i = 0; i < 9; ++i) l.v[i] <<= 1;  // 8L, |.| < 2^30.2
        f29_normalize(cy, l);                       // 8L (N')
        f29_sub(t, cx, dx);                         // S - X2, |.| < 2^29.3
        f29_mul_ilp(m2, m, t);                      // 2^29.2 x 2^29.3
        f29_sub(t, m2, cy);
        f29_normalize(dy, t);                       // Y2 (N')
        f29_add(z, qym, qym);                       // Z = 2y
    }
    f29 hs[kQTab - 1];  // Z ratios: Z(T_k) = Z(T_{k-1}) h_k
#pragma unroll 1
    for (int k = 1; k < kQTab; ++k) {  // ZADDU (p29_zaddu): H^2 | R^2, W1 | W2, A1 | R (W1 - X3)
        f29 h, r, c, dd, w1, w2, t, u, a1, c2;
        f29_sub(h, dx, cx);               // |.| < 2^29.3
        f29_sub(r, dy, cy);               // |.| < 2^29.3
        pmul(c, dd, h, h, r, r);
        pmul(w1, w2, dx, c, cx, c);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] = dd.v[i] - w1.v[i] - w2.v[i];  // (-2^30, 2^29)
        f29_normalize(cx, t);             // X3 (N')
        f29_sub(u, w1, w2);               // |.| < 2^29
        f29_sub(t, w1, cx);               // |.| < 2^29.2
        pmul(a1, c2, dy, u, r, t);
        f29_sub(t, c2, a1);
        f29_normalize(cy, t);             // Y3 (N')
        dx = w1;
        dy = a1;
        tx[k] = cx;
        ty[k] = cy;
        hs[k - 1] = h;
    }
    {  // Z(T_7) = z h_1 ... h_7 as a tree (limbs: z < 2^30, h < 2^29.3, products N)
        f29 p0, p1, p2, p3;
        pmul(p0, p1, z, hs[0], hs[1], hs[2]);
        pmul(p2, p3, hs[3], hs[4], hs[5], hs[6]);
        pmul(p0, p1, p0, p1, p2, p3);
        f29_mul_ilp(z, p0, p1);
    }
    f29 inv;  // 1 / Z(T_last), Montgomery form
    {
        const fe zi = inv_p(f29_canon_plain(z));
        f29_mul_ilp(inv, f29_from_u256(zi), r2);
    }
#pragma unroll 1
    for (int k = kQTab - 1; k >= 1; --k) {  // inv^2 | inv h_k, zi2 inv | x zi2, y zi3
        f29 zi2, nxt, zi3, xa;
        pmul(zi2, nxt, inv, inv, inv, hs[k - 1]);
        pmul(zi3, xa, zi2, inv, tx[k], zi2);
        f29_mul_ilp(ty[k], ty[k], zi3);
        tx[k] = xa;
        inv = nxt;  // 1 / Z(T_{k-1})
    }
}

// build_q_table_pair_m for the W-carrying ladders of the half kernel (p29_dbl_plw): the odd
// multiples of (qxm, qym) on E_c (y^2 = x^3 - 3c^2 x + b c^3; c = 1: the curve itself), stored
// divided by c. ac = c^2 enters DBLU's M = 3 (x^2 - c^2); the inversion is of z c, and 1 / z and
// 1 / c come out of one paired step. Each entry is then X (lam^2 / c) | (Y lam)(lam^2 / c) in three
// paired steps, as before. In: qxm, qym, ac, cc in N or N'. Out: entries in N.
template <class InvP, class Mark, class St, class Ld, class HSt, class HLd>
SBFT_DEV void build_q_table_pair_w(const f29& qxm, const f29& qym, const f29& ac, const f29& cc, bool odd, InvP inv_p,
                                   Mark mark, St st, Ld ld, HSt hst, HLd hld) {
    static_assert(kQTab == 8, "the Z-ratio product tree below is written for 7 ratios");
    auto pmul = [odd](f29& e, f29& d, const f29& a0, const f29& b0, const f29& a1, const f29& b1) {
        f29 o;
        f29_mul_ilp(o, f29_pick(odd, a0, a1), f29_pick(odd, b0, b1));
        f29_unpair(o, e, d);
    };
    const f29 r2 = f29_const(C29_R2);
    f29 dx, dy, cx, cy, z;
    {  // DBLU as build_q_table_pair_m, M = 3 (B - c^2)
        f29 b, e, l, t, m, m2;
        pmul(b, e, qxm, qxm, qym, qym);
        pmul(l, t, e, e, qxm, e);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] <<= 2;  // 4xE < 2^31
        f29_normalize(cx, t);                       // S (N')
#pragma unroll
        for (int i = 0; i < 9; ++i) m.v[i] = 3 * (b.v[i] - ac.v[i]);  // |.| < 3 2^29.2 < 2^30.8
        f29_normalize(m, m);                        // M (N')
        f29_mul_ilp(m2, m, m);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] = m2.v[i] - (cx.v[i] << 1);
        f29_normalize(dx, t);                       // X2 (N')
#pragma unroll
        for (int i = 0; i < 9; ++i) l.v[i] <<= 2;  // 4L < 2^31
        f29_normalize(l, l);
#pragma unroll
        for (int i = 0; i < 9; ++i) l.v[i] <<= 1;  // 8L, |.| < 2^30.2
        f29_normalize(cy, l);                       // 8L (N')
        f29_sub(t, cx, dx);                         // S - X2, |.| < 2^29.3
        f29_mul_ilp(m2, m, t);
        f29_sub(t, m2, cy);
        f29_normalize(dy, t);                       // Y2 (N')
        f29_add(z, qym, qym);                       // Z = 2y
    }
    // The co-Z entries go to their table slots (st: LDS) as they come and the Z ratios to LDS of
    // their own (hst), so nothing is live across the inversion (with all 16 coordinates in
    // registers the safegcd ran at half speed) and the loops stay rolled: unrolled, the table
    // build was ~40 KB of straight-line code that every workgroup streams through the instruction
    // cache once; rolled, a ZADDU or a conversion step is fetched once and run seven times.
#pragma unroll 1
    for (int k = 1; k < kQTab; ++k) {  // ZADDU (curve-independent), as build_q_table_pair_m
        f29 h, r, c, dd, w1, w2, t, u, a1, c2;
        f29_sub(h, dx, cx);
        f29_sub(r, dy, cy);
        pmul(c, dd, h, h, r, r);
        pmul(w1, w2, dx, c, cx, c);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] = dd.v[i] - w1.v[i] - w2.v[i];
        f29_normalize(cx, t);
        f29_sub(u, w1, w2);
        f29_sub(t, w1, cx);
        pmul(a1, c2, dy, u, r, t);
        f29_sub(t, c2, a1);
        f29_normalize(cy, t);
        dx = w1;
        dy = a1;
        st(k, cx, cy);
        hst(k - 1, h);
    }
    {  // Z(T_7) = z h_1 ... h_7 as a tree, then z c
        f29 p0, p1, p2, p3, h0, h1, h2, h3, h4, h5, h6;
        hld(0, h0);
        hld(1, h1);
        hld(2, h2);
        hld(3, h3);
        hld(4, h4);
        hld(5, h5);
        hld(6, h6);
        pmul(p0, p1, z, h0, h1, h2);
        pmul(p2, p3, h3, h4, h5, h6);
        pmul(p0, p1, p0, p1, p2, p3);
        f29_mul_ilp(z, p0, p1);
    }
    f29 zc, ic, lam, kap;
    f29_mul_ilp(zc, z, cc);
    mark(0);  // co-Z chain done
    {
        const fe zi = inv_p(f29_canon_plain(zc));
        f29_mul_ilp(ic, f29_from_u256(zi), r2);  // 1 / (z c)
    }
    mark(1);  // inverted
    pmul(lam, kap, ic, cc, ic, z);               // 1 / z | 1 / c
#pragma unroll 1
    for (int k = kQTab - 1; k >= 1; --k) {  // lam^2 | Y lam, lam^2 / c | lam h_k, X lam^2 / c | Y lam^3 / c
        f29 l2, yl, l2k, nxt, X, Y, hk;
        ld(k, X, Y);
        hld(k - 1, hk);
        pmul(l2, yl, lam, lam, Y, lam);
        pmul(l2k, nxt, l2, kap, lam, hk);
        pmul(X, Y, X, l2k, yl, l2k);
        st(k, X, Y);
        lam = nxt;  // 1 / Z(T_{k-1})
    }
    f29 x0, y0;
    pmul(x0, y0, qxm, kap, qym, kap);  // the base itself, divided by c
    st(0, x0, y0);
}

// build_q_table_pair_w on the four lanes of a quad (the wide half kernel, where lanes 2-3 of a
// quad used to repeat the pair's steps): the same products on the same operands, so the same
// table, in 39 product steps instead of 54. DBLU 3 steps (m^2 beside e^2 | x e); each co-Z
// addition after the first 2 steps, the next addition's H^2 (= (w1 - X3)^2) riding on the spare
// lane of this one's last step; the Z-ratio product tree and z c 4 steps; the conversion 2 steps
// per entry, each entry's last two products in the next entry's steps, the base's in the last.
template <class InvP, class Mark, class St, class Ld, class HSt, class HLd>
SBFT_DEV void build_q_table_quad_w(const f29& qxm, const f29& qym, const f29& ac, const f29& cc, InvP inv_p, Mark mark,
                                   St st, Ld ld, HSt hst, HLd hld) {
    static_assert(kQTab == 8, "the Z-ratio product tree below is written for 7 ratios");
    // lane j of the quad: a_j b_j
    auto qm = [](const f29& a0, const f29& b0, const f29& a1, const f29& b1, const f29& a2, const f29& b2,
                 const f29& a3, const f29& b3) {
        f29 o;
        f29_mul_ilp(o, f29_qsel<kQL3>(f29_qsel<kQL2>(f29_qsel<kQL1>(a0, a1), a2), a3),
                    f29_qsel<kQL3>(f29_qsel<kQL2>(f29_qsel<kQL1>(b0, b1), b2), b3));
        return o;
    };
    auto l0 = [](const f29& o) { return f29_qperm<0x00>(o); };
    auto l1 = [](const f29& o) { return f29_qperm<0x55>(o); };
    auto l2 = [](const f29& o) { return f29_qperm<0xAA>(o); };
    auto l3 = [](const f29& o) { return f29_qperm<0xFF>(o); };
    const f29 r2 = f29_const(C29_R2);
    f29 dx, dy, cx, cy, z;
    {  // DBLU as build_q_table_pair_w: x^2 | y^2, then e^2 | x e | m^2, then m (S - X2)
        f29 o = qm(qxm, qxm, qym, qym, qxm, qxm, qym, qym);
        const f29 b = l0(o), e = l1(o);
        f29 m, t, l, m2;
#pragma unroll
        for (int i = 0; i < 9; ++i) m.v[i] = 3 * (b.v[i] - ac.v[i]);  // |.| < 3 2^29.2 < 2^30.8
        f29_normalize(m, m);                                          // M (N')
        o = qm(e, e, qxm, e, m, m, m, m);
        l = l0(o);
        t = l1(o);
        m2 = l2(o);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] <<= 2;  // 4xE < 2^31
        f29_normalize(cx, t);                       // S (N')
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] = m2.v[i] - (cx.v[i] << 1);
        f29_normalize(dx, t);                       // X2 (N')
#pragma unroll
        for (int i = 0; i < 9; ++i) l.v[i] <<= 2;  // 4L < 2^31
        f29_normalize(l, l);
#pragma unroll
        for (int i = 0; i < 9; ++i) l.v[i] <<= 1;  // 8L, |.| < 2^30.2
        f29_normalize(cy, l);                       // 8L (N')
        f29_sub(t, cx, dx);                         // S - X2, |.| < 2^29.3
        f29_mul_ilp(m2, m, t);
        f29_sub(t, m2, cy);
        f29_normalize(dy, t);                       // Y2 (N')
        f29_add(z, qym, qym);                       // Z = 2y
    }
    f29 h, c;  // this addition's H = dx - cx and H^2
    f29_sub(h, dx, cx);
    f29_mul_ilp(c, h, h);
#pragma unroll 1
    for (int k = 1; k < kQTab; ++k) {  // ZADDU: R^2 | W1 | W2, then A1 | C2 | the next H^2
        f29 r, w1, w2, dd, t, u;
        f29_sub(r, dy, cy);
        f29 o = qm(r, r, dx, c, cx, c, r, r);
        dd = l0(o);
        w1 = l1(o);
        w2 = l2(o);
#pragma unroll
        for (int i = 0; i < 9; ++i) t.v[i] = dd.v[i] - w1.v[i] - w2.v[i];
        f29_normalize(cx, t);  // X3 (N')
        f29_sub(u, w1, w2);
        f29_sub(t, w1, cx);    // the next H (= w1 - X3)
        o = qm(dy, u, r, t, t, t, t, t);
        const f29 a1 = l0(o), c2 = l1(o);
        c = l2(o);
        f29_sub(u, c2, a1);
        f29_normalize(cy, u);  // Y3 (N')
        dx = w1;
        dy = a1;
        st(k, cx, cy);
        hst(k - 1, h);
        h = t;
    }
    f29 zt, zc;
    {  // Z(T_7) = z h_1 ... h_7 and z c as a tree
        f29 h0, h1, h2, h3, h4, h5, h6;
        hld(0, h0);
        hld(1, h1);
        hld(2, h2);
        hld(3, h3);
        hld(4, h4);
        hld(5, h5);
        hld(6, h6);
        f29 o = qm(z, h0, h1, h2, h3, h4, h5, h6);
        const f29 p0 = l0(o), p1 = l1(o), p2 = l2(o), p3 = l3(o);
        o = qm(p0, p1, p2, p3, p0, p1, p2, p3);
        const f29 q0 = l0(o), q1 = l1(o);
        o = qm(q0, q1, q1, cc, q0, q1, q1, cc);
        zt = l0(o);
        f29_mul_ilp(zc, q0, l1(o));
    }
    mark(0);  // co-Z chain done
    f29 ic, lam, kap;
    {
        const fe zi = inv_p(f29_canon_plain(zc));
        f29_mul_ilp(ic, f29_from_u256(zi), r2);  // 1 / (z c)
    }
    mark(1);  // inverted
    {
        const f29 o = qm(ic, cc, ic, zt, ic, cc, ic, zt);
        lam = l0(o);  // 1 / z
        kap = l1(o);  // 1 / c
    }
    // entry k: lam^2 | Y lam | lam h_k (the next lam) | (entry k+1's X lam^2 / c), then lam^2 / c |
    // (entry k+1's Y lam^3 / c)
    f29 px = kap, pyl = kap, pl2k = kap;  // entry k+1's X, Y lam, lam^2 / c (none before entry 7)
#pragma unroll 1
    for (int k = kQTab - 1; k >= 1; --k) {
        f29 X, Y, hk;
        ld(k, X, Y);
        hld(k - 1, hk);
        f29 o = qm(lam, lam, Y, lam, lam, hk, px, pl2k);
        const f29 l2v = l0(o), yl = l1(o), nxt = l2(o), xo = l3(o);
        o = qm(l2v, kap, pyl, pl2k, l2v, kap, pyl, pl2k);
        if (k < kQTab - 1) st(k + 1, xo, l1(o));
        pl2k = l0(o);
        px = X;
        pyl = yl;
        lam = nxt;  // 1 / Z(T_{k-1})
    }
    {  // entry 1's products and the base itself, divided by c
        const f29 o = qm(px, pl2k, pyl, pl2k, qxm, kap, qym, kap);
        st(1, l0(o), l1(o));
        st(0, l2(o), l3(o));
    }
}

// 2-3. w = s^-1 of tuple t from the launch-wide Montgomery trick (p256_sinv_* kernels: 1,024
// tuples per scan group), then u1 = e w, u2 = r w, recoded for the signed-odd ladders: an even
// u becomes n - u with the base negated ((n-u)(-P) = uP); u == 0 becomes n, whose ladder
// cancels to infinity. Invalid lanes get u1 = u2 = 1.
SBFT_DEV fe sinv_from_ws(const sinv_ws& ws, uint32_t t, uint32_t n, bool active) {
    fe w;
    const uint32_t pos = t & (SBFT_SINV_GROUP - 1);
    const fe kb = ld_fe(ws.kb + 2ull * (t >> SBFT_SINV_GROUP_LOG2));
    const fe one = fe_const(C_ONEN);
    const fe pre = (pos > 0 && active) ? ld_fe(ws.pre + 2ull * (t - 1)) : one;
    const fe suf = (pos < SBFT_SINV_GROUP - 1 && active && t + 1 < n) ? ld_fe(ws.suf + 2ull * (t + 1)) : one;
    fn_mul(w, kb, pre);
    fn_mul(w, w, suf);  // s^-1 * R (garbage for lanes whose s is invalid: masked by `valid`)
    return w;
}
// w = s^-1 R mod n (Montgomery form)
SBFT_DEV void verify_scalars(const fe& w, bool valid, const fe& e_raw, const fe& r, fe& u1, fe& u2, bool& neg1,
                             bool& neg2) {
    fe e;
    fn_canon(e, e_raw);
    fn_mul(u1, e, w);  // e*s^-1 (plain)
    fn_mul(u2, r, w);  // r*s^-1 (plain)
    fn_canon(u1, u1);
    fn_canon(u2, u2);
    if (!valid) {
        u1 = fe_zero();
        u1.v[0] = 1;
        u2 = u1;
    }
    neg1 = (u1.v[0] & 1u) == 0;
    neg2 = (u2.v[0] & 1u) == 0;
    fe t1, t2;
    u64 b1 = 0, b2 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u64 d1 = (u64)P256_N[k] - u1.v[k] - b1;
        const u64 d2 = (u64)P256_N[k] - u2.v[k] - b2;
        t1.v[k] = lo32(d1);
        t2.v[k] = lo32(d2);
        b1 = d1 >> 63;
        b2 = d2 >> 63;
    }
    fe_sel(u1, neg1, t1);
    fe_sel(u2, neg2, t2);
}

// Radix-2^w signed-odd digit i of u2 (u2 = sum_{i<K} d_i 2^(w i) + 2^(w K),
// d_i = 2*((u2 >> (w i + 1)) & (2^w - 1)) - (2^w - 1), odd and nonzero).
template <int W = kQWin>
SBFT_DEV int q_digit(const fe& k2, int i) {
    constexpr int tab = 1 << (W - 1);
    const int b = W * i + 1, lw = b >> 5;
    const u32 lo = k2.v[lw], hi = lw < 7 ? k2.v[lw + 1] : 0u;
    return 2 * (int)(__builtin_amdgcn_alignbit(hi, lo, b & 31) & (2 * tab - 1)) - (2 * tab - 1);
}

// q_digit with the two words picked by selects instead of a runtime index into k2: a runtime
// index makes k2 an alloca, which LLVM promotes to LDS (8 KB of the half kernel's workgroup, read
// back every digit); its absence measured 13 us less per 10k-tuple launch (profiles/
// r05ad_nolds_ab.txt: the table build ends ~10 us earlier). 16 selects per digit.
#ifndef SBFT_HALF_ENTRY_EARLY
#define SBFT_HALF_ENTRY_EARLY 1  // the half kernel's ladder reads a digit's entry before its doublings
#endif
#ifndef SBFT_PAIR_DIGIT_SEL
#define SBFT_PAIR_DIGIT_SEL 1  // the pair kernel's digits by selects as well
#endif
template <int W = kQWin>
SBFT_DEV int q_digit_sel(const fe& k2, int i) {
    constexpr int tab = 1 << (W - 1);
    const int b = W * i + 1, lw = b >> 5;
    u32 lo = 0u, hi = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        lo = lw == j ? k2.v[j] : lo;
        hi = lw + 1 == j ? k2.v[j] : hi;
    }
    return 2 * (int)(__builtin_amdgcn_alignbit(hi, lo, b & 31) & (2 * tab - 1)) - (2 * tab - 1);
}

// u1*G by the fixed-base comb in HBM (no doublings): u1 = sum_{i<K} d_i 2^(W i) + 2^(W K) with
// d_i = 2*((u1 >> (W i + 1)) & (2^W - 1)) - (2^W - 1) (odd, nonzero), i.e. K mixed additions of
// table[i][(|d_i| - 1) / 2] = |d_i| 2^(W i) G plus one of table[K][0] = 2^(W K) G.
// The next entry's five 16-B loads are issued before the current addition. add(acc, x, y) is
// the mixed addition of the calling kernel.
// PINGPONG (latency kernel): two entry buffers in fixed registers, loop unrolled by two, so
// that the next entry's loads are never waited on to shuffle registers (at one wave per SIMD
// the rotated one-buffer loop exposed an HBM round trip per addition).
// fix(reload) runs after every addition (add_aff_fix: the comb's points are added on top of
// u2 Q, so with a crafted Q any of them can meet acc == +-entry); reload(x, y) reloads the entry
// just added.
template <bool PINGPONG = false, class Acc, class AddAff, class Fix>
SBFT_DEV void comb_add_u1g(Acc& acc, const fe& u1, bool neg1, const uint4* __restrict__ gcomb, AddAff add,
                           Fix fix) {
    constexpr int T = kGK + 1;  // entries summed
    fe k1 = u1;
    uint4 cur[5], nxt[5];
    int dneg_cur = 0, dneg_nxt = 0;
    auto entry_xy = [neg1](const uint4* e, int dn, f29& gx, f29& gy) {
        const u32* w = reinterpret_cast<const u32*>(e);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            gx.v[k] = w[k];
            gy.v[k] = w[10 + k];
        }
        if ((dn != 0) != neg1) f29_neg(gy, gy);
    };
    // digit i of u1 -> (entry pointer, negative?)
    auto digit = [&](int i, const uint4*& ptr, int& neg) {
        if (i < kGK) {
            const u32 bits = (k1.v[0] >> 1) & kGMask;  // bits W i + 1 .. W i + W (k1 shifted)
            const int d = 2 * (int)bits - (int)kGMask;
            const u32 j = (u32)((d < 0 ? -d : d) >> 1);
            ptr = gcomb + ((size_t)i * SBFT_GCOMB_ENTRIES + j) * 5;
            neg = d < 0;
            // k1 >>= W for the next window
#pragma unroll
            for (int k = 0; k < 7; ++k) k1.v[k] = __builtin_amdgcn_alignbit(k1.v[k + 1], k1.v[k], kGWin);
            k1.v[7] >>= kGWin;
        } else {
            ptr = gcomb + (size_t)kGK * SBFT_GCOMB_ENTRIES * 5;
            neg = 0;
        }
    };
    const uint4* ptr;
    if (PINGPONG) {
        const uint4 *pc = nullptr, *pn = nullptr;  // the buffers' entry addresses (for the reload)
        auto add_entry = [&](const uint4 (&en)[5], int dn, const uint4* src) {
            f29 gx, gy;
            entry_xy(en, dn, gx, gy);
            add(acc, gx, gy);
            fix([&](f29& x, f29& y) { entry_xy(src, dn, x, y); });
        };
        digit(0, ptr, dneg_cur);
        pc = ptr;
#pragma unroll
        for (int k = 0; k < 5; ++k) cur[k] = ptr[k];
        int i = 0;
#pragma unroll 1
        for (; i + 1 < T; i += 2) {
            digit(i + 1, ptr, dneg_nxt);
            pn = ptr;
#pragma unroll
            for (int k = 0; k < 5; ++k) nxt[k] = ptr[k];
            add_entry(cur, dneg_cur, pc);
            if (i + 2 < T) {
                digit(i + 2, ptr, dneg_cur);
                pc = ptr;
#pragma unroll
                for (int k = 0; k < 5; ++k) cur[k] = ptr[k];
            }
            add_entry(nxt, dneg_nxt, pn);
        }
        if (i < T) add_entry(cur, dneg_cur, pc);  // odd entry count: the last one
        return;
    }
    const uint4 *pc = nullptr, *pn = nullptr;
    digit(0, ptr, dneg_nxt);
    pn = ptr;
#pragma unroll
    for (int k = 0; k < 5; ++k) nxt[k] = ptr[k];
#pragma unroll 1
    for (int i = 0; i < T; ++i) {
#pragma unroll
        for (int k = 0; k < 5; ++k) cur[k] = nxt[k];
        dneg_cur = dneg_nxt;
        pc = pn;
        if (i + 1 < T) {
            digit(i + 1, ptr, dneg_nxt);
            pn = ptr;
#pragma unroll
            for (int k = 0; k < 5; ++k) nxt[k] = ptr[k];
        }
        f29 gx, gy;
        entry_xy(cur, dneg_cur, gx, gy);
        add(acc, gx, gy);
        const int dn = dneg_cur;
        fix([&](f29& x, f29& y) { entry_xy(pc, dn, x, y); });
    }
}

// 5. verify_final (p256_f29.hpp): Z == 0 flags an exceptional tuple, else x(R) == r projectively.

// Throughput kernel: one verify per lane, 256-thread workgroups (four per 1,024-tuple s^-1 group).
__global__ __launch_bounds__(256, SBFT_VERIFY_WAVES) void p256_verify_kernel(const uint8_t* __restrict__ digest,
                                                          const uint8_t* __restrict__ rr,
                                                          const uint8_t* __restrict__ ss,
                                                          const uint8_t* __restrict__ qxx,
                                                          const uint8_t* __restrict__ qyy,
                                                          uint8_t* __restrict__ ok, uint32_t n,
                                                          uint32_t* __restrict__ work, sinv_ws ws,
                                                          const uint4* __restrict__ gcomb, int spread) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    inv::stage_divstep_table(dtab);  // ends with a barrier

    // this lane's tuple: 256 per workgroup, or (spread) the grid is a whole number of resident
    // rounds and workgroup b takes tuples [b n / G, (b + 1) n / G) (sbft_launch_p256_verify)
    uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, end = n;
    if (spread) {
        const uint32_t lo = (uint32_t)((uint64_t)blockIdx.x * n / gridDim.x);
        end = (uint32_t)((uint64_t)(blockIdx.x + 1) * n / gridDim.x);
        gid = lo + threadIdx.x;
        if (lo + (threadIdx.x & ~63u) >= end) return;  // a wave with no tuple (no barrier follows)
    }
    const bool active = gid < end;
    const uint32_t idx = active ? gid : (end - 1);

    const fe e_raw = load_be32(digest + 32ull * idx);
    const fe r = load_be32(rr + 32ull * idx);
    const fe s = load_be32(ss + 32ull * idx);
    const fe qx = load_be32(qxx + 32ull * idx);
    const fe qy = load_be32(qyy + 32ull * idx);
    const bool valid = verify_inputs_valid(r, s, qx, qy);

    f29 tx[kTTab], ty[kTTab];  // affine odd multiples (scratch)
    build_q_table(tx, ty, qx, qy, valid, [&](const fe& zp) {
        fe zi;
        inv::inv_mod_p(zi.v, zp.v, dtab);
        return zi;
    });
#if SBFT_QTAB_GLOBAL
    // the ladder reads the table from this lane's own contiguous 80 B x 2^(w-1) (5 x 16 B per entry) in
    // the workspace: a digit's entry is 72 contiguous bytes (two 64-B segments), where the
    // lane-interleaved scratch layout spreads it over 18 rows shared by the wave's 8 entries
    uint4* const qg = ws.qtab + (size_t)idx * (kTTab * 5);
    if (active) {
#pragma unroll
        for (int m = 0; m < kTTab; ++m) {
            uint4 e[5];
            pack_entry(tx[m], ty[m], e);
#pragma unroll
            for (int k = 0; k < 5; ++k) qg[m * 5 + k] = e[k];
        }
    }
#endif
    fe u1, u2;
    bool neg1, neg2;
    verify_scalars(sinv_from_ws(ws, gid, n, active), valid, e_raw, r, u1, u2, neg1, neg2);

    jp29 acc;  // reloaded from scratch: keeps q out of registers during the setup
    acc.x = tx[0];
    acc.y = ty[0];
    acc.z = f29_const(C29_ONE);
    if (neg2) f29_neg(acc.y, acc.y);
    // the accumulator starts at +-Q (the 2^(wK) term of u2). With odd digits the partial scalar
    // m of the ladder is odd and 16 m > |d| until the last digit, where 16 m = n + d is possible
    // (u2 = n - 2|d|, P + P): only the last addition can be exceptional (add_aff_fix).
    const fe k2 = u2;
    bool inf = false;  // acc is the point at infinity (add_aff_fix)
    auto dbl1 = [](jp29& p) { p29_dbl(p, p); };
    auto entry = [&](int i, f29& x2, f29& y2) __attribute__((always_inline)) {
        const int d2 = q_digit<kTWin>(k2, i);
#ifdef SBFT_TABLE_PROBE  // measurement only (wrong verdicts): the ladder reads one fixed entry
        const int m2 = 0;
#else
        const int m2 = (d2 < 0 ? -d2 : d2) >> 1;
#endif
#if SBFT_QTAB_GLOBAL
        uint4 e[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) e[k] = qg[m2 * 5 + k];
        const u32* w = reinterpret_cast<const u32*>(e);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            x2.v[k] = w[k];
            y2.v[k] = w[10 + k];
        }
#else
        x2 = tx[m2];
        y2 = ty[m2];
#endif
        if ((d2 < 0) != neg2) f29_neg(y2, y2);
    };
    auto digit_step = [&](int i) __attribute__((always_inline)) {
#pragma unroll kDblUnroll
        for (int d = 0; d < kTWin; ++d) p29_dbl(acc, acc);
        f29 x2, y2;
        entry(i, x2, y2);
        p29_add_aff_lean(acc, x2, y2);
    };
#pragma unroll 1
    for (int i = kTDigits - 1; i >= 1; --i) digit_step(i);
    digit_step(0);  // the last digit, peeled: the fix's state stays out of the loop
    add_aff_fix(acc, inf, dbl1, [&](f29& x2, f29& y2) { entry(0, x2, y2); });
    comb_add_u1g(acc, u1, neg1, gcomb, [](jp29& a, const f29& x, const f29& y) { p29_add_aff_lean(a, x, y); },
                 [&](auto reload) { add_aff_fix(acc, inf, dbl1, reload); });

    bool exc;
    bool accept = verify_final(acc, load_be32(rr + 32ull * idx), exc);  // r reloaded
    if (inf) {  // R = infinity: rejected (Go's Verify), not an exceptional tuple
        accept = false;
        exc = false;
    }
    if (active) {
        if (exc && valid) {
            const uint32_t slot = atomicAdd(work, 1u);
            work[1 + slot] = gid;
        } else {
            ok[gid] = (valid && accept) ? 1 : 0;
        }
    }
}

// Latency kernel for small batches (sbft_launch_p256_verify with lanes = 2). A batch of a few
// thousand tuples gives each busy SIMD one wave, so the launch takes one wave's instruction
// stream; this kernel shortens that stream at the price of more lanes: one verify on two
// adjacent lanes, the doublings and mixed additions split between them (p29_dbl_pair,
// p29_add_aff_pair); u1*G by the comb after the ladder. (Round 3's four-lane form, the comb on
// lanes 2-3 of a quad, measured no faster and is gone; the four-lane kernel now is
// p256_verify_half_kernel.) Setup (checks, Q table, scalars) and the final comparison run
// redundantly on both lanes of a tuple. The Q table lives in LDS (one copy per tuple). One wavefront per workgroup spreads a
// small batch over as many CUs as possible.
//
// FRAMED (sbft_launch_p256_verify_framed): the tuples come straight from a framed payload, and
// each workgroup has a second wavefront that hashes the tuples' messages (one lane per message)
// while the first builds its Q tables; the digests meet the scalars in LDS at the table
// barrier. r, s and Q are read from the payload in place (unaligned). No gather or hash
// kernel runs in front: the batch's serial hashing hides under the table build. A tuple that
// needs the exact fixup has its five fields written to the SoA rows the fixup kernel reads.
struct FramedIn {
    const uint8_t* blob;
    const uint64_t* off;
    const uint32_t* len;
    int32_t sig_rel, pub_rel;
    uint8_t *dig, *r, *s, *qx, *qy;  // SoA rows for the fixup kernel (flagged tuples only)
    uint32_t* flagged;  // non-null: set to 1 (mapped host memory) when a tuple is flagged, and the
                        // caller launches the fixup only then (sbft_launch_p256_verify_framed)
};

// 32 big-endian bytes at any byte address -> 8 little-endian limbs (reads up to 3 bytes past)
SBFT_DEV fe load_be32_any(const uint8_t* p) {
    typedef const __attribute__((address_space(1))) uint32_t gu32;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    gu32* base = (gu32*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t raw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) raw[i] = base[i];
    fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[7 - i] = __builtin_bswap32(__builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh));
    return r;
}

// SBFT_PAIR_COMB_WAVE (FRAMED pair kernel): u1*G on a wavefront of its own. The ladder needs only
// u2 = r s^-1; the digest, and with it u1, only the comb. The workgroup is four wavefronts: two
// verify wavefronts (64 tuples, two lanes each), the hash wavefront (one lane per tuple) and the
// comb wavefront (one lane per tuple), which inverts s itself, reads the digests at the table
// barrier, sums the K + 1 comb entries (add_aff_fix after each: partial sums can meet +-entry,
// u1 = 0 ends at infinity) and leaves the sum in LDS; each verify wavefront, its ladder done, adds
// it with one Jacobian addition and the same in-place case split (u1 G = u2 Q: a doubling;
// = -u2 Q: infinity). The 13 comb additions leave the verify wavefronts' stream. With 64 tuples
// per workgroup a 10k batch is 157 workgroups, at most one per CU, so every wavefront has a SIMD
// of its own (three wavefronts of 32 tuples put six on the CUs holding two workgroups, and the
// comb on the hash wavefront shares its SIMD's time: both were slower,
// profiles/r03cw_comb_wave_lat.txt).
#ifndef SBFT_PAIR_COMB_WAVE
#define SBFT_PAIR_COMB_WAVE 1
#endif
template <int LPT, bool FRAMED>
constexpr int small_kernel_threads() {
    return !FRAMED ? 64 : (LPT == 2 && SBFT_PAIR_COMB_WAVE) ? 256 : 128;
}
// tuples per workgroup
template <int LPT, bool FRAMED>
constexpr int small_kernel_tuples() {
    return (FRAMED && LPT == 2 && SBFT_PAIR_COMB_WAVE) ? 64 : 64 / LPT;
}

template <int LPT, bool FRAMED = false>
__global__ __launch_bounds__((small_kernel_threads<LPT, FRAMED>())) void p256_verify_small_kernel(const uint8_t* __restrict__ digest,
                                                                             const uint8_t* __restrict__ rr,
                                                                             const uint8_t* __restrict__ ss,
                                                                             const uint8_t* __restrict__ qxx,
                                                                             const uint8_t* __restrict__ qyy,
                                                                             uint8_t* __restrict__ ok, uint32_t n,
                                                                             uint32_t* __restrict__ work,
                                                                             const uint4* __restrict__ gcomb,
                                                                             FramedIn fr) {
    static_assert(LPT == 2, "two lanes per tuple");
    constexpr bool kCombWave = FRAMED && SBFT_PAIR_COMB_WAVE;
    constexpr int kTuples = small_kernel_tuples<LPT, FRAMED>();  // tuples per workgroup
    constexpr unsigned kVerifyThreads = kTuples * LPT;          // the verify wavefront(s)
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    // [entry][x limbs 0..8, y limbs 0..8][tuple]: the lanes of a tuple read the same word, the
    // tuples of the wave consecutive words
    __shared__ u32 qtab[kQTab * 18 * kTuples];
    __shared__ u32 edig[FRAMED ? 8 * kTuples : 1];  // FRAMED: the hash wave's digests [word][tuple]
    __shared__ u32 gsum[kCombWave ? 28 * kTuples : 1];  // the comb wave's u1 G: [x, y, z limbs, inf][tuple]
    inv::stage_divstep_table(dtab);  // ends with a barrier

    if constexpr (FRAMED) {
        if (threadIdx.x >= kVerifyThreads && threadIdx.x < kVerifyThreads + 64) {  // the hash wavefront
            const uint32_t lane = threadIdx.x - kVerifyThreads, th = blockIdx.x * kTuples + lane;
            if (lane < (uint32_t)kTuples && th < n) {
                const uint8_t* msg = fr.blob + fr.off[th];
                const uint32_t L = fr.len[th], nb = sha256_nblocks(L);
                uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
                uint32_t w[16];
                for (uint32_t b = 0; b < nb; ++b) {
                    sha256_block_at(msg, L, b, w);
                    compress(h, w);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) edig[k * kTuples + lane] = h[k];
            }
            // the verify wavefront's barriers: the Q table's and the comb wave's hand-over
            __syncthreads();
            if constexpr (kCombWave) __syncthreads();
            return;
        }
    }

    if constexpr (kCombWave) {
        if (threadIdx.x >= kVerifyThreads + 64) {  // the comb wavefront (wave-uniform branch)
            const uint32_t lane = threadIdx.x - kVerifyThreads - 64;
            const uint32_t slot = lane < (uint32_t)kTuples ? lane : 0u;
            const uint32_t tc = blockIdx.x * kTuples + slot;
            const uint32_t ic = tc < n ? tc : n - 1;
            const uint8_t* end = fr.blob + fr.off[ic] + fr.len[ic];
            const fe rc = load_be32_any(end + fr.sig_rel), sc = load_be32_any(end + fr.sig_rel + 32);
            const fe qxc = load_be32_any(end + fr.pub_rel), qyc = load_be32_any(end + fr.pub_rel + 32);
            const bool vc = verify_inputs_valid(rc, sc, qxc, qyc);
            fe x = fe_zero(), si;
            x.v[0] = 1;
            if (vc) x = sc;
            inv::inv_mod(si.v, x.v, dtab, false);  // plain s^-1 mod n (1 for an invalid s)
            __syncthreads();  // the table barrier: the hash wavefront's digests are in edig
            fe ec, w, u1c, u2c;
            bool n1, n2;
#pragma unroll
            for (int k = 0; k < 8; ++k) ec.v[7 - k] = edig[k * kTuples + slot];
            fn_mul(w, si, fe_const(C_R2N));  // s^-1 R
            verify_scalars(w, vc, ec, rc, u1c, u2c, n1, n2);
            jp29 g;
            g.x = g.y = g.z = f29_const(C29_ONE);
            bool ginf = true;  // the first addition returns its addend (add_aff_fix)
            comb_add_u1g(g, u1c, n1, gcomb,
                         [](jp29& a, const f29& x2, const f29& y2) { p29_add_aff_lean(a, x2, y2); },
                         [&](auto reload) { add_aff_fix(g, ginf, [](jp29& p) { p29_dbl(p, p); }, reload); });
            if (lane < (uint32_t)kTuples) {
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    gsum[k * kTuples + lane] = g.x.v[k];
                    gsum[(9 + k) * kTuples + lane] = g.y.v[k];
                    gsum[(18 + k) * kTuples + lane] = g.z.v[k];
                }
                gsum[27 * kTuples + lane] = ginf ? 1u : 0u;
            }
            __syncthreads();  // hand-over to the verify wavefronts
            return;
        }
    }
    const int pr = threadIdx.x / LPT;
    const bool odd = (threadIdx.x & 1) != 0;
    const uint32_t t = blockIdx.x * kTuples + pr;
    const bool active = t < n;
    const uint32_t idx = active ? t : (n - 1);

    fe e_raw, r, s, qx, qy;
    if constexpr (FRAMED) {
        const uint8_t* end = fr.blob + fr.off[idx] + fr.len[idx];
        r = load_be32_any(end + fr.sig_rel);
        s = load_be32_any(end + fr.sig_rel + 32);
        qx = load_be32_any(end + fr.pub_rel);
        qy = load_be32_any(end + fr.pub_rel + 32);
    } else {
        e_raw = load_be32(digest + 32ull * idx);
        r = load_be32(rr + 32ull * idx);
        s = load_be32(ss + 32ull * idx);
        qx = load_be32(qxx + 32ull * idx);
        qy = load_be32(qyy + 32ull * idx);
    }
    const bool valid = verify_inputs_valid(r, s, qx, qy);
    // The table's one inversion mod p (even lane) and s^-1 mod n (odd lane) run as one safegcd
    // instruction stream; no launch-wide s^-1 batching kernels in front of this one.
    fe s_inv;  // plain s^-1 mod n (1 for an invalid s: masked by `valid`)
    {
        f29 tx[kQTab], ty[kQTab];
#ifdef SBFT_PAIR_NO_TABLE  // development: phase timing only (wrong verdicts)
        s_inv = s;
#pragma unroll
        for (int m = 0; m < kQTab; ++m) {
            tx[m] = f29_from_u256(qx);
            ty[m] = f29_from_u256(qy);
        }
        if (0)
#endif
        build_q_table_pair(tx, ty, qx, qy, valid, odd, [&](const fe& zp) {
            fe x = zp, y, zi;
            if (odd) {
                x = fe_zero();
                x.v[0] = 1;
                if (valid) x = s;
            }
            inv::inv_mod(y.v, x.v, dtab, !odd);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                zi.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)y.v[k], 0xA0, 0xF, 0xF, false);     // even lane's
                s_inv.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)y.v[k], 0xF5, 0xF, 0xF, false);  // odd lane's
            }
            return zi;
        });
#pragma unroll
        for (int m = 0; m < kQTab; ++m)
#pragma unroll
            for (int k = 0; k < 9; ++k) {  // all lanes of the tuple store the same words
                qtab[(m * 18 + k) * kTuples + pr] = tx[m].v[k];
                qtab[(m * 18 + 9 + k) * kTuples + pr] = ty[m].v[k];
            }
    }
    __syncthreads();
    if constexpr (FRAMED) {
#pragma unroll
        for (int k = 0; k < 8; ++k) e_raw.v[7 - k] = edig[k * kTuples + pr];
    }
    fe u1, u2;
    bool neg1, neg2;
    {
        fe w;
        fn_mul(w, s_inv, fe_const(C_R2N));  // s^-1 R
        verify_scalars(w, valid, e_raw, r, u1, u2, neg1, neg2);
    }

    // comb entry i of u1 (see comb_add_u1g): |d_i| 2^(W i) G for i < K, 2^(W K) G for i = K
    auto comb_entry = [&](int i, uint4 (&en)[5], bool& dneg) {
        const uint4* ptr;
        if (i < kGK) {
            const int b = kGWin * i + 1, lw = b >> 5;
            const u32 lo = u1.v[lw], hi = lw < 7 ? u1.v[lw + 1] : 0u;
            const int d = 2 * (int)(__builtin_amdgcn_alignbit(hi, lo, b & 31) & kGMask) - (int)kGMask;
            ptr = gcomb + ((size_t)i * SBFT_GCOMB_ENTRIES + (u32)((d < 0 ? -d : d) >> 1)) * 5;
            dneg = d < 0;
        } else {
            ptr = gcomb + (size_t)kGK * SBFT_GCOMB_ENTRIES * 5;
            dneg = false;
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) en[k] = ptr[k];
    };
    auto entry_point = [&](const uint4 (&en)[5], bool dneg, f29& x, f29& y) {
        const u32* w = reinterpret_cast<const u32*>(en);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            x.v[k] = w[k];
            y.v[k] = w[10 + k];
        }
        if (dneg != neg1) f29_neg(y, y);
    };

    jp29 acc;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        acc.x.v[k] = qtab[k * kTuples + pr];
        acc.y.v[k] = qtab[(9 + k) * kTuples + pr];
    }
    acc.z = f29_const(C29_ONE);
    if (neg2) f29_neg(acc.y, acc.y);
    const fe k2 = u2;
    bool inf = false;  // acc is the point at infinity (add_aff_fix; the pair form only)
    auto dblp = [odd](jp29& p) { p29_dbl_pair(p, p, odd); };
#ifndef SBFT_PAIR_LADDER_DIGITS  // development: time the phases (tools/pair_probe.py --no-check)
#define SBFT_PAIR_LADDER_DIGITS kQDigits
#endif
    auto qentry = [&](int i, f29& x, f29& y) {
        const int d2 = SBFT_PAIR_DIGIT_SEL ? q_digit_sel(k2, i) : q_digit(k2, i);  // (see q_digit_sel)
        const int m2 = (d2 < 0 ? -d2 : d2) >> 1;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            x.v[k] = qtab[(m2 * 18 + k) * kTuples + pr];
            y.v[k] = qtab[(m2 * 18 + 9 + k) * kTuples + pr];
        }
        if ((d2 < 0) != neg2) f29_neg(y, y);
    };
    if (SBFT_PAIR_LANE_LOCAL && SBFT_PAIR_LADDER_DIGITS > 0) {
        // the ladder in the lane-local form; the last digit's addition (the only one that can
        // be exceptional) in the both-lanes form, for add_aff_fix
        pl29 q = pl29_from(acc, odd);
#pragma unroll 1
        for (int i = SBFT_PAIR_LADDER_DIGITS - 1; i >= 1; --i) {
#pragma unroll
            for (int d = 0; d < kQWin; ++d) p29_dbl_pl(q, odd);
            f29 x2, y2;
            qentry(i, x2, y2);
            p29_add_aff_pl(q, x2, y2);
        }
#pragma unroll
        for (int d = 0; d < kQWin; ++d) p29_dbl_pl(q, odd);
        pl29_to(acc, q);
        f29 x2, y2;
        qentry(0, x2, y2);
        p29_add_aff_pair(acc, x2, y2, odd);
        add_aff_fix(acc, inf, dblp, [&](f29& x, f29& y) { qentry(0, x, y); });
    } else {
#pragma unroll 1
        for (int i = SBFT_PAIR_LADDER_DIGITS - 1; i >= 0; --i) {
#pragma unroll
            for (int d = 0; d < kQWin; ++d) p29_dbl_pair(acc, acc, odd);
            f29 x2, y2;
            qentry(i, x2, y2);
            p29_add_aff_pair(acc, x2, y2, odd);
            if (i == 0) add_aff_fix(acc, inf, dblp, [&](f29& x, f29& y) { qentry(0, x, y); });
        }
    }
    if constexpr (kCombWave) {
        __syncthreads();  // the comb wavefront's sum is in gsum
        jp29 g;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            g.x.v[k] = gsum[k * kTuples + pr];
            g.y.v[k] = gsum[(9 + k) * kTuples + pr];
            g.z.v[k] = gsum[(18 + k) * kTuples + pr];
        }
        const bool ginf = gsum[27 * kTuples + pr] != 0;
        const jp29 a0 = acc;
        p29_add_jac_lean(acc, g);
        // H == 0 (Z3 = Z1 Z2 H = 0): X3 = r^2, so r == 0 (u1 G == u2 Q: the result is a doubling)
        // iff X3 == 0, else u1 G == -u2 Q and the result is infinity
        const bool hz = !inf && !ginf && f29_zero_mod_p(acc.z);
        if (__builtin_expect(__any(hz || inf || ginf), 0)) {
            const bool twice = hz && f29_zero_mod_p_any(acc.x);
            jp29 d = a0;
            dblp(d);
            if (twice) acc = d;
            if (ginf) acc = a0;
            if (inf) acc = g;
            inf = (hz && !twice) || (inf && ginf);
        }
    } else {
#ifndef SBFT_PAIR_NO_COMB
        if (SBFT_PAIR_LANE_LOCAL) {
            // lane-local comb additions; the exceptional-case repair (a wave-uniform branch that
            // only runs when a lane of the wave needs it) converts to the both-lanes form
            pl29 q = pl29_from(acc, odd);
            comb_add_u1g<true>(q, u1, neg1, gcomb, [](pl29& a, const f29& x, const f29& y) { p29_add_aff_pl(a, x, y); },
                               [&](auto reload) {
                                   const bool hz = !inf && f29_zero_mod_p(f29_sel_pair(q.zy, q.zo));
                                   if (__builtin_expect(__any(hz || inf), 0)) {
                                       pl29_to(acc, q);
                                       add_aff_fix(acc, inf, dblp, reload);
                                       q = pl29_from(acc, odd);
                                   }
                               });
            pl29_to(acc, q);
        } else {
            comb_add_u1g<true>(acc, u1, neg1, gcomb,
                               [odd](jp29& a, const f29& x, const f29& y) { p29_add_aff_pair(a, x, y, odd); },
                               [&](auto reload) { add_aff_fix(acc, inf, dblp, reload); });
        }
#endif
    }

    bool exc;
    bool accept = verify_final(acc, r, exc);
    if (inf) {  // R = infinity: rejected, not an exceptional tuple
        accept = false;
        exc = false;
    }
    if (active && (threadIdx.x % LPT) == 0) {
        if (exc && valid) {
            if constexpr (FRAMED) {  // the fixup kernel's inputs
                store_be32(fr.dig + 32ull * t, e_raw);
                store_be32(fr.r + 32ull * t, r);
                store_be32(fr.s + 32ull * t, s);
                store_be32(fr.qx + 32ull * t, qx);
                store_be32(fr.qy + 32ull * t, qy);
            }
            const uint32_t slot = atomicAdd(work, 1u);
            work[1 + slot] = t;
            if constexpr (FRAMED) {
                if (fr.flagged) *(volatile uint32_t*)fr.flagged = 1u;
            }
        } else {
            ok[t] = (valid && accept) ? 1 : 0;
        }
    }
}
// ---- half-size scalars: two 128-bit ladders side by side (p256_verify_half_kernel) ----
// The latency kernels' time is one wavefront's instruction stream, and 4/5 of the pair
// kernel's is the 256-doubling u2 Q ladder. With v u2 = w (mod n), |v|, w < 2^128
// (p256_halfgcd.hpp, Antipa et al. 2005) and R0 = (r, sqrt(r^3 - 3r + b)):
//   x((v u1) G + w Q) == x(v R0)  <=>  u1 G + u2 Q = +-R0  <=>  x(u1 G + u2 Q) == r,
// for r >= p - n (below that, x = r + n is a second candidate; such r are adversarial). Both
// sides are 128-bit ladders, so each tuple takes a quad: lanes 0-1 (pair A) run w Q, lanes 2-3
// (pair B) run v R0, in the same instruction stream as the pair kernel's lane-local ladder, over
// [1, 3, ..., 15]P tables of their own. The price is the square root (253 squarings, every lane)
// in front of the table build. A workgroup is three verify wavefronts (48 tuples) and a helper
// wavefront (one lane per tuple: the request hash, s^-1, u1, u2, the Euclid reduction to (v, w),
// then (v u1) G on the fixed-base comb), so a 10k batch is 209 workgroups, one per CU, each
// wavefront on a SIMD of its own.
// Every ladder here is free of exceptional additions: the partial scalars m of an odd k < 2^129
// stay odd and 16 m +- d < n, and an even k runs as k + 1 followed by one subtraction of the base
// (exceptional only for k = 0 or -2 mod n). The comb sum joins w Q with the comb wavefront
// kernel's case split. A tuple whose reduction gave up, or with r < p - n, is verified the
// classic way inside the same launch (v = 1, w = u2: a 64-digit ladder for its wavefront,
// verify_final's comparison with r and r + n), so a crafted batch costs at most what the pair
// kernel costs.
#ifndef SBFT_HALF_TUPLES
#define SBFT_HALF_TUPLES 48
#endif
constexpr int kHalfTuples = SBFT_HALF_TUPLES;  // per workgroup
#ifndef SBFT_HALF_DIGIT_SEL
#define SBFT_HALF_DIGIT_SEL 1  // digits by selects (q_digit_sel): no alloca, no LDS promotion
#endif
#ifndef SBFT_HALF_INV_PAIR
#define SBFT_HALF_INV_PAIR 1  // the table's inversion split over the pair (inv::inv_mod_pair)
#endif
static_assert(kHalfTuples % 16 == 0 && kHalfTuples <= 64, "16 quads per verify wavefront, one helper wavefront");
// The wide form (QUAD): each ladder on a quad of its own (q4_dbl / q4_add_rest, p256_f29.hpp), eight
// lanes per tuple, 24 tuples per workgroup: three verify wavefronts and the helper, as before. It
// takes per-device batches of at most one workgroup per CU (sbft_gv_opts.halfq_max), where the
// 1,024 SIMDs have room for the extra wavefronts.
constexpr int kHalfTuplesQ = 24;
static_assert(kHalfTuplesQ % 8 == 0 && kHalfTuplesQ <= 64, "8 tuples per verify wavefront, one helper wavefront");
constexpr int kHalfVerifyThreads = 4 * kHalfTuples;
constexpr int kHalfThreads = kHalfVerifyThreads + 64;
static_assert(8 * kHalfTuplesQ + 64 == kHalfThreads, "both forms launch 256-thread workgroups");
constexpr int kHalfDigits = 32;  // radix-16 digits of an odd k < 2^129
// b 2^261 mod p (radix 2^29) and p - n (8 x 32, < 2^127); tests/test_abi.py checks both
__device__ __constant__ static const u32 C29_B[9] = {0x1897bbfbu, 0x1cdf6229u, 0x018486c4u, 0x01732821u, 0x1dad59e0u,
                                                     0x0abf7212u, 0x1a06d110u, 0x17721d20u, 0x008600c3u};
__device__ __constant__ static const u32 P256_PMN[8] = {0x039cdaaeu, 0x0c46353du, 0x58e8617bu, 0x43190553u, 0u, 0u, 0u, 0u};

// verify_inputs_valid's curve equation in the ladders' radix-2^29 arithmetic (4 products against
// the 8 x 32 form's 5): y^2 - (x^3 - 3x + b) == 0 mod p, with the bounds of the half kernel's
// c = r^3 - 3r + b and of its square test (x, y < 2^256 in, as r there).
SBFT_DEV bool q_on_curve29(const fe& qx, const fe& qy) {
    const f29 r2c = f29_const(C29_R2), b = f29_const(C29_B);
    f29 xm, ym, t2, t3, cv, yy, dd;
    f29_mul_ilp(xm, f29_from_u256(qx), r2c);
    f29_mul_ilp(ym, f29_from_u256(qy), r2c);
    f29_sqr_ilp(t2, xm);
    f29_mul_ilp(t3, t2, xm);
#pragma unroll
    for (int i = 0; i < 9; ++i) cv.v[i] = t3.v[i] - 3u * xm.v[i] + b.v[i];  // |limb| < 2^31
    f29_normalize(cv, cv);                                                  // N'
    f29_sqr_ilp(yy, ym);
    f29_sub(dd, yy, cv);  // |limb| < 2^30, |.| < 2^259
    return f29_zero_mod_p_any(dd);
}

SBFT_DEV void f29_sqr_n(f29& t, int k) {
#pragma unroll 1
    for (int i = 0; i < k; ++i) f29_sqr_ilp(t, t);
}
// y = x^((p+1)/4), (p+1)/4 = ((2^64 - 2^32 + 1) 2^96 + 1) 2^94: 253 squarings, 7 products (the
// Montgomery forms of x in and y out; y^2 == x iff x is a square)
SBFT_DEV void f29_sqrt_chain(f29& y, const f29& x) {
    f29 t, x2, x4, x8, x16;
    f29_sqr_ilp(t, x);
    f29_mul_ilp(x2, t, x);  // x^(2^2 - 1)
    t = x2;
    f29_sqr_n(t, 2);
    f29_mul_ilp(x4, t, x2);  // 2^4 - 1
    t = x4;
    f29_sqr_n(t, 4);
    f29_mul_ilp(x8, t, x4);  // 2^8 - 1
    t = x8;
    f29_sqr_n(t, 8);
    f29_mul_ilp(x16, t, x8);  // 2^16 - 1
    t = x16;
    f29_sqr_n(t, 16);
    f29_mul_ilp(t, t, x16);  // 2^32 - 1
    f29_sqr_n(t, 32);
    f29_mul_ilp(t, t, x);  // 2^64 - 2^32 + 1
    f29_sqr_n(t, 96);
    f29_mul_ilp(t, t, x);
    f29_sqr_n(t, 94);
    y = t;
}

// z^-1 = z^(p - 2) in the Montgomery domain: 255 squarings and 13 products on the addition chain
// x2, x4, x8, x16, x24, x28, x30, x32 (x_k = z^(2^k - 1)), then (((x32 2^32 z) 2^128 x32) 2^32 x32)
// 2^30 x30, 2^2 z -- one rolled loop over the 13 links (a squaring loop, one product by a
// selected multiplier, the result kept by select), so the code is two products' worth.
SBFT_DEV void f29_inv_chain(f29& out, const f29& z) {
    // per link: squarings, multiplier (0 z, 1 x2, 2 x4, 3 x8, 4 x30, 5 x32), slot the result goes to
    constexpr u32 kSq = 1u | 2u << 8 | 4u << 16 | 8u << 24, kSq2 = 8u | 4u << 8 | 2u << 16 | 2u << 24,
                  kSq3 = 32u | 128u << 8 | 32u << 16 | 30u << 24;
    f29 m1 = z, m2 = z, m3 = z, m4 = z, m5 = z, t = z;
#pragma unroll 1
    for (int l = 0; l < 13; ++l) {
        const u32 sq = l < 4 ? (kSq >> (8 * l)) & 255u
                     : l < 8 ? (kSq2 >> (8 * (l - 4))) & 255u
                     : l < 12 ? (kSq3 >> (8 * (l - 8))) & 255u : 2u;
        // multiplier: links 0..12 -> z, x2, x4, x8, x8, x4, x2, x2, z, x32, x32, x30, z
        const int mi = (int)((0x455011233210ull >> (4 * l)) & 15);  // nibble l (link 0 lowest)
        f29_sqr_n(t, (int)sq);
        f29 m;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            u32 v = z.v[i];
            v = mi == 1 ? m1.v[i] : v;
            v = mi == 2 ? m2.v[i] : v;
            v = mi == 3 ? m3.v[i] : v;
            v = mi == 4 ? m4.v[i] : v;
            v = mi == 5 ? m5.v[i] : v;
            m.v[i] = v;
        }
        f29_mul_ilp(t, t, m);
        // results kept: link 0 -> x2, 1 -> x4, 2 -> x8, 6 -> x30, 7 -> x32
        if (l == 0) m1 = t;
        if (l == 1) m2 = t;
        if (l == 2) m3 = t;
        if (l == 6) m4 = t;
        if (l == 7) m5 = t;
    }
    out = t;
}

#ifndef SBFT_HALF_HPAIR
#define SBFT_HALF_HPAIR 1  // wide form: the helper on lane pairs (s^-1 split over the pair)
#endif
#ifndef SBFT_HALF_QTAB_QUAD
#define SBFT_HALF_QTAB_QUAD 1  // the wide form builds its tables on the quad (build_q_table_quad_w)
#endif
#ifndef SBFT_HALF_GAFF
#define SBFT_HALF_GAFF 2  // the wide form's affine (v u1) G: 1 safegcd, 2 Fermat chain, 0 none (general join)
#endif

template <bool FRAMED, bool QUAD = false>
__global__ __launch_bounds__(kHalfThreads) void p256_verify_half_kernel(const uint8_t* __restrict__ digest,
                                                                    const uint8_t* __restrict__ rr,
                                                                    const uint8_t* __restrict__ ss,
                                                                    const uint8_t* __restrict__ qxx,
                                                                    const uint8_t* __restrict__ qyy,
                                                                    uint8_t* __restrict__ ok, uint32_t n,
                                                                    uint32_t* __restrict__ work,
                                                                    const uint4* __restrict__ gcomb, FramedIn fr) {
    constexpr int T = QUAD ? kHalfTuplesQ : kHalfTuples;
    constexpr int VT = (QUAD ? 8 : 4) * T;  // verify threads (then the helper wavefront)
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    __shared__ u32 qtab[kQTab * 18 * 2 * T];    // [entry][x limbs, y limbs][pair A | pair B][tuple]
    __shared__ u32 hrat[(kQTab - 1) * 9 * 2 * T]; // the table build's Z ratios, [ratio][limb][column]
    __shared__ u32 edig[FRAMED ? 8 * T : 1];    // FRAMED: the helper's digests [word][tuple]
    __shared__ u32 hsc[17 * T];                 // the helper's scalars: [k_A 0..7, k_B 0..7, flags][tuple]
    __shared__ u32 gsum[28 * T];                // the helper's (v u1) G: [x, y, z limbs, inf][tuple]
    inv::stage_divstep_table(dtab);  // ends with a barrier
#ifdef SBFT_HALF_PROBE  // development: phase times of workgroup 0 (tools/half_probe.py), 100 MHz ticks,
                        // kept in registers and printed once at the end (a printf is a blocking host call)
    // (and the shader-clock counter beside it: the clock of a phase is its s_memtime ticks over its
    // real-time ticks times 100 MHz). Marks take constant slot numbers, so the stamps stay in
    // (scalar) registers: a runtime slot index put the arrays in scratch, whose stores then
    // lengthened the waits in front of the barriers (~20 us of a probed launch).
    const uint64_t probe_t0 = __builtin_amdgcn_s_memrealtime(), probe_c0 = __builtin_amdgcn_s_memtime();
    uint32_t probe_t[8] = {0, 0, 0, 0, 0, 0, 0, 0}, probe_c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto probe = [&](int i) {
        const uint32_t t = (uint32_t)(__builtin_amdgcn_s_memrealtime() - probe_t0);
        const uint32_t c = (uint32_t)(__builtin_amdgcn_s_memtime() - probe_c0);
        switch (i) {  // constant at every call site once inlined
        case 0: probe_t[0] = t; probe_c[0] = c; break;
        case 1: probe_t[1] = t; probe_c[1] = c; break;
        case 2: probe_t[2] = t; probe_c[2] = c; break;
        case 3: probe_t[3] = t; probe_c[3] = c; break;
        case 4: probe_t[4] = t; probe_c[4] = c; break;
        case 5: probe_t[5] = t; probe_c[5] = c; break;
        case 6: probe_t[6] = t; probe_c[6] = c; break;
        default: probe_t[7] = t; probe_c[7] = c; break;
        }
    };
    auto probe_dump = [&](const char* who, bool me) {
        if (me && blockIdx.x == 0) {
            printf("half-probe %s %u %u %u %u %u %u %u %u\n", who, probe_t[0], probe_t[1], probe_t[2], probe_t[3],
                   probe_t[4], probe_t[5], probe_t[6], probe_t[7]);
            printf("half-probe-clk %s %u %u %u %u %u %u %u %u\n", who, probe_c[0], probe_c[1], probe_c[2], probe_c[3],
                   probe_c[4], probe_c[5], probe_c[6], probe_c[7]);
        }
    };
#else
    auto probe = [](int) {};
    auto probe_dump = [](const char*, bool) {};
#endif

    auto load_tuple = [&](uint32_t idx, fe& r, fe& s, fe& qx, fe& qy) {
        if constexpr (FRAMED) {
            const uint8_t* end = fr.blob + fr.off[idx] + fr.len[idx];
            r = load_be32_any(end + fr.sig_rel);
            s = load_be32_any(end + fr.sig_rel + 32);
            qx = load_be32_any(end + fr.pub_rel);
            qy = load_be32_any(end + fr.pub_rel + 32);
        } else {
            r = load_be32(rr + 32ull * idx);
            s = load_be32(ss + 32ull * idx);
            qx = load_be32(qxx + 32ull * idx);
            qy = load_be32(qyy + 32ull * idx);
        }
    };
    auto mod_n_neg = [](const fe& a) {  // n - a (a in [0, n])
        fe t;
        u64 b = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const u64 d = (u64)P256_N[k] - a.v[k] - b;
            t.v[k] = lo32(d);
            b = d >> 63;
        }
        return t;
    };

    if (threadIdx.x >= VT) {  // the helper wavefront (wave-uniform branch)
        const uint32_t lane = threadIdx.x - VT;
        // The wide form (24 tuples) takes a lane pair per tuple: s^-1 split over the pair
        // (inv::inv_mod_pair), the even lane publishing; the four-lane form a lane per tuple.
        constexpr bool HP = QUAD && SBFT_HALF_HPAIR;
        const uint32_t hslot = HP ? lane >> 1 : lane;
        const bool hodd = HP && (lane & 1u) != 0;
        const bool mine = hslot < (uint32_t)T;
        const bool pub = mine && !hodd;
        const uint32_t slot = mine ? hslot : 0u;
        const uint32_t tc = blockIdx.x * T + slot;
        const uint32_t ic = tc < n ? tc : n - 1;
        fe r, s, qx, qy;
        load_tuple(ic, r, s, qx, qy);
        const bool valid = HP ? verify_inputs_in_range(r, s, qx, qy) && q_on_curve29(qx, qy)
                              : verify_inputs_valid(r, s, qx, qy);
        fe one = fe_zero();
        one.v[0] = 1;
        // barrier 1 waits for (v, w) only: s^-1, u2 and the reduction come first; the hash, u1 and
        // the comb sum are needed at barrier 2
        fe si, wm, u2;
        if constexpr (HP) inv::inv_mod_pair(si.v, (valid ? s : one).v, dtab, false, hodd);  // plain s^-1 mod n
        else inv::inv_mod(si.v, (valid ? s : one).v, dtab, false);
        fn_mul(wm, si, fe_const(C_R2N));                          // s^-1 R
        fn_mul(u2, r, wm);
        fn_canon(u2, u2);
        if (!valid) u2 = one;
        probe(0);
        hgcd::state hs;
        hgcd::init(hs, u2.v);
#pragma unroll 1
        for (int it = 0; it < 400; ++it) {
            const bool go = hgcd::more(hs);
            if (!__any(go)) break;
            if (go && !(SBFT_HGCD_LEHMER && hgcd::lehmer(hs))) hgcd::step(hs);
        }
        fe w, va;
        bool vneg;
        hgcd::result(hs, w.v, va.v, vneg);
        fe vr;
        fn_mul(vr, va, fe_const(C_R2N));  // |v| R
        bool good = hs.ok && !hgcd::more(hs) && !fe_is_zero_raw(w) && va.v[4] <= 1u;
        {  // v u2 == +-w (mod n): the result is used only when it provably holds
            fe t;
            fn_mul(t, vr, u2);
            fn_canon(t, t);
            good = good && fe_eq(t, vneg ? mod_n_neg(w) : w);
        }
        probe(1);
        const bool fb = valid && (!good || fe_lt(r, P256_PMN));  // the classic way: v = 1, w = u2
        fe ka = w, kb = va;
        if (fb || !valid) {
            ka = u2;
            kb = one;
            vneg = false;
        }
        if (pub) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                hsc[k * T + slot] = ka.v[k];
                hsc[(8 + k) * T + slot] = kb.v[k];
            }
            hsc[16 * T + slot] = (vneg ? 1u : 0u) | (fb ? 2u : 0u) | (valid ? 4u : 0u);
        }
        probe(2);
        __syncthreads();  // #1: the scalars are in hsc (the verify wavefronts' tables in qtab)
        probe(3);
        fe e_raw;
        if constexpr (FRAMED) {
            uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
            if (mine && tc < n) {
                const uint8_t* msg = fr.blob + fr.off[ic];
                const uint32_t L = fr.len[ic], nb = sha256_nblocks(L);
                uint32_t wd[16];
                for (uint32_t b = 0; b < nb; ++b) {
                    sha256_block_at(msg, L, b, wd);
                    compress(h, wd);
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                e_raw.v[7 - k] = h[k];
                if (pub) edig[k * T + slot] = h[k];
            }
        } else {
            e_raw = load_be32(digest + 32ull * ic);
        }
        probe(4);
        fe e, u1, c;
        fn_canon(e, e_raw);
        fn_mul(u1, e, wm);
        fn_canon(u1, u1);
        fn_mul(c, vr, u1);  // |v| u1
        fn_canon(c, c);
        if (vneg && !fe_is_zero_raw(c)) c = mod_n_neg(c);
        if (fb || !valid) c = u1;
        // c G on the comb, in comb_add_u1g's odd recoding (even c -> n - c, base negated; c = 0
        // becomes n, whose comb sum cancels to infinity)
        const bool neg1 = (c.v[0] & 1u) == 0;
        if (neg1) c = mod_n_neg(c);
        jp29 g;
        g.x = g.y = g.z = f29_const(C29_ONE);
        bool ginf = true;  // the first addition returns its addend (add_aff_fix)
        comb_add_u1g(g, c, neg1, gcomb, [](jp29& a, const f29& x2, const f29& y2) { p29_add_aff_lean(a, x2, y2); },
                     [&](auto reload) { add_aff_fix(g, ginf, [](jp29& p) { p29_dbl(p, p); }, reload); });
        // The verify wavefronts join the sum with one mixed addition (a quad's or a pair's), so it
        // is made affine here: the helper has ~150 us to spare after the comb for one inversion and
        // four products. Z = 0 without the infinity flag (no honest tuple) keeps the Jacobian sum
        // for the general join.
        bool gaff = false;
        if constexpr (SBFT_HALF_GAFF != 0) {
            gaff = !ginf && !f29_zero_mod_p(g.z);
            f29 zinv, z2, z3, ax, ay;
            if (SBFT_HALF_GAFF == 1) {
                fe zi;
                inv::inv_mod(zi.v, f29_canon_plain(gaff ? g.z : f29_const(C29_ONE)).v, dtab, true);
                f29_mul(zinv, f29_from_u256(zi), f29_const(C29_R2));  // 1 / Z
            } else {
                f29_inv_chain(zinv, g.z);
            }
            f29_sqr(z2, zinv);
            f29_mul(z3, z2, zinv);
            f29_mul(ax, g.x, z2);
            f29_mul(ay, g.y, z3);
            if (gaff) {
                g.x = ax;
                g.y = ay;
                g.z = f29_const(C29_ONE);
            }
        }
        probe(5);
        // No square test here (round 5): whether x = r is on the curve at all (r^3 - 3r + b a
        // square) is decided by the comparison itself; only an irregular end of the ladders
        // (Z_T or W_V = 0, never for an honest tuple) needs it, and the verify wavefronts compute
        // it for that case (the irregular branch of the final comparison)
        if (pub) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                gsum[k * T + slot] = g.x.v[k];
                gsum[(9 + k) * T + slot] = g.y.v[k];
                gsum[(18 + k) * T + slot] = g.z.v[k];
            }
            gsum[27 * T + slot] = (ginf ? 1u : 0u) | (gaff ? 2u : 0u);
        }
        __syncthreads();  // #2: hand-over to the verify wavefronts
        probe_dump("helper sinv,hgcd,published,barrier1,hash,comb", lane == 0);
        return;
    }

    const int tid = threadIdx.x;
    const int pr = QUAD ? tid >> 3 : tid >> 2;                // tuple in the workgroup
    const int role = QUAD ? (tid >> 2) & 1 : (tid >> 1) & 1;  // 0: pair / quad A (w Q), 1: B (v R0)
    // odd lane of a pair: the table build runs on pairs (QUAD: lanes 2-3 of a quad repeat 0-1)
    const bool odd = (tid & 1) != 0;
    const int col = role * T + pr;          // this pair's column of qtab
    const uint32_t t = blockIdx.x * T + pr;
    const bool active = t < n;
    const uint32_t idx = active ? t : (n - 1);
    fe r, s, qx, qy;
    load_tuple(idx, r, s, qx, qy);
    // No input checks here: the helper makes them (valid arrives with the scalars at barrier 1).
    // An invalid tuple's pairs run on whatever its r and Q are -- pure arithmetic with wave-uniform
    // trip counts, whose result only the masked verdict would read.

    // Pair A's base is Q on the curve; pair B's is P' = (c r, c^2) on E_c, c = r^3 - 3r + b (the
    // image of R0 = (r, sqrt(c)) when c is a square; the helper decides that by barrier 2)
    const f29 r2c = f29_const(C29_R2), one29 = f29_const(C29_ONE);
    f29 rm, rhs;
    f29_mul_ilp(rm, f29_from_u256(r), r2c);  // |r R| < 2^256.1 (product output)
    {
        f29 t2, t3;
        const f29 b = f29_const(C29_B);
        f29_sqr_ilp(t2, rm);
        f29_mul_ilp(t3, t2, rm);
#pragma unroll
        for (int i = 0; i < 9; ++i) rhs.v[i] = t3.v[i] - 3u * rm.v[i] + b.v[i];  // |limb| < 2^31, |.| < 2^259
        f29_normalize(rhs, rhs);                                                  // c (N')
    }
    probe(0);
    const bool onc = role == 1;  // this pair runs on E_c (pair A on the curve, c = 1)
    f29 px, py, cc, ac;
    {
        f29 o;  // A: qx R2 | qy R2, B: c r | c c, one paired step
        const f29 qa = f29_pick(odd, f29_from_u256(qx), f29_from_u256(qy));
        f29_mul_ilp(o, role ? rhs : qa, role ? f29_pick(odd, rm, rhs) : r2c);
        f29_unpair(o, px, py);
        cc = onc ? rhs : one29;  // c (never 0: the curve has no point of order 2)
        ac = onc ? py : one29;   // c^2 = y(P')
        // both lanes of the pair store the same words in this pair's column of qtab
        auto st = [&](int m, const f29& x, const f29& y) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                qtab[(m * 18 + k) * 2 * T + col] = x.v[k];
                qtab[(m * 18 + 9 + k) * 2 * T + col] = y.v[k];
            }
        };
        auto ld = [&](int m, f29& x, f29& y) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                x.v[k] = qtab[(m * 18 + k) * 2 * T + col];
                y.v[k] = qtab[(m * 18 + 9 + k) * 2 * T + col];
            }
        };
        auto inv_zc = [&](const fe& zp) {  // both lanes of the pair hold the same z c
            fe zi;
            if (SBFT_HALF_INV_PAIR) inv::inv_mod_pair(zi.v, zp.v, dtab, true, odd);
            else inv::inv_mod(zi.v, zp.v, dtab, true);
            return zi;
        };
        auto mark = [&](int m) { probe(m ? (m == 1 ? 2 : 3) : 1); };
        auto hst = [&](int m, const f29& h) {
#pragma unroll
            for (int k = 0; k < 9; ++k) hrat[(m * 9 + k) * 2 * T + col] = h.v[k];
        };
        auto hld = [&](int m, f29& h) {
#pragma unroll
            for (int k = 0; k < 9; ++k) h.v[k] = hrat[(m * 9 + k) * 2 * T + col];
        };
        if constexpr (QUAD && SBFT_HALF_QTAB_QUAD) build_q_table_quad_w(px, py, ac, cc, inv_zc, mark, st, ld, hst, hld);
        else build_q_table_pair_w(px, py, ac, cc, odd, inv_zc, mark, st, ld, hst, hld);
    }
    probe(3);
    __syncthreads();  // #1: tables in qtab, the helper's scalars in hsc
    probe(4);

    const u32 flags = hsc[16 * T + pr];
    const bool valid = (flags & 4u) != 0;
    const bool fb = (flags & 2u) != 0;
    const bool negb = role == 1 && (flags & 1u) != 0;  // v < 0: v R0 = |v| (-R0)
    fe k;
#pragma unroll
    for (int i = 0; i < 8; ++i) k.v[i] = hsc[(role * 8 + i) * T + pr];
    const bool keven = (k.v[0] & 1u) == 0;
    if (keven) {  // k + 1 (k < n: no carry out)
        u64 c = 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c += k.v[i];
            k.v[i] = lo32(c);
            c >>= 32;
        }
    }
    const int L = __any(fb) ? kQDigits : kHalfDigits;  // wave-uniform

    auto tab_entry = [&](int m, f29& x, f29& y) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            x.v[i] = qtab[(m * 18 + i) * 2 * T + col];
            y.v[i] = qtab[(m * 18 + 9 + i) * 2 * T + col];
        }
    };
    auto qentry = [&](int i, f29& x, f29& y) {
        const int d = SBFT_HALF_DIGIT_SEL ? q_digit_sel(k, i) : q_digit(k, i);
        tab_entry((d < 0 ? -d : d) >> 1, x, y);
        if ((d < 0) != negb) f29_neg(y, y);
    };
    auto base_neg = [&](f29& x, f29& y) {
        tab_entry(0, x, y);
        if (!negb) f29_neg(y, y);
    };
    auto dblp = [odd](jp29& p) { p29_dbl_pair(p, p, odd); };
    // acc: the ladder's end (after digit 0's addition and, for an even k, the base's subtraction),
    // vw: its W = c Z^2; q (q4): the state before digit 0's addition, where the classic ladders'
    // exact repairs start
    jp29 acc;
    f29 vw;
    plw29 q;
    q4w q4, qfin;  // QUAD: the ladder's end as a quad state (the join's mixed addition starts there)
    plw29 qfinp;   // the same as a pair state (four-lane form)
    if constexpr (QUAD) {
        // the top term 16^L: the base itself, Z = 1, W = c
        {
            f29 y0 = py;
            if (negb) f29_neg(y0, y0);
            q4w_init(q4, px, y0, one29, cc);
        }
        f29 ut;
#pragma unroll 1
        for (int i = L - 1; i >= 1; --i) {
            f29 x2, y2;
            // the digit's LDS reads issued before the doublings (x2 enters step 3 of the last)
            const int d = q_digit_sel(k, i);
            tab_entry((d < 0 ? -d : d) >> 1, x2, y2);
            const bool ng = (d < 0) != negb;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int dd = 0; dd + 1 < kQWin; ++dd) q4_dbl<false>(q4, x2, ut);
            q4_dbl<true>(q4, x2, ut);
#pragma unroll
            for (int t = 0; t < 9; ++t) y2.v[t] = ng ? 0u - y2.v[t] : y2.v[t];
            q4_add_rest(q4, y2, ut);
        }
        f29 x2, y2;
        qentry(0, x2, y2);
#pragma unroll
        for (int dd = 0; dd + 1 < kQWin; ++dd) q4_dbl<false>(q4, x2, ut);
        q4_dbl<true>(q4, x2, ut);
        // the last addition (digit 0) and, for an even k, the subtraction of the base: free of
        // exceptional cases on the half-size ladders
        q4w qw = q4;
        q4_add_rest(qw, y2, ut);
        if (__any(keven)) {  // k + 1 ran: subtract the base once
            q4w q2 = qw;
            base_neg(x2, y2);
            q4_add_full(q2, x2, y2);
            if (keven) qw = q2;
        }
        q4w_to(acc, qw);
        vw = q4w_w(qw);
        qfin = qw;
    } else {
        // the top term 16^L (k = 16^L + sum d_i 16^i): the base itself, Z = 1, W = c
        {
            f29 y0 = py;
            if (negb) f29_neg(y0, y0);
            q.xb = px;
            q.zy = f29_sel_pair(one29, y0);
            q.zo = one29;
            q.w = cc;
        }
#pragma unroll 1
        for (int i = L - 1; i >= 1; --i) {
            f29 x2, y2;
            bool ng = false;
            if (SBFT_HALF_ENTRY_EARLY) {
                // the digit's LDS reads issued before the doublings (pinned there), its sign applied
                // after them: read after the doublings, each digit waited on LDS latency
                const int d = SBFT_HALF_DIGIT_SEL ? q_digit_sel(k, i) : q_digit(k, i);
                tab_entry((d < 0 ? -d : d) >> 1, x2, y2);
                ng = (d < 0) != negb;
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int d = 0; d < kQWin; ++d) p29_dbl_plw(q);
            if (SBFT_HALF_ENTRY_EARLY) {
#pragma unroll
                for (int t = 0; t < 9; ++t) y2.v[t] = ng ? 0u - y2.v[t] : y2.v[t];
            } else {
                qentry(i, x2, y2);
            }
            p29_add_aff_plw(q, x2, y2);
        }
#pragma unroll
        for (int d = 0; d < kQWin; ++d) p29_dbl_plw(q);
        // The last addition (digit 0) and, for an even k, the subtraction of the base: free of
        // exceptional cases on the half-size ladders (both pairs, W kept).
        plw29 qw = q;
        {
            f29 x2, y2;
            qentry(0, x2, y2);
            p29_add_aff_plw(qw, x2, y2);
        }
        if (__any(keven)) {  // k + 1 ran: subtract the base once
            plw29 q2 = qw;
            f29 x2, y2;
            base_neg(x2, y2);
            p29_add_aff_plw(q2, x2, y2);
            if (keven) qw = q2;
        }
        plw29_to(acc, qw);
        vw = qw.w;
        qfinp = qw;
    }
    bool inf = false;  // only a classic (fb) ladder can meet infinity, at its last addition
    if (__builtin_expect(__any(fb), 0)) {  // classic ladders (pair A, c = 1): the exact repairs
        jp29 a;
        if constexpr (QUAD) q4w_to(a, q4);
        else plw29_to(a, q);
        bool infa = false;
        f29 x2, y2;
        qentry(0, x2, y2);
        p29_add_aff_pair(a, x2, y2, odd);
        add_aff_fix(a, infa, dblp, [&](f29& x, f29& y) { qentry(0, x, y); });
        if (__any(keven)) {
            jp29 a2 = a;
            bool inf2 = infa;
            base_neg(x2, y2);
            p29_add_aff_pair(a2, x2, y2, odd);
            add_aff_fix(a2, inf2, dblp, base_neg);
            if (keven) {
                a = a2;
                infa = inf2;
            }
        }
        if (fb) {
            acc = a;
            inf = infa;
        }
    }
    probe(5);
    // pair (quad) B's X and W = c Z^2 of v R0, on pair (quad) A's lanes: quad_perm [2,3,2,3] (QUAD:
    // row_shl:4, lane i gets lane i + 4's)
    f29 VX, VW;
    constexpr int kMoveB = QUAD ? 0x104 : 0xEE;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        VX.v[i] = (u32)__builtin_amdgcn_mov_dpp((int)acc.x.v[i], kMoveB, 0xF, 0xF, false);
        VW.v[i] = (u32)__builtin_amdgcn_mov_dpp((int)vw.v[i], kMoveB, 0xF, 0xF, false);
    }

    __syncthreads();  // #2: the helper's (v u1) G and the square test are in gsum
    probe(6);
    const u32 gflags = gsum[27 * T + pr];
    jp29 g;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        g.x.v[i] = gsum[i * T + pr];
        g.y.v[i] = gsum[(9 + i) * T + pr];
        g.z.v[i] = gsum[(18 + i) * T + pr];
    }
    // T = acc + g (pair / quad A), V on E_c: x(V) = X_V / W_V. Accept iff T != infinity and
    // X_T W_V == X_V Z_T^2. No square test is needed for a regular end (Z_T, W_V != 0): if c =
    // r^3 - 3r + b is not a square, E_c is the quadratic twist, and x(V) = X_V / W_V has f(x) =
    // x^3 - 3x + b = (Y_V / c)^2 / c a non-square (f has no root: the curve has no point of order
    // 2), so it is the x of no point of the curve, T's included, and the comparison fails -- as
    // Go's x(R) = r must, since no point has x = r. (A twist point of small order, which could end V
    // at infinity, is out of reach: the twist order is 3 5 13 179 times a 241-bit prime, and P' is
    // fixed by r.)
    bool accept = false, irregular = false, exc = false, joined = false;
    if constexpr (QUAD) {
        // The wide form's join: the helper's affine sum added to quad A's end state by one quad
        // mixed addition (4 steps) and both sides of the comparison in one step, W_T = Z_T^2 on
        // the curve (c = 1), instead of the general Jacobian addition and three products on every
        // lane (19 products in sequence). Only when no tuple of the wavefront runs the classic
        // ladder, every sum is affine and no addition meets H = 0 (c G = +-w Q): else the general
        // join below, from the same end state.
        if (!__any(fb || (gflags & 2u) == 0)) {
            q4w t4 = qfin;
            q4_add_full(t4, g.x, g.y);
            const f29 zt = f29_qperm<0xAA>(t4.z);
            const bool hz = role == 0 && f29_zero_mod_p(zt);
            if (!__any(hz)) {
                joined = true;
                f29 o, d;
                f29_mul_ilp(o, f29_qsel<kQL1>(t4.xy, VX), f29_qsel<kQL1>(VW, f29_qperm<0xAA>(t4.w)));  // X_T W_V | X_V W_T
                f29_sub(d, f29_qperm<0x00>(o), f29_qperm<0x55>(o));
                irregular = f29_zero_mod_p(zt) || f29_zero_mod_p(VW);
                accept = !irregular && f29_zero_mod_p_any(d);
            }
        }
    } else {
        // The four-lane form's join, the same way: one paired mixed addition (5 steps) and one
        // paired step for both sides of the comparison
        if (!__any(fb || (gflags & 2u) == 0)) {
            plw29 t2 = qfinp;
            p29_add_aff_plw(t2, g.x, g.y);
            const f29 zt = f29_sel_pair(t2.zy, t2.zo);  // Z_T in both lanes
            const bool hz = role == 0 && f29_zero_mod_p(zt);
            if (!__any(hz)) {
                joined = true;
                f29 o, d;
                f29_mul_ilp(o, f29_sel_pair(t2.xb, VX), f29_sel_pair(VW, t2.w));  // X_T W_V | X_V W_T
                f29_sub(d, o, f29_swap_pair(o));
                irregular = f29_zero_mod_p(zt) || f29_zero_mod_p(VW);
                accept = !irregular && f29_zero_mod_p_any(d);
            }
        }
    }
    if (!joined) {  // wave-uniform
        const bool ginf = (gflags & 1u) != 0;
        const jp29 a0 = acc;
        p29_add_jac_lean(acc, g);
        // H == 0 (Z3 = 0): a doubling if X3 == 0 (c G == w Q), else infinity (c G == -w Q)
        const bool hz = !inf && !ginf && f29_zero_mod_p(acc.z);
        if (__builtin_expect(__any(hz || inf || ginf), 0)) {
            const bool twice = hz && f29_zero_mod_p_any(acc.x);
            jp29 d = a0;
            dblp(d);
            if (twice) acc = d;
            if (ginf) acc = a0;
            if (inf) acc = g;
            inf = (hz && !twice) || (inf && ginf);
        }
        f29 zt2, lhs, rhs2, d;
        f29_sqr(zt2, acc.z);
        f29_mul(lhs, acc.x, VW);
        f29_mul(rhs2, VX, zt2);
        f29_sub(d, lhs, rhs2);  // |limb| < 2^29.2, |.| < 2^257
        irregular = f29_zero_mod_p(acc.z) || f29_zero_mod_p(VW);
        accept = !irregular && f29_zero_mod_p_any(d);
    }
    {
        // never for a valid honest tuple; an invalid one (rejected whatever its pairs computed)
        // must not send its wavefront down this path
        if (__builtin_expect(__any(irregular && !inf && valid && !fb), 0)) {
            // the fixup net takes it if x = r is on the curve (then it is truly exceptional);
            // otherwise it is a rejection. r^3 - 3r + b a square: y = (.)^((p+1)/4), y^2 == it
            f29 rmm, t2, t3, cv, y0, yy, dd;
            const f29 b = f29_const(C29_B);
            f29_mul_ilp(rmm, f29_from_u256(r), f29_const(C29_R2));
            f29_sqr_ilp(t2, rmm);
            f29_mul_ilp(t3, t2, rmm);
#pragma unroll
            for (int i = 0; i < 9; ++i) cv.v[i] = t3.v[i] - 3u * rmm.v[i] + b.v[i];  // |limb| < 2^31
            f29_normalize(cv, cv);                                                    // N'
            f29_sqrt_chain(y0, cv);
            f29_sqr_ilp(yy, y0);
            f29_sub(dd, yy, cv);  // |limb| < 2^30, |.| < 2^259
            exc = irregular && f29_zero_mod_p_any(dd);  // fixup net
        }
    }
    if (__builtin_expect(__any(fb), 0)) {
        bool exc_f;
        const bool acc_f = verify_final(acc, r, exc_f);
        if (fb) {
            accept = acc_f;
            exc = exc_f;
        }
    }
    if (inf) {  // R = infinity: rejected, not an exceptional tuple
        accept = false;
        exc = false;
    }
    probe(7);
    probe_dump(tid == 0 ? "verify inputs,chain,inverse,tables,barrier1,ladder,barrier2,final"
                        : (tid == 64 ? "verify-w1" : "verify-w2"),
               tid == 0 || tid == 64 || tid == 128);
    if (active && (tid & (QUAD ? 7 : 3)) == 0) {
        if (exc && valid) {
            if constexpr (FRAMED) {  // the fixup kernel's inputs
                fe e_raw;
#pragma unroll
                for (int i = 0; i < 8; ++i) e_raw.v[7 - i] = edig[i * T + pr];
                store_be32(fr.dig + 32ull * t, e_raw);
                store_be32(fr.r + 32ull * t, r);
                store_be32(fr.s + 32ull * t, s);
                store_be32(fr.qx + 32ull * t, qx);
                store_be32(fr.qy + 32ull * t, qy);
            }
            const uint32_t slot = atomicAdd(work, 1u);
            work[1 + slot] = t;
            if constexpr (FRAMED) {
                if (fr.flagged) *(volatile uint32_t*)fr.flagged = 1u;
            }
        } else {
            ok[t] = (valid && accept) ? 1 : 0;
        }
    }
}

// ---- registered keys, large batches: four lanes per signature (p256_verify_keyed_lanes) ----
// For batches too large for one wavefront per signature (p256_keyed.hip's latency kernel),
// each signature takes a quad: lane j sums 16 comb entries with lean mixed additions in
// radix 2^29 — j = 0, 1: windows 0-15 / 16-31 of u1 over G's table; j = 2, 3: the same of u2
// over the key's table — then the quad adds the four partial sums (two lean Jacobian
// additions) and checks x(R) = r. Each lane inverts s itself (safegcd, LDS divstep table).
// No partial sum inside a chain or of two chains of the same scalar can meet an exceptional
// case (they are m P for distinct 0 < m < n over disjoint windows); only G part + Q part can
// (u1 G = +-u2 Q, craftable with related keys). That shows as Z = 0, and the quad then
// recomputes the signature with the exact 8 x 32 additions (infinity, doubling, cancellation).
SBFT_DEV void jp29_pick(jp29& out, bool c, const jp29& a) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        out.x.v[k] = c ? a.x.v[k] : out.x.v[k];
        out.y.v[k] = c ? a.y.v[k] : out.y.v[k];
        out.z.v[k] = c ? a.z.v[k] : out.z.v[k];
    }
}
// acc + (partner lane's acc) with infinity flags, lean (quad_perm control CTRL picks the partner)
template <int CTRL>
SBFT_DEV void quad_combine(jp29& acc, bool& inf) {
    jp29 o;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        o.x.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)acc.x.v[k], CTRL, 0xf, 0xf, false);
        o.y.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)acc.y.v[k], CTRL, 0xf, 0xf, false);
        o.z.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)acc.z.v[k], CTRL, 0xf, 0xf, false);
    }
    const bool oinf = __builtin_amdgcn_mov_dpp(inf ? 1 : 0, CTRL, 0xf, 0xf, false) != 0;
    jp29 sum = acc;
    p29_add_jac_lean(sum, o);
    jp29_pick(sum, inf, o);
    jp29_pick(sum, oinf && !inf, acc);
    acc = sum;
    inf = inf && oinf;
}

// FRAMED (sbft_launch_p256_verify_keyed_framed): the signatures' bodies lie in a payload
// (fr.blob/off/len, r || s at the body's end + fr.sig_rel); a fifth wavefront per workgroup
// hashes the workgroup's 64 bodies into LDS while the four verify wavefronts invert s, and
// the digests are picked up after that barrier. No hash kernel in front.
#ifndef SBFT_KEYED_LANES_ILP
#define SBFT_KEYED_LANES_ILP 1  // the comb's additions in the pipelined ILP product form
#endif
#ifndef SBFT_KEYED_LANES_PINGPONG
#define SBFT_KEYED_LANES_PINGPONG 1  // the comb's entries in two fixed buffers (see the kernel)
#endif
// FRAMED: signatures per workgroup (a multiple of 16). 48: three verify wavefronts and the hash
// wavefront, one per SIMD, so the hash (the comb's wait for its digests) does not share a SIMD
// with an inverting wavefront; 64: four verify wavefronts and the hash wavefront on five.
#ifndef SBFT_KEYED_LANES_ZPRE
#define SBFT_KEYED_LANES_ZPRE 1  // the comb's next Z^2, Z^3 formed inside the current addition
#endif
#ifndef SBFT_KEYED_FRAMED_TPB
#define SBFT_KEYED_FRAMED_TPB 48
#endif
template <bool FRAMED = false>
__global__ __launch_bounds__(FRAMED ? 4 * SBFT_KEYED_FRAMED_TPB + 64 : 256) void p256_verify_keyed_lanes_kernel(
    const uint8_t* __restrict__ digest, const uint8_t* __restrict__ rr, const uint8_t* __restrict__ ss,
    const uint32_t* __restrict__ key, const uint4* const* __restrict__ keytab, uint32_t nkeys,
    uint8_t* __restrict__ ok, uint32_t n, FramedIn fr) {
    __shared__ __attribute__((aligned(16))) uint32_t dtab[SBFT_DIVSTEP5_WORDS];
    __shared__ u32 edig[FRAMED ? 8 * 64 : 1];  // FRAMED: [word][signature of the workgroup]
    inv::stage_divstep_table(dtab);  // ends with a barrier
#ifdef SBFT_KEYED_PROBE  // development: phase times of workgroup 0 (tools/keyed_lanes_probe.py), as the
                         // half kernel's SBFT_HALF_PROBE: 100 MHz real-time ticks in constant slots
    const uint64_t probe_t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t probe_t[6] = {0, 0, 0, 0, 0, 0};
    auto probe = [&](int i) {
        const uint32_t t = (uint32_t)(__builtin_amdgcn_s_memrealtime() - probe_t0);
        switch (i) {
        case 0: probe_t[0] = t; break;
        case 1: probe_t[1] = t; break;
        case 2: probe_t[2] = t; break;
        case 3: probe_t[3] = t; break;
        case 4: probe_t[4] = t; break;
        default: probe_t[5] = t; break;
        }
    };
    auto probe_dump = [&](const char* who) {
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)
            printf("keyed-probe %s %u %u %u %u %u %u\n", who, probe_t[0], probe_t[1], probe_t[2], probe_t[3],
                   probe_t[4], probe_t[5]);
    };
#else
    auto probe = [](int) {};
    auto probe_dump = [](const char*) {};
#endif
    if constexpr (FRAMED) {
        if (threadIdx.x >= 4 * SBFT_KEYED_FRAMED_TPB) {  // the hash wavefront
            const uint32_t lane = threadIdx.x - 4 * SBFT_KEYED_FRAMED_TPB, th = blockIdx.x * SBFT_KEYED_FRAMED_TPB + lane;
            if (lane < SBFT_KEYED_FRAMED_TPB && th < n) {
                const uint8_t* msg = fr.blob + fr.off[th];
                const uint32_t L = fr.len[th], nb = sha256_nblocks(L);
                uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
                uint32_t w[16];
                for (uint32_t b = 0; b < nb; ++b) {
                    sha256_block_at(msg, L, b, w);
                    compress(h, w);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) edig[k * 64 + lane] = h[k];
            }
            probe(0);
            __syncthreads();  // the verify wavefronts' digest barrier
            probe(1);
            probe_dump("hash");
            return;
        }
    }
    const uint32_t gid = blockIdx.x * (FRAMED ? 4 * SBFT_KEYED_FRAMED_TPB : 256) + threadIdx.x;
    const uint32_t t = gid >> 2, j = gid & 3u;
    const bool active = t < n;
    const uint32_t idx = active ? t : n - 1;
    fe r, s;
    if constexpr (FRAMED) {
        const uint8_t* sig = fr.blob + fr.off[idx] + fr.len[idx] + fr.sig_rel;
        r = load_be32_any(sig);
        s = load_be32_any(sig + 32);
    } else {
        r = load_be32(rr + 32ull * idx);
        s = load_be32(ss + 32ull * idx);
    }
    const uint32_t kid = key[idx];
    const bool valid = !fe_is_zero_raw(r) && fe_lt(r, P256_N) && !fe_is_zero_raw(s) && fe_lt(s, P256_N) &&
                       kid >= 1 && kid < nkeys && keytab[kid] != nullptr;
    // s^-1 in Montgomery form by each lane's own safegcd (the scaled start, p256_inv.hpp): at
    // these batch sizes the launch-wide batched inversion's two kernels cost ~90 us of latency
    fe w;
    {
        fe sv = s;
        if (!valid) {
            sv = fe_zero();
            sv.v[0] = 1;
        }
        const fe rn = fe_const(C_ONEN);  // 2^256 mod n
        inv::inv_mod(w.v, sv.v, dtab, false, rn.v);
    }
    probe(0);
    fe e, u;
    if constexpr (FRAMED) {
        __syncthreads();  // the hash wavefront's digests
        probe(1);
        fe d;
        const uint32_t sl = threadIdx.x >> 2;
#pragma unroll
        for (int k = 0; k < 8; ++k) d.v[7 - k] = edig[k * 64 + sl];
        fn_canon(e, d);
    } else {
        fn_canon(e, load_be32(digest + 32ull * idx));
    }
    fn_mul(u, j < 2 ? e : r, w);  // u1 = e s^-1 (j < 2) or u2 = r s^-1 (plain)
    fn_canon(u, u);
#if defined(SBFT_KEYED_HOT_TABLE) && !defined(SBFT_KEYED_PROBE)
#error "SBFT_KEYED_HOT_TABLE returns wrong verdicts (timing probe only): build it with SBFT_KEYED_PROBE"
#endif
#ifdef SBFT_KEYED_HOT_TABLE  // development (timing only, wrong verdicts): every u2 Q from one key's table
    const uint4* tab = keytab[j < 2 ? 0u : (valid ? 1u : 0u)];
#else
    const uint4* tab = keytab[j < 2 ? 0u : (valid ? kid : 0u)];
#endif
    const u32 w0 = 16u * (j & 1u);
    jp29 acc;
    bool inf = true;
    acc.z = f29_const(C29_ONE);
    auto add_entry = [&](const uint4 (&cur)[4], bool zero) {
        const fe ex = {{cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y, cur[1].z, cur[1].w}};
        const fe ey = {{cur[2].x, cur[2].y, cur[2].z, cur[2].w, cur[3].x, cur[3].y, cur[3].z, cur[3].w}};
        const f29 x2 = f29_from_mont256(ex), y2 = f29_from_mont256(ey);
        jp29 sum = acc;
        if (SBFT_KEYED_LANES_ILP) p29_add_aff_lean_ilp(sum, x2, y2);
        else p29_add_aff_lean(sum, x2, y2);
        if (!zero) {
            if (inf) {
                acc.x = x2;
                acc.y = y2;
                acc.z = f29_const(C29_ONE);
            } else {
                acc = sum;
            }
            inf = false;
        }
    };
    probe(2);
    if (SBFT_KEYED_LANES_PINGPONG) {
        // 16 entries in two fixed buffers, the loop unrolled by two: each entry's loads are issued
        // one addition before it is used and never waited on to move registers (the rotated
        // buffer of the form below waited on them at every iteration, as did the digit's scratch
        // load queued behind them). The lane's 16 scalar bytes (windows w0 .. w0 + 15: words
        // 4 (j & 1) .. + 3 of u) are shifted out of registers, and the table is read with global
        // (not flat) loads.
#if defined(__HIP_DEVICE_COMPILE__)
        typedef const __attribute__((address_space(1))) uint4 gu4;
#else
        typedef const uint4 gu4;  // the kernel body's host pass (HIP_vector_type has no such overload)
#endif
        gu4* const gtab = (gu4*)tab;
        u32 ub[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) ub[k] = (j & 1u) ? u.v[4 + k] : u.v[k];
        uint4 ea[4], eb[4];
        // SBFT_KEYED_LANES_ZPRE: the next accumulator's Z^2 and Z^3 are formed inside the current
        // addition, beside its X3 and Y3 products (whose Montgomery passes were single-product
        // stages with their serial chains exposed); the values are the same as forming them at the
        // start of the next addition.
        const f29 one29 = f29_const(C29_ONE);
        f29 zz = one29, zzz = one29;  // acc.z^2, acc.z^3 (acc starts at infinity with Z = 1)
        auto add_entry_zz = [&](const uint4 (&cur)[4], bool zero) {
            const fe ex = {{cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y, cur[1].z, cur[1].w}};
            const fe ey = {{cur[2].x, cur[2].y, cur[2].z, cur[2].w, cur[3].x, cur[3].y, cur[3].z, cur[3].w}};
            const f29 x2 = f29_from_mont256(ex), y2 = f29_from_mont256(ey);
            f29 u2, s2, h, rr, hh, hhh, v, z3, x3, y3, t, nd, zn, zz2, zzz2;
            f29_mul_ilp(u2, x2, zz);
            f29_mul_ilp(s2, y2, zzz);         // S2 = y2 Z1^3
            f29_sub(h, u2, acc.x);            // (-2^29.2, 2^29 + 2^25)
            f29_sub(rr, s2, acc.y);           // (-2^29.2, 2^29.2)
            f29_sqr_ilp(hh, h);
            f29_mul_ilp(hhh, hh, h);
            f29_mul_ilp(v, acc.x, hh);        // V = X1 H^2
            f29_mul_ilp(z3, acc.z, h);        // Z3 = Z1 H
#pragma unroll
            for (int k = 0; k < 9; ++k) zn.v[k] = zero ? acc.z.v[k] : (inf ? one29.v[k] : z3.v[k]);
            {
                const f29* const va[2] = {&hhh, &v};
                const u32 c[2] = {(u32)-1, (u32)-2};
                f29_mulsq_add_ilp<true, 2>(x3, rr, rr, va, c, ~0u);  // X3 = r^2 - HHH - 2V: N'
            }
            f29_sqr_ilp(zz2, zn);             // the next addition's Z1^2 ...
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                t.v[k] = v.v[k] - x3.v[k];    // (-2^29.2, 2^29 + 2^25)
                nd.v[k] = 0u - hhh.v[k];
            }
            f29_mul_sub_ilp(y3, rr, t, acc.y, nd);  // r t - Y1 H^3: N
            f29_mul_ilp(zzz2, zn, zz2);       // ... and Z1^3
            if (!zero) {
                acc.x = inf ? x2 : x3;
                acc.y = inf ? y2 : y3;
                inf = false;
            }
            acc.z = zn;
            zz = zz2;
            zzz = zzz2;
        };
        auto add_pp = [&](const uint4 (&cur)[4], bool zero) {
            if (SBFT_KEYED_LANES_ZPRE) add_entry_zz(cur, zero);
            else add_entry(cur, zero);
        };
        auto entry = [&](u32 i, u32 byte, uint4 (&en)[4]) {
            gu4* p = gtab + (size_t)((w0 + i) * COMB_ENTRIES + byte) * COMB_ENTRY_U4;
#pragma unroll
            for (int k = 0; k < 4; ++k) en[k] = p[k];
            __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk towards their use
        };
        entry(0, ub[0] & 255u, ea);
#pragma unroll 1
        for (u32 i = 0; i < 16; i += 2) {
            const u32 b0 = ub[0] & 255u, b1 = (ub[0] >> 8) & 255u;
            entry(i + 1, b1, eb);
            add_pp(ea, b0 == 0);
            // unconditional (the last pass reloads entry 15, unused): a load behind a branch
            // made the wait below it count every load in flight
            const bool more = i + 2 < 16;
            entry(more ? i + 2 : i + 1, more ? (ub[0] >> 16) & 255u : b1, ea);
            add_pp(eb, b1 == 0);
            ub[0] = __builtin_amdgcn_alignbit(ub[1], ub[0], 16);
            ub[1] = __builtin_amdgcn_alignbit(ub[2], ub[1], 16);
            ub[2] = __builtin_amdgcn_alignbit(ub[3], ub[2], 16);
            ub[3] >>= 16;
        }
    } else {
        // 16 entries, the next one's loads issued before the current addition
        uint4 cur[4], nxt[4];
        auto entry = [&](u32 i, uint4 (&en)[4]) {
            const u32 win = w0 + i;
            const uint4* p = tab + (size_t)(win * COMB_ENTRIES + byte_of(u, win)) * COMB_ENTRY_U4;
#pragma unroll
            for (int k = 0; k < 4; ++k) en[k] = p[k];
        };
        entry(0, nxt);
#pragma unroll 1
        for (u32 i = 0; i < 16; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
            if (i < 15) entry(i + 1, nxt);
            add_entry(cur, byte_of(u, w0 + i) == 0);
        }
    }
    probe(3);
    quad_combine<0xB1>(acc, inf);  // quad_perm [1,0,3,2]: u1 G on lanes 0-1, u2 Q on lanes 2-3
    quad_combine<0x4E>(acc, inf);  // quad_perm [2,3,0,1]: R on every lane
    probe(4);
    bool exc = false;
    bool accept = verify_final(acc, r, exc) && !inf;
    probe(5);
    probe_dump("verify");
    exc = exc && !inf;
    if (__builtin_expect(__any(exc), 0)) {  // rare: the exact recomputation on the quad's lane 0
        fe u1v, u2v;  // every lane of the quad gets both scalars (DPP before the branch)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u1v.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)u.v[k], 0x00, 0xf, 0xf, false);  // quad_perm [0,0,0,0]
            u2v.v[k] = (u32)__builtin_amdgcn_mov_dpp((int)u.v[k], 0xAA, 0xf, 0xf, false);  // quad_perm [2,2,2,2]
        }
        if (exc && j == 0) {
            jp a8;
            bool inf8 = true;
            a8.x = a8.y = a8.z = fe_zero();
            const uint4* qt = keytab[valid ? kid : 0u];
#pragma unroll 1
            for (u32 h = 0; h < 64; ++h) {
                const u32 win = h & 31u;
                const fe& uu = h < 32 ? u1v : u2v;
                const u32 d = byte_of(uu, win);
                const uint4* en = (h < 32 ? keytab[0] : qt) + (size_t)(win * COMB_ENTRIES + d) * COMB_ENTRY_U4;
                jp b;
                b.x = {{en[0].x, en[0].y, en[0].z, en[0].w, en[1].x, en[1].y, en[1].z, en[1].w}};
                b.y = {{en[2].x, en[2].y, en[2].z, en[2].w, en[3].x, en[3].y, en[3].z, en[3].w}};
                b.z = fe_const(C_ONEP);
                pt_add_jac(a8, inf8, b, d != 0);
            }
            accept = !inf8 && x_matches_r(a8, r);
        }
    }
    if (active && j == 0) ok[t] = (valid && accept) ? 1 : 0;
}

}  // namespace sbft

// Workspace layout (sbft_verify_work_bytes): [0, 4(n+1)) fixup counter + list, then the
// batched-inversion arrays pre | suf (32 B per tuple) and tot | kb (32 B per workgroup), then
// (256-aligned) the throughput kernel's per-lane Q tables (SBFT_VERIFY_QTAB_BYTES per tuple).
// The counter is zeroed on the stream before the lean kernel; the fixup grid reads it on the
// device, so the whole sequence stays asynchronous.
extern "C" size_t sbft_verify_work_bytes(size_t n) {
    const size_t blocks = (n + 255) / 256;
    return ((((4 * (n + 1) + 255) & ~(size_t)255) + 64 * n + 64 * blocks + 255) & ~(size_t)255) +
           (size_t)SBFT_VERIFY_QTAB_BYTES * n;
}

// The wide half kernel's workgroup uses ~65 KB of static LDS, so two could share a CU (160 KB):
// their three verify wavefronts would then share SIMDs and both run at half speed. Its launches
// ask for enough dynamic LDS to make a workgroup take more than half of a CU's, so workgroups of
// concurrent launches (other callers, or the K slots of a one-GPU split rehearsal) wait for a
// CU of their own instead. One CU per workgroup is how a launch of up to halfq_max tuples lays
// out anyway. (Dynamic LDS the kernel never touches: a reservation only.)
static size_t halfq_dyn_lds(const void* kernel) {
    hipFuncAttributes a{};
    if (hipFuncGetAttributes(&a, kernel) != hipSuccess) return 0;
    const size_t want = 82u * 1024u;  // > 160 KB / 2
    return a.sharedSizeBytes >= want ? 0 : want - a.sharedSizeBytes;
}

extern "C" int sbft_launch_p256_verify(const uint8_t* d_digest, const uint8_t* d_r, const uint8_t* d_s,
                                       const uint8_t* d_qx, const uint8_t* d_qy, uint8_t* d_ok,
                                       uint32_t n, uint32_t* d_work, const void* d_gcomb, hipStream_t stream,
                                       hipEvent_t ev0, hipEvent_t ev1, int lanes, int work_zeroed) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    const unsigned threads = 256;
    const unsigned blocks = (n + threads - 1) / threads;
    uint8_t* base = reinterpret_cast<uint8_t*>(d_work);
    const size_t o_pre = (4ull * (n + 1) + 255) & ~255ull;
    sbft::sinv_ws ws;
    ws.pre = reinterpret_cast<uint4*>(base + o_pre);
    ws.suf = reinterpret_cast<uint4*>(base + o_pre + 32ull * n);
    ws.tot = reinterpret_cast<uint4*>(base + o_pre + 64ull * n);
    ws.kb = reinterpret_cast<uint4*>(base + o_pre + 64ull * n + 32ull * blocks);
    ws.qtab = reinterpret_cast<uint4*>(base + ((o_pre + 64ull * n + 64ull * blocks + 255) & ~255ull));
#ifdef SBFT_DEBUG_BOUNDS
#define SBFT_STEP(name)                                                                      \
    do {                                                                                     \
        hipError_t e_ = hipStreamSynchronize(stream);                                        \
        fprintf(stderr, "[sbft debug] n=%u after %s: %s\n", n, name, hipGetErrorString(e_)); \
        if (e_ != hipSuccess) return -1;                                                     \
    } while (0)
#else
#define SBFT_STEP(name) \
    do {                \
    } while (0)
#endif
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    if (lanes == 0) {  // the exact net alone: every tuple is "flagged"
        hipLaunchKernelGGL(sbft::p256_fixup_all_kernel, dim3(blocks), dim3(threads), 0, stream, d_work, n);
        SBFT_STEP("fixup list");
        if (ev0 && hipEventRecord(ev0, stream) != hipSuccess) return -1;
        hipLaunchKernelGGL(sbft::p256_verify_fixup_kernel, dim3(blocks < 8u * (unsigned)cus ? blocks : 8u * (unsigned)cus),
                           dim3(threads), 0, stream, d_digest, d_r, d_s, d_qx, d_qy, d_ok, (const uint32_t*)d_work);
        if (ev1 && hipEventRecord(ev1, stream) != hipSuccess) return -1;
        SBFT_STEP("fixup");
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (!work_zeroed && hipMemsetAsync(d_work, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
    SBFT_STEP("memset");
    if (lanes < 2) {  // the small-batch kernels invert s themselves
        const unsigned groups = (n + SBFT_SINV_GROUP - 1) / SBFT_SINV_GROUP;  // <= blocks: fits tot / kb
        hipLaunchKernelGGL(sbft::p256_sinv_prep_kernel, dim3(groups), dim3(128), 0, stream, d_s, n, ws);
        SBFT_STEP("prep");
        hipLaunchKernelGGL(sbft::p256_sinv_totals_kernel, dim3(1), dim3(threads), 0, stream, (uint32_t)groups,
                           ws);
        SBFT_STEP("totals");
    }
    if (ev0 && hipEventRecord(ev0, stream) != hipSuccess) return -1;
    if (lanes == 3) {  // half-size scalars: 48 tuples per workgroup (three quad wavefronts + a helper)
        const unsigned hblocks = (n + sbft::kHalfTuples - 1) / sbft::kHalfTuples;
        hipLaunchKernelGGL(sbft::p256_verify_half_kernel<false>, dim3(hblocks), dim3(sbft::kHalfThreads), 0, stream,
                           d_digest, d_r, d_s, d_qx, d_qy, d_ok, n, d_work, (const uint4*)d_gcomb, sbft::FramedIn{});
    } else if (lanes == 4) {  // ... a quad per ladder: 24 tuples per workgroup
        const unsigned hblocks = (n + sbft::kHalfTuplesQ - 1) / sbft::kHalfTuplesQ;
        static const size_t dyn = halfq_dyn_lds((const void*)sbft::p256_verify_half_kernel<false, true>);
        hipLaunchKernelGGL((sbft::p256_verify_half_kernel<false, true>), dim3(hblocks), dim3(sbft::kHalfThreads), dyn,
                           stream, d_digest, d_r, d_s, d_qx, d_qy, d_ok, n, d_work, (const uint4*)d_gcomb,
                           sbft::FramedIn{});
    } else if (lanes == 2) {  // 64-lane workgroups of 32 tuples
        const unsigned sblocks = (n + 31) / 32;
        hipLaunchKernelGGL(sbft::p256_verify_small_kernel<2>, dim3(sblocks), dim3(64), 0, stream, d_digest, d_r, d_s,
                           d_qx, d_qy, d_ok, n, d_work, (const uint4*)d_gcomb, sbft::FramedIn{});
    } else {
        // Waves are issue-bound at 4 per SIMD, and all take the same time. When the last
        // resident round would be mostly full, a whole number of rounds with the tuples spread
        // evenly over the workgroups (a few idle lanes per wave) finishes sooner than the partial
        // round (tools/ladder_ceiling: 1M tuples 12.94 -> 12.82 ms); a round less than ~80% full
        // is cheaper as it is (its SIMDs run 3 waves faster than 4).
        const unsigned slots = (unsigned)SBFT_VERIFY_WAVES * (unsigned)cus;  // resident workgroups
        const unsigned last = blocks % slots;
        static const bool spread_on = [] {  // SBFT_VERIFY_SPREAD=0: A/B measurement only
            const char* e = getenv("SBFT_VERIFY_SPREAD");
            return !e || e[0] != '0';
        }();
        const bool spread = spread_on && blocks > slots && last != 0 && 5u * last >= 4u * slots;
        const unsigned grid = spread ? (blocks / slots + 1) * slots : blocks;
        hipLaunchKernelGGL(sbft::p256_verify_kernel, dim3(grid), dim3(threads), 0, stream, d_digest, d_r, d_s,
                           d_qx, d_qy, d_ok, n, d_work, ws, (const uint4*)d_gcomb, spread ? 1 : 0);
    }
    if (ev1 && hipEventRecord(ev1, stream) != hipSuccess) return -1;
    SBFT_STEP("verify");
    // The flagged count is known only on the device: size the grid for the worst case (every
    // tuple exceptional, e.g. a batch of crafted R = infinity signatures), capped at one
    // resident round of the chip; blocks past the count exit at once.
    const unsigned fix_cap = 8u * (unsigned)cus;
    const unsigned fix_blocks = blocks < fix_cap ? blocks : fix_cap;
    hipLaunchKernelGGL(sbft::p256_verify_fixup_kernel, dim3(fix_blocks), dim3(threads), 0, stream,
                       d_digest, d_r, d_s, d_qx, d_qy, d_ok, (const uint32_t*)d_work);
    SBFT_STEP("fixup");
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Registered-key verify of a large batch, four lanes per signature.
extern "C" int sbft_launch_p256_verify_keyed_lanes(const uint8_t* d_digest, const uint8_t* d_r, const uint8_t* d_s,
                                                   const uint32_t* d_key, const void* const* d_keytab, uint32_t nkeys,
                                                   uint8_t* d_ok, uint32_t n, hipStream_t stream) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    const unsigned threads = 256;
    const unsigned kblocks = (unsigned)((4ull * n + threads - 1) / threads);
    hipLaunchKernelGGL(sbft::p256_verify_keyed_lanes_kernel<false>, dim3(kblocks), dim3(threads), 0, stream, d_digest,
                       d_r, d_s, d_key, (const uint4* const*)d_keytab, nkeys, d_ok, n, sbft::FramedIn{});
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sbft_launch_p256_verify_keyed_framed(const uint8_t* d_blob, const uint64_t* d_off,
                                                    const uint32_t* d_len, int32_t sig_rel, const uint32_t* d_key,
                                                    const void* const* d_keytab, uint32_t nkeys, uint8_t* d_ok,
                                                    uint32_t n, hipStream_t stream) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    constexpr unsigned tpb = SBFT_KEYED_FRAMED_TPB;  // signatures per workgroup
    static_assert(tpb % 16 == 0 && tpb <= 64, "whole verify wavefronts, one hash wavefront");
    const unsigned kblocks = (unsigned)((n + tpb - 1) / tpb);
    const sbft::FramedIn fr{d_blob, d_off, d_len, sig_rel, 0, nullptr, nullptr, nullptr, nullptr, nullptr};
    hipLaunchKernelGGL(sbft::p256_verify_keyed_lanes_kernel<true>, dim3(kblocks), dim3(4 * tpb + 64), 0, stream, nullptr,
                       nullptr, nullptr, d_key, (const uint4* const*)d_keytab, nkeys, d_ok, n, fr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" size_t sbft_gcomb_table_bytes(void) { return SBFT_GCOMB_BYTES; }

extern "C" int sbft_launch_gcomb_build(void* d_table, hipStream_t stream) {
    const unsigned total = SBFT_GCOMB_WINDOWS * SBFT_GCOMB_ENTRIES + 1;
    hipLaunchKernelGGL(sbft::p256_gcomb_build_kernel, dim3((total + 255) / 256), dim3(256), 0, stream,
                       (uint4*)d_table);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Framed tuples on the small-batch kernels (lanes 2 or 4): hash, field reads and verify in one
// launch (p256_verify_small_kernel<LPT, true>), then the fixup. The SoA rows (32 B per tuple
// each) are written only for the rare tuples the fixup takes; d_work's counter must be zero.
extern "C" int sbft_launch_p256_verify_fixup(const uint8_t* d_dig, const uint8_t* d_r, const uint8_t* d_s,
                                             const uint8_t* d_qx, const uint8_t* d_qy, uint8_t* d_ok,
                                             const uint32_t* d_work, uint32_t n, hipStream_t stream) {
    if (n == 0) return 0;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    const unsigned blocks = (n + 255) / 256, fix_cap = 8u * (unsigned)cus;
    hipLaunchKernelGGL(sbft::p256_verify_fixup_kernel, dim3(blocks < fix_cap ? blocks : fix_cap), dim3(256), 0,
                       stream, d_dig, d_r, d_s, d_qx, d_qy, d_ok, d_work);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sbft_launch_p256_verify_framed(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                              uint32_t n, int32_t sig_rel, int32_t pub_rel, uint8_t* d_dig,
                                              uint8_t* d_r, uint8_t* d_s, uint8_t* d_qx, uint8_t* d_qy,
                                              uint8_t* d_ok, uint32_t* d_work, const void* d_gcomb,
                                              hipStream_t stream, int lanes, uint32_t* h_flagged) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    if (lanes != 2 && lanes != 3 && lanes != 4) return -1;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    const sbft::FramedIn fr{d_blob, d_off, d_len, sig_rel, pub_rel, d_dig, d_r, d_s, d_qx, d_qy, h_flagged};
    const unsigned tpw = lanes == 4   ? (unsigned)sbft::kHalfTuplesQ
                         : lanes == 3 ? (unsigned)sbft::kHalfTuples
                                      : (unsigned)sbft::small_kernel_tuples<2, true>();
    const unsigned sblocks = (n + tpw - 1) / tpw;
    static const size_t dynq = halfq_dyn_lds((const void*)sbft::p256_verify_half_kernel<true, true>);
    if (lanes == 4)
        hipLaunchKernelGGL((sbft::p256_verify_half_kernel<true, true>), dim3(sblocks), dim3(sbft::kHalfThreads), dynq,
                           stream, d_dig, d_r, d_s, d_qx, d_qy, d_ok, n, d_work, (const uint4*)d_gcomb, fr);
    else if (lanes == 3)
        hipLaunchKernelGGL((sbft::p256_verify_half_kernel<true>), dim3(sblocks), dim3(sbft::kHalfThreads), 0, stream,
                           d_dig, d_r, d_s, d_qx, d_qy, d_ok, n, d_work, (const uint4*)d_gcomb, fr);
    else
        hipLaunchKernelGGL((sbft::p256_verify_small_kernel<2, true>), dim3(sblocks),
                           dim3((sbft::small_kernel_threads<2, true>())), 0, stream, d_dig,
                           d_r, d_s, d_qx, d_qy, d_ok, n, d_work, (const uint4*)d_gcomb, fr);
    if (hipGetLastError() != hipSuccess) return -1;
    if (h_flagged) return 0;  // the caller launches the fixup if a tuple was flagged
    return sbft_launch_p256_verify_fixup(d_dig, d_r, d_s, d_qx, d_qy, d_ok, d_work, n, stream);
}
