// sha256.hip — batched SHA-256 (FIPS 180-4) over variable-length request payloads, gfx950.
//
// One message per lane for the compression. sha256_lds_kernel (the default) moves the bytes
// wave-cooperatively through LDS with coalesced 16-B LDS-DMA loads; sha256_stream_kernel, the
// per-lane-load form it replaced, is kept for A/B measurement (SBFT_SHA_VARIANT=0). Arbitrary
// byte alignment. HBM traffic = payload bytes + 32 B digest. Restated (independently) in
// oracle/p256_oracle.c oracle_sha256 for parity.
#include <cstdlib>

#include "sha256_dev.hpp"
#include "sbft_kernels.h"

namespace sbft {

#define SHA_CHUNK 64u

// Persistent, load-balanced batch hashing. Each lane hashes one message block by block; when
// it finishes it writes the digest and takes the next message from its wavefront's queue of
// consecutive message indices (refilled 64 at a time from one global atomic counter). So no
// lane idles while a wavefront-mate finishes a longer message (random 1-64 KiB payloads left
// ~half the lanes idle with one message per lane), the grid needs no tail of long messages,
// and a wavefront's streams stay on consecutive messages (a length sort would scatter them
// over the blob; page-translation misses then cost ~40%, tools/sha_ceiling.hip).
// order (optional): the queue yields order[k] instead of k.
__global__ __launch_bounds__(256) void sha256_stream_kernel(const uint8_t* __restrict__ blob,
                                                            const uint64_t* __restrict__ off,
                                                            const uint32_t* __restrict__ len,
                                                            const uint32_t* __restrict__ order,
                                                            uint8_t* __restrict__ dig, uint32_t n,
                                                            uint32_t* __restrict__ ctr) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t pos = 0, end = 0;  // this wavefront's queue [pos, end) (wave-uniform)
    bool exhausted = false;     // the global counter passed n (wave-uniform)
    bool act = false;
    uint32_t mi = 0, ml = 0, b = 0, nb = 0;
    const uint8_t* mp = blob;
    uint32_t h[8];
    while (true) {
        const bool need = !act && !exhausted;
        const uint64_t nm = __ballot(need);
        if (nm) {  // wave-uniform
            const uint32_t cnt = (uint32_t)__popcll(nm);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0u));
            const uint32_t avail = end - pos;
            uint32_t idx;
            if (avail >= cnt) {
                idx = pos + rank;
                pos += cnt;
            } else {
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(ctr, SHA_CHUNK);
                c = __shfl(c, 0, 64);
                idx = rank < avail ? pos + rank : c + (rank - avail);
                pos = c + (cnt - avail);
                end = c + SHA_CHUNK;
                if (c >= n) exhausted = true;
            }
            if (need && idx < n) {
                act = true;
                mi = order ? order[idx] : idx;
                ml = len[mi];
                mp = blob + off[mi];
                b = 0;
                nb = sha256_nblocks(ml);
                h[0] = 0x6a09e667;
                h[1] = 0xbb67ae85;
                h[2] = 0x3c6ef372;
                h[3] = 0xa54ff53a;
                h[4] = 0x510e527f;
                h[5] = 0x9b05688c;
                h[6] = 0x1f83d9ab;
                h[7] = 0x5be0cd19;
            }
        }
        if (!__any(act)) break;
        if (act) {
            uint32_t w[16];
            sha256_block_at(mp, ml, b, w);
            compress(h, w);
            if (++b == nb) {
                uint4* out = reinterpret_cast<uint4*>(dig + 32ull * mi);
                out[0] = make_uint4(__builtin_bswap32(h[0]), __builtin_bswap32(h[1]), __builtin_bswap32(h[2]),
                                    __builtin_bswap32(h[3]));
                out[1] = make_uint4(__builtin_bswap32(h[4]), __builtin_bswap32(h[5]), __builtin_bswap32(h[6]),
                                    __builtin_bswap32(h[7]));
                act = false;
            }
        }
    }
}

// ------------------------------------------------------------ coalesced (LDS-staged) hashing
// sha256_stream_kernel above reads each lane's own message with per-lane loads: every load
// instruction touches 64 different lines, and with ~1,300 streams per CU the 32 KiB L1 cannot
// hold a line until its next use, so each 4-byte load refetches a line from L2 (L2 -> L1
// traffic ~20-30x the payload; the kernel ran at 17% of HBM).
//
// This kernel keeps one message per lane for the compression (the serial part of SHA-256) but
// moves the bytes wave-cooperatively: a wavefront owns 64 slots (its lanes' messages) and, per
// step, fetches the next C 64-byte blocks of all 64 messages with P = 4C + 1 LDS-DMA
// instructions (global_load_lds_dwordx4, 16 B per lane, 1 KiB per instruction): instruction i,
// lane L fetches piece g = 64 i + L, i.e. piece g mod P of slot g / P, from that slot's
// 16-B-aligned chunk address (read from its owner lane with a ds_bpermute). Every instruction
// thus reads 64 x 16 B as runs of P consecutive pieces (80 B for C = 1) of ~13 messages, and
// the LDS image is slot-major rows of P pieces, contiguous in lane order as LDS-DMA requires.
// The extra piece covers the message's start offset mod 16. Double-buffered: the DMA of step
// t + 1 is issued before the compression of step t, so the wave waits on it only after a
// whole step of compute.
//
// Each lane then reads its own row (ds_read_b32 from its start offset mod 16; one v_perm_b32
// per word does the byte funnel and the big-endian swap together). Lanes step C blocks at a
// time in lock-step; a lane whose message ends mid-step is masked for the rest of it (random
// 1-64 KiB messages: < 0.2% of the block slots for C = 1). The message queue is the one of
// sha256_stream_kernel (consecutive indices per wavefront, refilled 64 at a time), drawn one
// step ahead: a lane that finishes in step t takes its next message at the start of step t so
// that step t + 1's DMA already fetches it.
//
// The DMA reads up to 16 P + 64 bytes past a message's end (it fetches whole steps; the
// padding blocks are built in registers): callers pad the blob by SBFT_SHA_BLOB_PAD bytes.
template <int C, int M, bool DB>
struct ShaLds {
    static constexpr int P = 4 * C + 1;       // 16-B pieces per slot row
    static constexpr int ROW = 16 * P;        // bytes per slot row
    static constexpr int SLOTS = 64 * M;      // a wavefront's messages in flight (M per lane)
    static constexpr int BUF = SLOTS * ROW;   // one wavefront's step buffer
    static constexpr int NBUF = DB ? 2 : 1;   // double-buffered: step t+1's DMA overlaps step t
    static constexpr int WAVES = 4;           // wavefronts per workgroup
    static constexpr int LDS = WAVES * NBUF * BUF;
};

// the wave's queue of message indices (wave-uniform state); lanes with `need` get the next
// index, or n when the batch is exhausted
struct ShaQueue {
    uint32_t pos = 0, end = 0;
    bool exhausted = false;
    __device__ __forceinline__ uint32_t take(bool need, uint32_t lane, uint32_t n, uint32_t* ctr) {
        const uint64_t nm = __ballot(need);
        uint32_t idx = n;
        if (nm && !exhausted) {  // wave-uniform
            const uint32_t cnt = (uint32_t)__popcll(nm);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0u));
            const uint32_t avail = end - pos;
            if (avail >= cnt) {
                idx = pos + rank;
                pos += cnt;
            } else {
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(ctr, SHA_CHUNK);
                c = __shfl(c, 0, 64);
                idx = rank < avail ? pos + rank : c + (rank - avail);
                pos = c + (cnt - avail);
                end = c + SHA_CHUNK;
                if (c >= n) exhausted = true;
            }
            if (!need || idx > n) idx = n;
        }
        return idx;
    }
};

// The last 16-B granule a fetch for a message may touch: the one holding its last byte (for an
// empty message the byte before it, or the blob's first granule). Pieces past it are clamped
// onto it, so the DMA never reads beyond the granules that hold message bytes: no blob padding
// is needed, and a blob sized exactly to its messages cannot fault. (The bytes past a message's
// end are masked off by the tail code either way.)
__device__ __forceinline__ uint64_t sha_last_granule(uint64_t base, uint32_t ml, uint64_t blob0) {
    const uint64_t last = ml ? base + ml - 1 : (base > blob0 ? base - 1 : base);
    return last & ~(uint64_t)15;
}

// One step's DMA: slot s = m * 64 + lane fetches its P pieces from chunk[m] of its owner lane,
// none past the slot's limit granule lim[m]. A wave whose slots all have their step inside the
// message (the common case: a lane's message ends in about one step in eight) takes the plain
// path. Otherwise the owner packs its chunk address, moved two granules down, with
// d' = 2 + (granules from the chunk to the limit, at least -1: a step starts at most 8 bytes
// past its message's end) saturated to 15 into one 64-bit value, and piece j reads granule
// min(j + 2, d') of that base: one and, one min and one add per piece.
template <int C, int M>
__device__ __forceinline__ void sha_lds_fetch(uint8_t* buf, const uint64_t (&chunk)[M], const uint64_t (&lim)[M],
                                              uint32_t lane) {
    typedef __attribute__((address_space(3))) void* lptr;
    typedef __attribute__((address_space(1))) void* gptr;
    constexpr int P = 4 * C + 1;
    static_assert(P + 1 <= 15, "the piece index + 2 must fit the 4-bit limit field");
    uint32_t dp[M];
    bool clamp = false;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int64_t dg = ((int64_t)lim[m] - (int64_t)(chunk[m] & ~(uint64_t)15)) >> 4;
        dp[m] = dg >= 13 ? 15u : dg <= -2 ? 0u : (uint32_t)(dg + 2);
        clamp = clamp || dp[m] < 15u;
    }
    // the slot's chunk address (packed form when clamping), from its owner lane
    auto src_of = [&](int i, const uint32_t (&alo)[M], const uint32_t (&ahi)[M], uint32_t& piece) {
        const uint32_t g = (uint32_t)i * 64u + lane;
        const uint32_t slot = g / (uint32_t)P;
        piece = g - slot * (uint32_t)P;
        const uint32_t owner = slot & 63u, m = slot >> 6;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) {  // the slot's sub-index m is per lane: fetch each, keep one
            const uint32_t l = (uint32_t)__shfl((int)alo[k], (int)owner, 64), h = (uint32_t)__shfl((int)ahi[k], (int)owner, 64);
            if (M == 1 || m == (uint32_t)k) {
                lo = l;
                hi = h;
            }
        }
        return ((uint64_t)hi << 32) | lo;
    };
    uint32_t alo[M], ahi[M];
#ifdef SBFT_SHA_NOCLAMP  // A/B measurement only: the unclamped DMA (needs the blob padding)
    clamp = false;
#endif
    if (__any(clamp)) {  // wave-uniform
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const uint64_t ab = ((chunk[m] & ~(uint64_t)15) - 32) | dp[m];
            alo[m] = (uint32_t)ab;
            ahi[m] = (uint32_t)(ab >> 32);
        }
#pragma unroll
        for (int i = 0; i < M * P; ++i) {
            uint32_t piece;
            const uint64_t a = src_of(i, alo, ahi, piece);
            const uint32_t pe = min(piece + 2u, (uint32_t)a & 15u);
            const uint64_t src = (a & ~(uint64_t)15) + 16u * pe;
            __builtin_amdgcn_global_load_lds((gptr)(uintptr_t)src, (lptr)(buf + i * 1024), 16, 0, 0);
        }
    } else {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const uint64_t a = chunk[m] & ~(uint64_t)15;
            alo[m] = (uint32_t)a;
            ahi[m] = (uint32_t)(a >> 32);
        }
#pragma unroll
        for (int i = 0; i < M * P; ++i) {
            uint32_t piece;
            const uint64_t src = src_of(i, alo, ahi, piece) + 16u * piece;
            __builtin_amdgcn_global_load_lds((gptr)(uintptr_t)src, (lptr)(buf + i * 1024), 16, 0, 0);
        }
    }
}

__device__ __forceinline__ void sha_init(uint32_t (&h)[8]) {
    h[0] = 0x6a09e667;
    h[1] = 0xbb67ae85;
    h[2] = 0x3c6ef372;
    h[3] = 0xa54ff53a;
    h[4] = 0x510e527f;
    h[5] = 0x9b05688c;
    h[6] = 0x1f83d9ab;
    h[7] = 0x5be0cd19;
}

template <int C, int M, bool DB>
__global__ __launch_bounds__(256) void sha256_lds_kernel(const uint8_t* __restrict__ blob,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len,
                                                         const uint32_t* __restrict__ order,
                                                         uint8_t* __restrict__ dig, uint32_t n,
                                                         uint32_t* __restrict__ ctr) {
    using L = ShaLds<C, M, DB>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[L::LDS];
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint8_t* const wbuf = lds + wid * L::NBUF * L::BUF;
    const uint64_t blob0 = (uint64_t)(uintptr_t)blob;
    ShaQueue q;
    // this lane's M current messages: index, length, blocks, next block, start address, state
    bool act[M];
    uint32_t mi[M], ml[M], nb[M], b[M];
    uint64_t base[M], pf[M], pl[M];
    uint32_t h[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const uint32_t idx = q.take(true, lane, n, ctr);
        act[m] = idx < n;
        mi[m] = ml[m] = nb[m] = b[m] = 0;
        base[m] = blob0;
        if (act[m]) {
            mi[m] = order ? order[idx] : idx;
            ml[m] = len[mi[m]];
            base[m] = blob0 + off[mi[m]];
            nb[m] = sha256_nblocks(ml[m]);
        }
        sha_init(h[m]);
        pf[m] = base[m];
        pl[m] = sha_last_granule(base[m], ml[m], blob0);
    }
    sha_lds_fetch<C, M>(wbuf, pf, pl, lane);
    for (uint32_t t = 0;; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step t's rows have landed
        bool any = false;
#pragma unroll
        for (int m = 0; m < M; ++m) any = any || act[m];
        if (!__any(any)) break;
        const uint8_t* cur = wbuf + (DB ? (t & 1u) * L::BUF : 0);
        // messages that end in this step draw their successors now, so that step t+1's DMA
        // fetches them
        bool fin[M];
        uint32_t nidx[M], nmi[M], nml[M];
        uint64_t nbase[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            fin[m] = act[m] && b[m] + C >= nb[m];
            nidx[m] = q.take(fin[m], lane, n, ctr);
            nmi[m] = nml[m] = 0;
            nbase[m] = blob0;
            pf[m] = blob0;
            pl[m] = blob0 & ~(uint64_t)15;
            if (fin[m] && nidx[m] < n) {
                nmi[m] = order ? order[nidx[m]] : nidx[m];
                nml[m] = len[nmi[m]];
                nbase[m] += off[nmi[m]];
                pf[m] = nbase[m];
                pl[m] = sha_last_granule(nbase[m], nml[m], blob0);
            } else if (act[m] && !fin[m]) {
                pf[m] = base[m] + 64ull * (b[m] + C);
                pl[m] = sha_last_granule(base[m], ml[m], blob0);
            }
        }
        if (DB) sha_lds_fetch<C, M>(wbuf + ((t + 1u) & 1u) * L::BUF, pf, pl, lane);
#pragma unroll
        for (int j = 0; j < C; ++j) {
            uint32_t w[M][16];
            bool live[M];
#pragma unroll
            for (int m = 0; m < M; ++m) {
                // this message's row: bytes [o, o + 64 C) hold blocks b .. b + C - 1
                const uint32_t bi = b[m] + j;
                live[m] = act[m] && bi < nb[m];
                const uint32_t o = (uint32_t)base[m] & 15u;
                const uint32_t* row = reinterpret_cast<const uint32_t*>(cur + (m * 64u + lane) * L::ROW) + (o >> 2);
                const uint32_t sh = o & 3u;
                // v_perm_b32 selector: big-endian word of stream bytes sh .. sh + 3 of (hi:lo)
                const uint32_t sel = ((sh) << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
                uint32_t lo = row[16 * j];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t hi = row[16 * j + i + 1];
                    w[m][i] = __builtin_amdgcn_perm(hi, lo, sel);
                    lo = hi;
                }
                const uint32_t full = ml[m] >> 6;
                if (__builtin_expect(__any(live[m] && bi >= full), 0)) {
                    if (bi >= full) {
                        // the padded tail: rem data bytes, 0x80, zeros, the 64-bit bit length
                        const uint32_t rem = ml[m] & 63u;
                        const bool first = bi == full;
                        const uint32_t krem = first ? rem : 0;
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const uint32_t b0 = 4 * i;
                            uint32_t keep_mask;
                            if (b0 + 4 <= krem) keep_mask = 0xffffffffu;
                            else if (b0 >= krem) keep_mask = 0;
                            else keep_mask = 0xffffffffu << (8 * (4 - (krem - b0)));
                            uint32_t v = w[m][i] & keep_mask;
                            if (first && rem >= b0 && rem < b0 + 4) v |= 0x80u << (8 * (3 - (rem - b0)));
                            w[m][i] = v;
                        }
                        if (bi + 1 == nb[m]) {
                            const uint64_t bits = (uint64_t)ml[m] * 8;
                            w[m][14] = (uint32_t)(bits >> 32);
                            w[m][15] = (uint32_t)bits;
                        }
                    }
                }
            }
            bool any_live = false;
#pragma unroll
            for (int m = 0; m < M; ++m) any_live = any_live || live[m];
            if (any_live) compress_multi<M>(h, w, live);
        }
        if (!DB) sha_lds_fetch<C, M>(wbuf, pf, pl, lane);  // the step's reads are consumed: refill in place
#pragma unroll
        for (int m = 0; m < M; ++m) {
            if (fin[m]) {
                uint4* out = reinterpret_cast<uint4*>(dig + 32ull * mi[m]);
                out[0] = make_uint4(__builtin_bswap32(h[m][0]), __builtin_bswap32(h[m][1]), __builtin_bswap32(h[m][2]),
                                    __builtin_bswap32(h[m][3]));
                out[1] = make_uint4(__builtin_bswap32(h[m][4]), __builtin_bswap32(h[m][5]), __builtin_bswap32(h[m][6]),
                                    __builtin_bswap32(h[m][7]));
                act[m] = nidx[m] < n;
                mi[m] = nmi[m];
                ml[m] = nml[m];
                base[m] = nbase[m];
                b[m] = 0;
                nb[m] = sha256_nblocks(nml[m]);
                sha_init(h[m]);
            } else if (act[m]) {
                b[m] += C;
            }
        }
    }
}

// Framed tuples: message k's signature r || s is the 64 bytes at off[k] + len[k] + sig_rel
// of the blob and its public key x || y the 64 bytes at off[k] + len[k] + pub_rel. One thread
// per (message, 32-byte field) copies the field into the SoA verify inputs (byte loads: the
// fields are not aligned in the payload).
__global__ __launch_bounds__(256) void gather_framed_kernel(const uint8_t* __restrict__ blob,
                                                            const uint64_t* __restrict__ off,
                                                            const uint32_t* __restrict__ len, uint32_t n,
                                                            int32_t sig_rel, int32_t pub_rel,
                                                            uint8_t* __restrict__ r, uint8_t* __restrict__ s,
                                                            uint8_t* __restrict__ qx, uint8_t* __restrict__ qy,
                                                            uint32_t* zero0, uint32_t* zero1) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid == 0) {
        if (zero0) *zero0 = 0;
        if (zero1) *zero1 = 0;
    }
    if (gid >= 4u * n) return;
    const uint32_t k = gid >> 2, f = gid & 3u;
    const int64_t end = (int64_t)(off[k] + len[k]);
    const uint8_t* src = blob + end + (f < 2 ? sig_rel : pub_rel) + 32 * (f & 1u);
    uint8_t* dst = (f == 0 ? r : f == 1 ? s : f == 2 ? qx : qy) + 32ull * k;
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        w[j] = (uint32_t)src[4 * j] | ((uint32_t)src[4 * j + 1] << 8) | ((uint32_t)src[4 * j + 2] << 16) |
               ((uint32_t)src[4 * j + 3] << 24);
    uint4* d = reinterpret_cast<uint4*>(dst);
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// ------------------------------------------------------------ longest-first order
// Lanes hash whole messages from their wavefront's queue. Once the queue is empty, the lanes
// still inside long messages set the kernel's tail: a 64 KiB message is ~1,000 serial blocks,
// milliseconds at full occupancy. Taking the messages longest first (LPT) all but removes it.
// The order is a counting sort of the block counts, exact up to 1,023 blocks (64 KiB) and in
// eighth-octave classes above (lengths within a class differ by < 10%), longest first, in
// three small kernels. Config 5 (2M random 1-64 KiB messages, tools/sha_order_probe.py): index
// order 47.4 ms, quarter-octave classes 41.6 ms, an exact sort 39.7 ms.
#define SHA_LPT_CLASSES 1280u
__device__ __forceinline__ uint32_t lpt_class(uint32_t len) {
    const uint32_t nb = sha256_nblocks(len);  // 1 .. 2^26 + 1
    uint32_t key = nb;
    if (nb >= 1024u) {
        const uint32_t lg = 31u - (uint32_t)__builtin_clz(nb);  // 10 .. 26
        key = 1024u + 8u * (lg - 10u) + ((nb >> (lg - 3u)) & 7u);  // < 1160
    }
    return SHA_LPT_CLASSES - 1u - key;  // 0 = longest
}

// ws[0 .. C): class counts (zeroed by the launch), ws[C .. 2C): the classes' cursors
__global__ __launch_bounds__(256) void sha_lpt_count_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                            uint32_t* __restrict__ ws) {
    __shared__ uint32_t h[SHA_LPT_CLASSES];
    for (uint32_t c = threadIdx.x; c < SHA_LPT_CLASSES; c += blockDim.x) h[c] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&h[lpt_class(len[i])], 1u);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < SHA_LPT_CLASSES; c += blockDim.x)
        if (h[c]) atomicAdd(&ws[c], h[c]);
}

// one 256-thread workgroup: exclusive scan of the class counts into the cursors (each thread
// sums 5 consecutive classes, then a Hillis-Steele scan of the 256 partial sums)
__global__ __launch_bounds__(256) void sha_lpt_scan_kernel(uint32_t* __restrict__ ws) {
    constexpr uint32_t K = SHA_LPT_CLASSES / 256u;
    static_assert(SHA_LPT_CLASSES % 256u == 0, "classes per thread");
    __shared__ uint32_t v[256];
    const uint32_t t = threadIdx.x;
    uint32_t c[K], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        c[k] = ws[K * t + k];
        sum += c[k];
    }
    v[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 256u; off <<= 1) {
        const uint32_t x = t >= off ? v[t - off] : 0u;
        __syncthreads();
        v[t] += x;
        __syncthreads();
    }
    uint32_t run = v[t] - sum;  // exclusive prefix of this thread's first class
#pragma unroll
    for (uint32_t k = 0; k < K; ++k) {
        ws[SHA_LPT_CLASSES + K * t + k] = run;
        run += c[k];
    }
}

// Each workgroup places a chunk of 256 messages: class counts in LDS, one global reservation
// per class present, then each message takes the next slot of its class's range.
__global__ __launch_bounds__(256) void sha_lpt_place_kernel(const uint32_t* __restrict__ len, uint32_t n,
                                                            uint32_t* __restrict__ ws, uint32_t* __restrict__ order) {
    __shared__ uint32_t h[SHA_LPT_CLASSES], base[SHA_LPT_CLASSES];
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gridDim.x * blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        const uint32_t c = i < n ? lpt_class(len[i]) : 0u;
        h[c] = 0;  // only the classes this chunk uses need clearing
        __syncthreads();
        const uint32_t r = i < n ? atomicAdd(&h[c], 1u) : 0u;
        __syncthreads();
        if (i < n && r == 0) base[c] = atomicAdd(&ws[SHA_LPT_CLASSES + c], h[c]);  // one per class
        __syncthreads();
        if (i < n) order[base[c] + r] = i;
        __syncthreads();
    }
}

}  // namespace sbft

extern "C" size_t sbft_sha256_lpt_ws_bytes(void) { return 2 * SHA_LPT_CLASSES * sizeof(uint32_t); }

extern "C" int sbft_launch_sha256_lpt_order(const uint32_t* d_len, uint32_t n, uint32_t* d_ws, uint32_t* d_order,
                                            hipStream_t stream) {
    if (n == 0) return 0;
    if (hipMemsetAsync(d_ws, 0, SHA_LPT_CLASSES * sizeof(uint32_t), stream) != hipSuccess) return -1;
    const unsigned g = (unsigned)((n + 255) / 256), grid = g < 1024u ? g : 1024u;
    hipLaunchKernelGGL(sbft::sha_lpt_count_kernel, dim3(grid), dim3(256), 0, stream, d_len, n, d_ws);
    hipLaunchKernelGGL(sbft::sha_lpt_scan_kernel, dim3(1), dim3(256), 0, stream, d_ws);
    hipLaunchKernelGGL(sbft::sha_lpt_place_kernel, dim3(grid), dim3(256), 0, stream, d_len, n, d_ws, d_order);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sbft_launch_gather_framed(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                         uint32_t n, int32_t sig_rel, int32_t pub_rel, uint8_t* d_r, uint8_t* d_s,
                                         uint8_t* d_qx, uint8_t* d_qy, hipStream_t stream, uint32_t* zero0,
                                         uint32_t* zero1) {
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((4ull * n + 255) / 256);
    hipLaunchKernelGGL(sbft::gather_framed_kernel, dim3(blocks), dim3(256), 0, stream, d_blob, d_off, d_len, n,
                       sig_rel, pub_rel, d_r, d_s, d_qx, d_qy, zero0, zero1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sbft_launch_sha256(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                  const uint32_t* d_order, uint8_t* d_dig, uint32_t n, uint32_t* d_ctr,
                                  hipStream_t stream, int ctr_zeroed) {
    if (sbft_fault_hit(2)) return -1;  // SBFT_GV_FAULT_LAUNCH (tests only)
    if (n == 0) return 0;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    const unsigned threads = 256;
    const unsigned need = (n + threads - 1) / threads;
    if (!ctr_zeroed && hipMemsetAsync(d_ctr, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
    static int variant = -1;
    if (variant < 0) {
        // A/B measurement only: 0 the per-lane-load kernel; else the LDS-staged kernel with
        // (C blocks per step, M messages per lane, double-buffered) = 1: (1, 1, yes),
        // 2: (2, 1, yes), 3: (2, 1, no), 5: (1, 2, yes), 6: (1, 2, no), 7: (2, 2, no)
        const char* e = getenv("SBFT_SHA_VARIANT");
        variant = e ? atoi(e) : 2;
    }
    auto launch = [&](auto kern, int lds_bytes) {
        // persistent grid: the resident capacity (LDS-bound: 160 KiB per CU)
        const unsigned cap = (160u * 1024u / (unsigned)lds_bytes) * (unsigned)cus, blocks = need < cap ? need : cap;
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, stream, d_blob, d_off, d_len, d_order, d_dig, n,
                           d_ctr);
    };
    switch (variant) {
    case 0: {
        // persistent grid: the resident capacity (5 waves per SIMD at 82 VGPRs)
        const unsigned cap = 5u * (unsigned)cus, blocks = need < cap ? need : cap;
        hipLaunchKernelGGL(sbft::sha256_stream_kernel, dim3(blocks), dim3(threads), 0, stream, d_blob, d_off,
                           d_len, d_order, d_dig, n, d_ctr);
        break;
    }
    case 1: launch(sbft::sha256_lds_kernel<1, 1, true>, sbft::ShaLds<1, 1, true>::LDS); break;
    case 3: launch(sbft::sha256_lds_kernel<2, 1, false>, sbft::ShaLds<2, 1, false>::LDS); break;
    case 5: launch(sbft::sha256_lds_kernel<1, 2, true>, sbft::ShaLds<1, 2, true>::LDS); break;
    case 6: launch(sbft::sha256_lds_kernel<1, 2, false>, sbft::ShaLds<1, 2, false>::LDS); break;
    case 7: launch(sbft::sha256_lds_kernel<2, 2, false>, sbft::ShaLds<2, 2, false>::LDS); break;
    default: launch(sbft::sha256_lds_kernel<2, 1, true>, sbft::ShaLds<2, 1, true>::LDS); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
