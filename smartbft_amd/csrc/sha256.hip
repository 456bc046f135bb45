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
template <int C, bool DB>
struct ShaLds {
    static constexpr int P = 4 * C + 1;       // 16-B pieces per slot row
    static constexpr int ROW = 16 * P;        // bytes per slot row
    static constexpr int BUF = 64 * ROW;      // one wavefront's step buffer
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

template <int C>
__device__ __forceinline__ void sha_lds_fetch(uint8_t* buf, uint64_t chunk, uint32_t lane) {
    typedef __attribute__((address_space(3))) void* lptr;
    typedef __attribute__((address_space(1))) void* gptr;
    constexpr int P = 4 * C + 1;
    const uint64_t a = chunk & ~(uint64_t)15;
    const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32);
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t g = (uint32_t)i * 64u + lane;
        const uint32_t slot = g / (uint32_t)P, piece = g - slot * (uint32_t)P;
        const uint32_t lo = (uint32_t)__shfl((int)alo, (int)slot, 64), hi = (uint32_t)__shfl((int)ahi, (int)slot, 64);
        const uint64_t src = (((uint64_t)hi << 32) | lo) + 16u * piece;
        __builtin_amdgcn_global_load_lds((gptr)(uintptr_t)src, (lptr)(buf + i * 1024), 16, 0, 0);
    }
}

template <int C, bool DB>
__global__ __launch_bounds__(256) void sha256_lds_kernel(const uint8_t* __restrict__ blob,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len,
                                                         const uint32_t* __restrict__ order,
                                                         uint8_t* __restrict__ dig, uint32_t n,
                                                         uint32_t* __restrict__ ctr) {
    using L = ShaLds<C, DB>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[L::LDS];
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint8_t* const wbuf = lds + wid * L::NBUF * L::BUF;
    ShaQueue q;
    // this lane's current message: start address, length, blocks, next block
    bool act = false;
    uint32_t mi = 0, ml = 0, nb = 0, b = 0;
    uint64_t base = (uint64_t)(uintptr_t)blob;
    uint32_t h[8];
    auto start = [&](uint32_t idx) {
        act = idx < n;
        if (!act) return;
        mi = order ? order[idx] : idx;
        ml = len[mi];
        base = (uint64_t)(uintptr_t)blob + off[mi];
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
    };
    start(q.take(true, lane, n, ctr));
    sha_lds_fetch<C>(wbuf, act ? base : (uint64_t)(uintptr_t)blob, lane);
    for (uint32_t t = 0;; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step t's rows have landed
        if (!__any(act)) break;
        const uint8_t* cur = wbuf + (DB ? (t & 1u) * L::BUF : 0);
        // lanes whose message ends in this step draw their next one now, so that step t+1's
        // DMA fetches it
        const bool fin = act && b + C >= nb;
        const uint32_t nidx = q.take(fin, lane, n, ctr);
        uint32_t nmi = 0, nml = 0;
        uint64_t nbase = (uint64_t)(uintptr_t)blob, pf = nbase;
        if (fin && nidx < n) {
            nmi = order ? order[nidx] : nidx;
            nml = len[nmi];
            nbase += off[nmi];
            pf = nbase;
        } else if (act && !fin) {
            pf = base + 64ull * (b + C);
        }
        if (DB) sha_lds_fetch<C>(wbuf + ((t + 1u) & 1u) * L::BUF, pf, lane);
        if (act) {
            // this lane's row: bytes [o, o + 64 C) hold blocks b .. b + C - 1
            const uint32_t o = (uint32_t)base & 15u;
            const uint32_t* row = reinterpret_cast<const uint32_t*>(cur + lane * L::ROW) + (o >> 2);
            const uint32_t sh = o & 3u;
            // v_perm_b32 selector: big-endian word of stream bytes sh .. sh + 3 of (hi:lo)
            const uint32_t sel = ((sh) << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
#pragma unroll
            for (int j = 0; j < C; ++j) {
                const uint32_t bi = b + j;
                if (bi < nb) {
                    uint32_t w[16];
                    uint32_t lo = row[16 * j];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t hi = row[16 * j + i + 1];
                        w[i] = __builtin_amdgcn_perm(hi, lo, sel);
                        lo = hi;
                    }
                    const uint32_t full = ml >> 6;
                    if (__builtin_expect(__any(bi >= full), 0)) {
                        if (bi >= full) {
                            const uint32_t rem = ml & 63u;
                            const bool first = bi == full;
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
                            if (bi + 1 == nb) {
                                const uint64_t bits = (uint64_t)ml * 8;
                                w[14] = (uint32_t)(bits >> 32);
                                w[15] = (uint32_t)bits;
                            }
                        }
                    }
                    compress(h, w);
                }
            }
        }
        if (!DB) sha_lds_fetch<C>(wbuf, pf, lane);  // the step's reads are consumed: refill in place
        if (fin) {
            uint4* out = reinterpret_cast<uint4*>(dig + 32ull * mi);
            out[0] = make_uint4(__builtin_bswap32(h[0]), __builtin_bswap32(h[1]), __builtin_bswap32(h[2]),
                                __builtin_bswap32(h[3]));
            out[1] = make_uint4(__builtin_bswap32(h[4]), __builtin_bswap32(h[5]), __builtin_bswap32(h[6]),
                                __builtin_bswap32(h[7]));
            act = false;
            if (nidx < n) {
                act = true;
                mi = nmi;
                ml = nml;
                base = nbase;
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
        } else if (act) {
            b += C;
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
                                                            uint8_t* __restrict__ qx, uint8_t* __restrict__ qy) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
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

}  // namespace sbft

extern "C" int sbft_launch_gather_framed(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                         uint32_t n, int32_t sig_rel, int32_t pub_rel, uint8_t* d_r, uint8_t* d_s,
                                         uint8_t* d_qx, uint8_t* d_qy, hipStream_t stream) {
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((4ull * n + 255) / 256);
    hipLaunchKernelGGL(sbft::gather_framed_kernel, dim3(blocks), dim3(256), 0, stream, d_blob, d_off, d_len, n,
                       sig_rel, pub_rel, d_r, d_s, d_qx, d_qy);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sbft_launch_sha256(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                  const uint32_t* d_order, uint8_t* d_dig, uint32_t n, uint32_t* d_ctr,
                                  hipStream_t stream) {
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
    if (hipMemsetAsync(d_ctr, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
    static int variant = -1;
    if (variant < 0) {
        // A/B measurement only: 0 the per-lane-load kernel; 1..4 the LDS-staged kernel with
        // (C blocks per step, double-buffered) = (1, yes), (2, yes), (2, no), (4, no)
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
    case 1: launch(sbft::sha256_lds_kernel<1, true>, sbft::ShaLds<1, true>::LDS); break;
    case 3: launch(sbft::sha256_lds_kernel<2, false>, sbft::ShaLds<2, false>::LDS); break;
    case 4: launch(sbft::sha256_lds_kernel<4, false>, sbft::ShaLds<4, false>::LDS); break;
    default: launch(sbft::sha256_lds_kernel<2, true>, sbft::ShaLds<2, true>::LDS); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
