// sha256.hip — batched SHA-256 (FIPS 180-4) over variable-length request payloads, gfx950.
//
// One message per lane; the lane streams its own payload block by block, so every
// 64-byte block it fetches is consumed whole (HBM traffic = payload bytes + 32 B digest).
// Arbitrary byte alignment: aligned dword loads are funnel-shifted with v_alignbyte. The
// host pads the device blob by >= 64 bytes so the funnel's one-dword over-read stays in
// bounds. Restated (independently) in oracle/p256_oracle.c oracle_sha256 for parity.
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
    // persistent grid: the resident capacity (5 waves per SIMD at 82 VGPRs), never more than the work
    const unsigned threads = 256;
    const unsigned need = (n + threads - 1) / threads, cap = 5u * (unsigned)cus;
    const unsigned blocks = need < cap ? need : cap;
    if (hipMemsetAsync(d_ctr, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
    hipLaunchKernelGGL(sbft::sha256_stream_kernel, dim3(blocks), dim3(threads), 0, stream, d_blob, d_off, d_len,
                       d_order, d_dig, n, d_ctr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
