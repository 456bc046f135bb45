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

// order (optional): lane i hashes message order[i]. With order sorted by length, the lanes of
// a wave walk messages of similar length, so no lane idles while its wave finishes a long one.
__global__ __launch_bounds__(256) void sha256_kernel(const uint8_t* __restrict__ blob,
                                                     const uint64_t* __restrict__ off,
                                                     const uint32_t* __restrict__ len,
                                                     const uint32_t* __restrict__ order,
                                                     uint8_t* __restrict__ dig, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t i = order ? order[t] : t;
    uint32_t h[8];
    sha256_one(blob + off[i], len[i], h);
    uint4* out = reinterpret_cast<uint4*>(dig + 32ull * i);
    out[0] = make_uint4(__builtin_bswap32(h[0]), __builtin_bswap32(h[1]), __builtin_bswap32(h[2]),
                        __builtin_bswap32(h[3]));
    out[1] = make_uint4(__builtin_bswap32(h[4]), __builtin_bswap32(h[5]), __builtin_bswap32(h[6]),
                        __builtin_bswap32(h[7]));
}

}  // namespace sbft

extern "C" int sbft_launch_sha256(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                  const uint32_t* d_order, uint8_t* d_dig, uint32_t n, hipStream_t stream) {
    if (n == 0) return 0;
    const unsigned threads = 256;
    const unsigned blocks = (n + threads - 1) / threads;
    hipLaunchKernelGGL(sbft::sha256_kernel, dim3(blocks), dim3(threads), 0, stream, d_blob, d_off, d_len,
                       d_order, d_dig, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
