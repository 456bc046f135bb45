// SHA-256 throughput experiments (diagnostics only).
// argv: lanes mode   mode 0: uniform 512 blocks, identity
//                    mode 1: random 16..1024 blocks, identity order
//                    mode 2: random, globally sorted by length (desc)
//                    mode 3: random, sorted within windows of 4096
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
#include "../smartbft_amd/csrc/sha256_dev.hpp"
using namespace sbft;

__global__ __launch_bounds__(256) void with_loads(uint32_t* out, const uint8_t* blob, const uint64_t* off,
                                                  const uint32_t* nb, const uint32_t* order, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t i = order[t];
    uint32_t h[8] = {1, 2, 3, 4, 5, 6, 7, 8};
    uint32_t w[16];
    const uint8_t* p = blob + off[i];
    const uint32_t blocks = nb[i];
    for (uint32_t b = 0; b < blocks; ++b) {
        load_block(p + 64 * b, w);
        compress(h, w);
    }
    out[i] = h[0] ^ h[7];
}
int main(int argc, char** argv) {
    const int lanes = atoi(argv[1]), mode = atoi(argv[2]), W = argc > 3 ? atoi(argv[3]) : 4096;
    std::mt19937 rng(5);
    std::vector<uint32_t> nb(lanes);
    for (auto& x : nb) x = mode == 0 ? 512 : 16 + rng() % 1009;
    std::vector<uint64_t> off(lanes);
    uint64_t at = 0;
    for (int i = 0; i < lanes; ++i) { off[i] = at; at += (uint64_t)nb[i] * 64 + 3; }
    std::vector<uint32_t> order(lanes);
    for (int i = 0; i < lanes; ++i) order[i] = i;
    auto bylen = [&](uint32_t a, uint32_t b) { return nb[a] > nb[b]; };
    if (mode == 2) std::stable_sort(order.begin(), order.end(), bylen);
    if (mode == 3)
        for (int i = 0; i < lanes; i += W) std::stable_sort(order.begin() + i, order.begin() + std::min(lanes, i + W), bylen);
    uint32_t* d; uint8_t* blob; uint64_t* doff; uint32_t *dnb, *dord;
    hipMalloc(&d, (size_t)lanes * 4);
    hipMalloc(&blob, at + 256);
    hipMemset(blob, 7, at + 256);
    hipMalloc(&doff, lanes * 8); hipMalloc(&dnb, lanes * 4); hipMalloc(&dord, lanes * 4);
    hipMemcpy(doff, off.data(), lanes * 8, hipMemcpyHostToDevice);
    hipMemcpy(dnb, nb.data(), lanes * 4, hipMemcpyHostToDevice);
    hipMemcpy(dord, order.data(), lanes * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float ms;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a); with_loads<<<(lanes + 255) / 256, 256>>>(d, blob, doff, dnb, dord, lanes); hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
    }
    printf("W %d lanes %d mode %d: ", W); printf("%.3f ms  %.1f GB/s (%.1f GB)\n", lanes, mode, ms, (double)at / ms / 1e6, at / 1e9);
    return 0;
}
