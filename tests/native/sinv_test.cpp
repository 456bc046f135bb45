// CPU build of smartbft_amd/csrc/sinv_host.hpp (the keyed path's host-side batch of s^-1) for
// tests/test_native.py: reads one s per line (64 hex digits, big-endian) as ONE batch, prints
// w = s^-1 2^256 mod n per line (8 little-endian 32-bit words, most significant first).
#include <cstdio>
#include <vector>

#include "../../smartbft_amd/csrc/sinv_host.hpp"

int main() {
    std::vector<uint8_t> s;
    char h[80];
    while (scanf("%64s", h) == 1) {
        for (int i = 0; i < 32; ++i) {
            unsigned v = 0;
            sscanf(h + 2 * i, "%2x", &v);
            s.push_back((uint8_t)v);
        }
    }
    const size_t n = s.size() / 32;
    std::vector<uint32_t> w(8 * n + 1);
    sbft::modn::sinv_batch_mont(s.data(), n, w.data());
    for (size_t i = 0; i < n; ++i) {
        for (int k = 7; k >= 0; --k) printf("%08x", w[8 * i + k]);
        printf("\n");
    }
    return 0;
}
