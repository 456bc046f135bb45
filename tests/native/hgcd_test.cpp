// CPU build of smartbft_amd/csrc/p256_halfgcd.hpp (the latency kernel's half-size scalars) for
// tests/test_native.py: reads hex u per line on stdin, prints "1 w v neg" (hex w, hex |v|,
// 0/1) or "0" when the reduction gave up (the kernel's classic fallback).
#include <cstdio>
#include <cstring>

#include "../../smartbft_amd/csrc/p256_halfgcd.hpp"

int main() {
    char line[256];
    while (fgets(line, sizeof line, stdin)) {
        uint32_t u[8] = {0}, w[8], v[8];
        size_t L = strcspn(line, "\r\n");
        line[L] = 0;
        for (int k = 0; k < 8; ++k) {
            unsigned x = 0;
            sscanf(line + 8 * (7 - k), "%8x", &x);
            u[k] = x;
        }
        bool neg = false;
        if (!sbft::hgcd::half_gcd(u, w, v, neg)) {
            printf("0\n");
            continue;
        }
        printf("1 ");
        for (int k = 7; k >= 0; --k) printf("%08x", w[k]);
        printf(" ");
        for (int k = 7; k >= 0; --k) printf("%08x", v[k]);
        printf(" %d\n", neg ? 1 : 0);
    }
    return 0;
}
