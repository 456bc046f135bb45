// CPU build of smartbft_amd/csrc/modn_host.hpp (the pooled signer's host arithmetic) for
// tests/test_native.py: reads "a b" (64 hex digits each, big-endian) per line, prints
// "a*b mod n" and "a+b mod n".
#include <cstdio>
#include <cstring>

#include "../../smartbft_amd/csrc/modn_host.hpp"

static void hex_to_be(const char* h, uint8_t out[32]) {
    for (int i = 0; i < 32; ++i) {
        unsigned v = 0;
        sscanf(h + 2 * i, "%2x", &v);
        out[i] = (uint8_t)v;
    }
}

int main() {
    char a[80], b[80];
    while (scanf("%64s %64s", a, b) == 2) {
        uint8_t ab[32], bb[32], o1[32], o2[32];
        hex_to_be(a, ab);
        hex_to_be(b, bb);
        sbft::modn::u64 x[4], y[4], p[4], s[4];
        sbft::modn::from_be32(x, ab);
        sbft::modn::from_be32(y, bb);
        sbft::modn::mul_mod(p, x, y);
        sbft::modn::add_mod(s, x, y);
        sbft::modn::to_be32(o1, p);
        sbft::modn::to_be32(o2, s);
        for (int i = 0; i < 32; ++i) printf("%02x", o1[i]);
        printf(" ");
        for (int i = 0; i < 32; ++i) printf("%02x", o2[i]);
        printf("\n");
    }
    return 0;
}
