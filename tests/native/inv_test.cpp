// CPU build of smartbft_amd/csrc/p256_inv.hpp (the device inversion) for tests/test_native.py:
// reads hex x per line on stdin, prints hex x^-1 mod n (argument "p": mod the field prime;
// "nR": 2^256 x^-1 mod n, the scaled form the keyed kernel takes).
#include <cstdio>
#include <cstring>

#include "../../smartbft_amd/csrc/p256_inv.hpp"

static const uint32_t TAB[SBFT_DIVSTEP5_WORDS] = SBFT_DIVSTEP5_TABLE;

int main(int argc, char** argv) {
    const bool modp = argc > 1 && std::strcmp(argv[1], "p") == 0;
    const bool scaled = argc > 1 && std::strcmp(argv[1], "nR") == 0;
    // 2^256 mod n, little-endian words
    const uint32_t RN[8] = {0x039cdaafu, 0x0c46353du, 0x58e8617bu, 0x43190552u,
                            0x00000000u, 0x00000000u, 0xffffffffu, 0x00000000u};
    char line[256];
    while (fgets(line, sizeof line, stdin)) {
        uint32_t x[8] = {0}, out[8];
        size_t L = strcspn(line, "\r\n");
        line[L] = 0;
        // big-endian hex, 64 digits
        for (int w = 0; w < 8; ++w) {
            unsigned v = 0;
            sscanf(line + 8 * (7 - w), "%8x", &v);
            x[w] = v;
        }
        if (modp)
            sbft::inv::inv_mod_p(out, x, TAB);
        else if (scaled)
            sbft::inv::inv_mod_n_scaled(out, x, RN, TAB);
        else
            sbft::inv::inv_mod_n(out, x, TAB);
        for (int w = 7; w >= 0; --w) printf("%08x", out[w]);
        printf("\n");
    }
    return 0;
}
