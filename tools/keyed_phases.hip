// Phase timeline of the keyed wave kernel (p256_keyed.hip, the VerifyConsenterSig latency path):
// includes the kernel source with SBFT_KEYED_MARK recording s_memtime / s_memrealtime on lane 0
// of workgroup 0, signs a message with the GPU signer over G's comb table, builds the signer's
// key table, and prints where the launch's time goes. Diagnostics only (not the product build).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__device__ unsigned long long g_mark_clk[16];
__device__ unsigned long long g_mark_wall[16];
#define SBFT_KEYED_MARK(i)                                  \
    do {                                                    \
        if (threadIdx.x == 0 && blockIdx.x == 0) {          \
            g_mark_clk[i] = clock64();                      \
            g_mark_wall[i] = wall_clock64();                \
        }                                                   \
    } while (0)
#include "../smartbft_amd/csrc/p256_keyed.hip"
// the engine's test-only fault injection lives in gpuverify.cpp, which this tool does not link
extern "C" int sbft_fault_hit(int) { return 0; }

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

static void be_from_hex(uint8_t* out, const char* hex) {
    for (int i = 0; i < 32; ++i) sscanf(hex + 2 * i, "%2hhx", &out[i]);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 67;
    uint8_t gx[32], gy[32];
    be_from_hex(gx, "6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296");
    be_from_hex(gy, "4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5");
    const size_t tb = sbft_comb_table_bytes();
    void *gtab, *qtab;
    CHK(hipMalloc(&gtab, tb));
    CHK(hipMalloc(&qtab, tb));
    uint8_t* dbuf;
    CHK(hipMalloc(&dbuf, 1 << 20));
    uint32_t* dst;
    CHK(hipMalloc(&dst, 64));
    // G's table
    CHK(hipMemcpy(dbuf, gx, 32, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dbuf + 32, gy, 32, hipMemcpyHostToDevice));
    if (sbft_launch_comb_build(dbuf, dbuf + 32, gtab, dst, 1, 0)) return 1;
    CHK(hipDeviceSynchronize());
    void** keytab;
    CHK(hipMalloc(&keytab, 2 * sizeof(void*)));
    void* kt[2] = {gtab, qtab};
    CHK(hipMemcpy(keytab, kt, sizeof(kt), hipMemcpyHostToDevice));
    // sign n digests with one private key d (nonces k_i), on the GPU
    std::vector<uint8_t> d(32 * n), k(32 * n), e(32 * n);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint8_t)x; };
    uint8_t dk[32];
    for (int i = 0; i < 32; ++i) dk[i] = rnd();
    dk[0] &= 0x7f;
    for (int t = 0; t < n; ++t) {
        memcpy(&d[32 * t], dk, 32);
        for (int i = 0; i < 32; ++i) k[32 * t + i] = rnd(), e[32 * t + i] = rnd();
        k[32 * t] &= 0x7f;
    }
    uint8_t *dd = dbuf, *dkk = dbuf + 32 * n, *de = dbuf + 64 * n, *o = dbuf + 96 * n;
    CHK(hipMemcpy(dd, d.data(), 32 * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dkk, k.data(), 32 * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(de, e.data(), 32 * n, hipMemcpyHostToDevice));
    uint8_t *qx = o, *qy = o + 32 * n, *r = o + 64 * n, *s = o + 96 * n, *st = o + 128 * n;
    if (sbft_launch_p256_sign_wave(dd, dkk, de, (const void* const*)keytab, qx, qy, r, s, st, n, 0)) return 1;
    CHK(hipDeviceSynchronize());
    if (sbft_launch_comb_build(qx, qy, qtab, dst, 1, 0)) return 1;
    std::vector<uint32_t> key(n, 1u);
    uint32_t* dkey = (uint32_t*)(o + 160 * n + 256);
    uint8_t* dok = (uint8_t*)(dkey + n + 64);
    CHK(hipMemcpy(dkey, key.data(), 4 * n, hipMemcpyHostToDevice));
    CHK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    unsigned long long clk[16], wall[16], bclk[16] = {}, bwall[16] = {};
    for (int rep = 0; rep < 20; ++rep) {
        CHK(hipEventRecord(a));
        if (sbft_launch_p256_verify_keyed(de, nullptr, nullptr, nullptr, r, s, dkey, (const void* const*)keytab, 2,
                                          dok, n, 0, nullptr, 0))
            return 1;
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        CHK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_mark_clk), sizeof(clk)));
        CHK(hipMemcpyFromSymbol(wall, HIP_SYMBOL(g_mark_wall), sizeof(wall)));
        if (ms < best) {
            best = ms;
            memcpy(bclk, clk, sizeof(clk));
            memcpy(bwall, wall, sizeof(wall));
        }
    }
    std::vector<uint8_t> ok(n);
    CHK(hipMemcpy(ok.data(), dok, n, hipMemcpyDeviceToHost));
    int acc = 0;
    for (int t = 0; t < n; ++t) acc += ok[t];
    printf("n=%d accepted=%d/%d kernel(event) best %.1f us\n", n, acc, n, best * 1e3);
    const char* names[] = {"start",        "divstep table staged", "s^-1 (wave 1) + barrier", "u1, u2",
                           "table entry loaded", "butterfly level 0 (affine pair)", "levels 1-5 (quad)",
                           "final x == r check"};
    for (int i = 1; i < 8; ++i)
        printf("  %-34s %8llu cycles %7.2f us\n", names[i], bclk[i] - bclk[i - 1], (bwall[i] - bwall[i - 1]) / 100.0);
    printf("  %-34s %8llu cycles %7.2f us\n", "total (mark 0 -> 7)", bclk[7] - bclk[0], (bwall[7] - bwall[0]) / 100.0);
    return acc == n ? 0 : 2;
}
