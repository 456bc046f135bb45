// config2_harness.cpp — BASELINE config 2 (1M synthetic P-256 verifies, ~10% corrupted, distinct
// keys, device-resident) through the C ABI alone, on the HIP runtime the engine ships with
// (/opt/rocm's libamdhip64, as a cgo deployment loads it: go/gpuverify/verifier.go), with no torch
// in the process. bench.py's headline runs inside a torch process, whose own libamdhip64 the
// engine then binds to; this is the same measurement without it. Measurement
// tooling, not product code.
//
//   config2_harness N STEPS WARMUP
//
// The workload follows smartbft_amd/workload.py: d_i = SHA-256(seed|"key"|le64 i) mod n,
// m_i = SHA-256(seed|"msg"|i) || SHA-256(seed|"ms2"|i), e_i = SHA-256(m_i), k_i = SHA-256(seed|"k"|i)
// mod n, signed by the engine's signer; corrupted iff SHA-256(seed|"c"|i)[0] < 26, kind i mod 7
// (flip an r / s / e bit, r = 0, s = n, Q off-curve, the neighbour's key). Hashes and signatures
// come from the engine's own kernels (host-buffer calls); the five SoA arrays are copied to HBM
// once (engine-independent hipMalloc), then STEPS calls of sbft_gv_verify_p256_dev on one stream
// are timed (wall clock over the synchronised loop, and HIP events around the verify kernel via
// sbft_gv_kernel_timing). Parity: verdict == not corrupted for every tuple. Prints one JSON line.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <set>
#include <string>
#include <vector>

#include "../include/sbft_gpuverify.h"

static const uint8_t kN[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0x00, 0x00, 0x00, 0x00, 0xFF, 0xFF, 0xFF,
                               0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xBC, 0xE6, 0xFA, 0xAD, 0xA7, 0x17,
                               0x9E, 0x84, 0xF3, 0xB9, 0xCA, 0xC2, 0xFC, 0x63, 0x25, 0x51};

#define CHK(x)                                                                       \
    do {                                                                             \
        int rc_ = (int)(x);                                                          \
        if (rc_) {                                                                   \
            std::fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

// SHA-256 of seed|tag|le64(i) for i in [0, n), on the engine (host-buffer call)
static int tag_sha(sbft_gv_ctx* ctx, const char* tag, size_t n, std::vector<uint8_t>& out) {
    const std::string head = std::string("SBFT-GPUV-1") + tag;
    const size_t w = head.size() + 8;
    std::vector<uint8_t> blob(n * w + SBFT_GV_SHA_BLOB_PAD);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n, (uint32_t)w);
    for (size_t i = 0; i < n; ++i) {
        std::memcpy(&blob[i * w], head.data(), head.size());
        const uint64_t le = i;  // little-endian host
        std::memcpy(&blob[i * w + head.size()], &le, 8);
        off[i] = i * w;
    }
    out.resize(32 * n);
    return sbft_gv_sha256(ctx, blob.data(), n * w, off.data(), len.data(), n, out.data());
}

static bool ge_n(const uint8_t* x) {
    for (int k = 0; k < 32; ++k)
        if (x[k] != kN[k]) return x[k] > kN[k];
    return true;
}
static void reduce_mod_n(uint8_t* x) {  // x - n when x >= n (probability ~2^-32)
    if (!ge_n(x)) return;
    int borrow = 0;
    for (int k = 31; k >= 0; --k) {
        const int d = (int)x[k] - (int)kN[k] - borrow;
        x[k] = (uint8_t)(d & 0xFF);
        borrow = d < 0;
    }
}

static std::vector<std::string> mapped_runtime() {
    std::set<std::string> libs;
    std::ifstream f("/proc/self/maps");
    std::string line;
    while (std::getline(f, line)) {
        const size_t p = line.find('/');
        if (p != std::string::npos && line.find("libamdhip64") != std::string::npos) libs.insert(line.substr(p));
    }
    return {libs.begin(), libs.end()};
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? (size_t)std::atol(argv[1]) : 1000000;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 20;
    const int warmup = argc > 3 ? std::atoi(argv[3]) : 3;
    sbft_gv_opts o{};
    o.device_mask = 1;
    sbft_gv_ctx* ctx = nullptr;
    CHK(sbft_gv_init(&o, &ctx));
    std::vector<uint8_t> d, k, m1, m2, c;
    CHK(tag_sha(ctx, "key", n, d));
    CHK(tag_sha(ctx, "k", n, k));
    CHK(tag_sha(ctx, "msg", n, m1));
    CHK(tag_sha(ctx, "ms2", n, m2));
    CHK(tag_sha(ctx, "c", n, c));
    for (size_t i = 0; i < n; ++i) {
        reduce_mod_n(&d[32 * i]);
        reduce_mod_n(&k[32 * i]);
    }
    std::vector<uint8_t> msg(64 * n + SBFT_GV_SHA_BLOB_PAD), e(32 * n);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n, 64);
    for (size_t i = 0; i < n; ++i) {
        std::memcpy(&msg[64 * i], &m1[32 * i], 32);
        std::memcpy(&msg[64 * i + 32], &m2[32 * i], 32);
        off[i] = 64 * i;
    }
    CHK(sbft_gv_sha256(ctx, msg.data(), 64 * n, off.data(), len.data(), n, e.data()));
    std::vector<uint8_t> qx(32 * n), qy(32 * n), r(32 * n), s(32 * n), st(n);
    CHK(sbft_gv_sign_p256(ctx, d.data(), k.data(), e.data(), n, qx.data(), qy.data(), r.data(), s.data(), st.data()));
    for (size_t i = 0; i < n; ++i)
        if (st[i] != 1) {
            std::fprintf(stderr, "signer rejected tuple %zu\n", i);
            return 1;
        }
    // corruption, in workload.py's order: kinds 0-5, then kind 6 from the keys as they are then
    std::vector<uint8_t> expect(n, 1);
    std::vector<size_t> swap;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* ci = &c[32 * i];
        if (ci[0] >= 26) continue;
        expect[i] = 0;
        const int kind = (int)(i % 7), byte = ci[1] % 32;
        const uint8_t bit = (uint8_t)(1u << (ci[2] % 8));
        switch (kind) {
        case 0: r[32 * i + byte] ^= bit; break;
        case 1: s[32 * i + byte] ^= bit; break;
        case 2: e[32 * i + byte] ^= bit; break;
        case 3: std::memset(&r[32 * i], 0, 32); break;
        case 4: std::memcpy(&s[32 * i], kN, 32); break;
        case 5: qy[32 * i + 31] ^= 1; break;
        default: swap.push_back(i); break;
        }
    }
    {
        const std::vector<uint8_t> qx0 = qx, qy0 = qy;
        for (size_t i : swap) {
            const size_t nb = (i + 1) % n;
            std::memcpy(&qx[32 * i], &qx0[32 * nb], 32);
            std::memcpy(&qy[32 * i], &qy0[32 * nb], 32);
        }
    }
    // HBM-resident inputs, staged once
    CHK(hipSetDevice(0));
    uint8_t* dev = nullptr;
    CHK(hipMalloc((void**)&dev, 5 * 32 * n + n));
    uint8_t *dd = dev, *dr = dd + 32 * n, *ds = dr + 32 * n, *dqx = ds + 32 * n, *dqy = dqx + 32 * n, *dok = dqy + 32 * n;
    CHK(hipMemcpy(dd, e.data(), 32 * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dr, r.data(), 32 * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(ds, s.data(), 32 * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dqx, qx.data(), 32 * n, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dqy, qy.data(), 32 * n, hipMemcpyHostToDevice));
    hipStream_t stream;
    CHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (int w = 0; w < warmup; ++w) CHK(sbft_gv_verify_p256_dev(ctx, 0, dd, dr, ds, dqx, dqy, n, dok, stream));
    CHK(hipStreamSynchronize(stream));
    std::vector<uint8_t> ok(n);
    CHK(hipMemcpy(ok.data(), dok, n, hipMemcpyDeviceToHost));
    size_t mism = 0, accepts = 0;
    for (size_t i = 0; i < n; ++i) {
        mism += ok[i] != expect[i];
        accepts += expect[i];
    }
    CHK(sbft_gv_kernel_timing(ctx, 1));
    uint64_t nl = 0;
    double kms = 0;
    CHK(sbft_gv_kernel_time(ctx, &nl, &kms));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    CHK(hipEventRecord(e0, stream));
    for (int i = 0; i < steps; ++i) CHK(sbft_gv_verify_p256_dev(ctx, 0, dd, dr, ds, dqx, dqy, n, dok, stream));
    CHK(hipEventRecord(e1, stream));
    CHK(hipStreamSynchronize(stream));
    const double wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    float ev_ms = 0;
    CHK(hipEventElapsedTime(&ev_ms, e0, e1));
    CHK(sbft_gv_kernel_time(ctx, &nl, &kms));
    CHK(hipMemcpy(ok.data(), dok, n, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) mism += ok[i] != expect[i];
    std::string rt = "[";
    for (const auto& p : mapped_runtime()) rt += (rt.size() > 1 ? ", \"" : "\"") + p + "\"";
    rt += "]";
    std::printf("{\"mode\": \"config2\", \"n\": %zu, \"steps\": %d, \"warmup\": %d, \"verifies_per_s\": %.1f, "
                "\"ms_per_step\": %.4f, \"stream_events_ms_per_step\": %.4f, \"avg_kernel_ms\": %.4f, "
                "\"kernel_launches\": %llu, \"expected_accepts\": %zu, \"mismatches\": %zu, \"hip_runtime\": %s}\n",
                n, steps, warmup, (double)n * steps / wall_s, wall_s * 1e3 / steps, ev_ms / steps,
                nl ? kms / (double)nl : 0.0, (unsigned long long)nl, accepts, mism, rt.c_str());
    (void)hipFree(dev);
    sbft_gv_destroy(ctx);
    return mism ? 2 : 0;
}
