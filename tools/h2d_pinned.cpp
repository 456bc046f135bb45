// Host-to-device copy of a proposal-sized payload (3.7 MB) from pageable memory: the runtime's
// own pageable hipMemcpyAsync against staging it ourselves -- T pool threads memcpy chunks of C
// bytes into page-locked memory and queue each chunk's DMA as soon as it is staged (one stream
// per thread). Diagnostics for VerifyProposal's payload copy. Prints the median
// microseconds from the submit to the last stream's completion.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

int main() {
    const size_t bytes = 3700000;
    std::vector<unsigned char> host(bytes);
    for (size_t i = 0; i < bytes; ++i) host[i] = (unsigned char)(i * 131u);
    unsigned char *pin = nullptr, *dev = nullptr;
    if (hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault) != hipSuccess || hipMalloc((void**)&dev, bytes) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    constexpr int kMaxT = 8;
    hipStream_t st[kMaxT];
    for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    // a spinning pool (a job = a generation number), as an engine's helper threads would be
    std::atomic<int> gen{0}, done{0}, quit{0};
    int T = 1;
    size_t C = bytes;
    std::vector<std::thread> pool;
    auto run = [&](bool pageable) {
        std::vector<double> t;
        for (int rep = 0; rep < 60; ++rep) {
            for (size_t i = 0; i < bytes; i += 4096) host[i] ^= 1;  // as a caller that just built it
            const auto t0 = std::chrono::steady_clock::now();
            if (pageable) {
                hipMemcpyAsync(dev, host.data(), bytes, hipMemcpyHostToDevice, st[0]);
                hipStreamSynchronize(st[0]);
            } else {
                done.store(0);
                gen.fetch_add(1, std::memory_order_acq_rel);
                while (done.load(std::memory_order_acquire) < kMaxT) {
                }
                for (int k = 0; k < T; ++k) hipStreamSynchronize(st[k]);
            }
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(t.begin(), t.end());
        return t;
    };
    auto start_pool = [&] {
    for (int t = 0; t < kMaxT; ++t)
        pool.emplace_back([&, t] {
            int seen = 0;
            for (;;) {
                int g;
                while ((g = gen.load(std::memory_order_acquire)) == seen)
                    if (quit.load()) return;
                seen = g;
                if (t < T) {
                    const size_t nch = (bytes + C - 1) / C;
                    for (size_t c = t; c < nch; c += T) {
                        const size_t a = c * C, n = std::min(bytes, a + C) - a;
                        std::memcpy(pin + a, host.data() + a, n);
                        hipMemcpyAsync(dev + a, pin + a, n, hipMemcpyHostToDevice, st[t]);
                    }
                }
                done.fetch_add(1, std::memory_order_acq_rel);
            }
        });
    };
    auto t0 = run(true);  // before the (spinning) pool exists
    printf("pageable: median %.1f us, p10 %.1f, p90 %.1f\n", t0[30], t0[6], t0[54]);
    start_pool();
    for (int round = 0; round < 2; ++round) {
        std::vector<double> t;
        for (int tt : {1, 2, 4, 8})
            for (size_t cc : {(size_t)262144, (size_t)524288, (size_t)1048576}) {
                T = tt;
                C = cc;
                t = run(false);
                printf("pinned T=%d C=%zu: median %.1f us, p10 %.1f, p90 %.1f\n", tt, cc, t[30], t[6], t[54]);
            }
    }
    quit.store(1);
    gen.fetch_add(1);
    for (auto& th : pool) th.join();
    t0 = run(true);
    printf("pageable: median %.1f us, p10 %.1f, p90 %.1f\n", t0[30], t0[6], t0[54]);
    return 0;
}
