// Pageable host-to-device copy of a proposal-sized payload (3.7 MB): one hipMemcpyAsync against
// the same bytes split over 2 or 4 threads, each on a stream of its own (the runtime stages a
// pageable copy through pinned buffers with a CPU memcpy). Diagnostics for VerifyProposal's
// payload copy. Prints median microseconds from the first submit to the last
// stream's completion.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

int main() {
    const size_t bytes = 3700000;
    std::vector<unsigned char> host(bytes);
    for (size_t i = 0; i < bytes; ++i) host[i] = (unsigned char)(i * 131u);
    void* dev;
    hipMalloc(&dev, bytes);
    hipStream_t st[4];
    for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int parts : {1, 2, 4, 1, 2, 4}) {
        std::vector<double> t;
        for (int rep = 0; rep < 60; ++rep) {
            // touch the source as a caller that just built the proposal would
            for (size_t i = 0; i < bytes; i += 4096) host[i] ^= 1;
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            const size_t chunk = (bytes + parts - 1) / parts;
            for (int p = 1; p < parts; ++p)
                th.emplace_back([&, p] {
                    const size_t a = p * chunk, n = std::min(bytes, a + chunk) - a;
                    hipMemcpyAsync((char*)dev + a, host.data() + a, n, hipMemcpyHostToDevice, st[p]);
                });
            hipMemcpyAsync(dev, host.data(), std::min(chunk, bytes), hipMemcpyHostToDevice, st[0]);
            for (auto& x : th) x.join();
            for (int p = 0; p < parts; ++p) hipStreamSynchronize(st[p]);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(t.begin(), t.end());
        printf("parts %d: median %.1f us, p10 %.1f, p90 %.1f\n", parts, t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    }
    return 0;
}
