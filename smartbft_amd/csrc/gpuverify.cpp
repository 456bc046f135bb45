// gpuverify.cpp — host runtime behind include/sbft_gpuverify.h (libsbft_gpuverify.so).
//
// One slot per selected HIP device: a non-blocking stream and device staging grown on
// demand. A host-buffer call splits its batch into contiguous chunks, one per device
// (no collective: every tuple is independent), enqueues H2D -> kernel(s)
// -> D2H on each device's stream, then synchronises all of them. Small batches (below
// min_split) stay on one device, picked round-robin so concurrent quorum-sized calls from
// different goroutines spread over the GPUs. Calls on one slot are serialised by its mutex.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <new>
#include <pthread.h>
#include <vector>

#include "../../include/sbft_gpuverify.h"
#include "engine_internal.h"
#include "sinv_host.hpp"
#include "sbft_kernels.h"

static inline void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
}

// ---- test-only fault injection (sbft_gv_inject_fault) ----
// The armed kind fires at its fault points: the staging allocations (NOMEM), the kernel launchers
// (LAUNCH: they return failure before launching) and the checked stream synchronisations after the
// work has drained (SYNC), so every injected failure leaves the device quiescent, as a real
// allocation or launch failure would. left > 0 counts down, < 0 fires until disarmed.
static std::atomic<int> g_fault_kind{SBFT_GV_FAULT_OFF};
static std::atomic<int> g_fault_left{0};
extern "C" __attribute__((visibility("hidden"))) int sbft_fault_hit(int kind) {
    if (g_fault_kind.load(std::memory_order_relaxed) != kind) return 0;
    int left = g_fault_left.load(std::memory_order_relaxed);
    for (;;) {
        if (left < 0) return 1;
        if (left == 0) return 0;
        if (g_fault_left.compare_exchange_weak(left, left - 1)) return 1;
    }
}
// hipStreamSynchronize, then the SYNC fault point (the stream has drained either way)
static hipError_t stream_sync(hipStream_t st) {
    const hipError_t e = hipStreamSynchronize(st);
    return (e == hipSuccess && sbft_fault_hit(SBFT_GV_FAULT_SYNC)) ? hipErrorUnknown : e;
}
#define NOMEM_POINT()                                              \
    do {                                                           \
        if (sbft_fault_hit(SBFT_GV_FAULT_NOMEM)) return SBFT_GV_ENOMEM; \
    } while (0)

namespace {

// One helper thread per context for host work that can overlap a caller's PCIe copy (the
// proposal parse of sbft_gv_framed_overlapped). A submitted job runs at once if the helper is
// idle; a second concurrent caller finds it busy and runs its job inline. After a job the
// helper spins ~2 ms before sleeping, so back-to-back proposals do not pay a wake-up.
struct Helper {
    std::mutex mu;
    std::condition_variable cv;
    std::thread th;
    std::function<void()> job;
    std::atomic<int> state{0};  // 0 idle, 1 job queued, 2 job done
    std::atomic<bool> busy{false};
    bool stop = false;

    void loop() {
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            while (state.load(std::memory_order_acquire) != 1 &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2))
                std::this_thread::yield();
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || state.load() == 1; });
                if (stop) return;
                f = std::move(job);
            }
            f();
            state.store(2, std::memory_order_release);
        }
    }
    // false: the helper is busy with another caller's job (run it inline instead)
    bool try_submit(std::function<void()> f) {
        bool expect = false;
        if (!busy.compare_exchange_strong(expect, true)) return false;
        {
            std::lock_guard<std::mutex> g(mu);
            if (!th.joinable()) th = std::thread([this] {
                pthread_setname_np(pthread_self(), "sbft-helper");  // per-thread CPU accounting
                loop();
            });
            job = std::move(f);
            state.store(1, std::memory_order_release);
        }
        cv.notify_one();
        return true;
    }
    void wait() {
        while (state.load(std::memory_order_acquire) != 2) std::this_thread::yield();
        state.store(0);
        busy.store(false);
    }
    ~Helper() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_one();
        if (th.joinable()) th.join();
    }
};

// Persistent host workers that drive the shares of a split batch: share i >= 1 of every call
// runs on worker i (started on first use, kept for the context's life), share 0 on the
// calling thread. A worker job only enqueues on, and synchronises, its own slot; it never waits
// for another worker, so concurrent split calls queue per worker and cannot deadlock.
struct Workers {
    struct W {
        std::mutex mu;
        std::condition_variable cv;
        std::vector<std::function<void()>> q;
        std::thread th;
        bool stop = false;
        void loop() {
            for (;;) {
                std::vector<std::function<void()>> jobs;
                {
                    std::unique_lock<std::mutex> g(mu);
                    cv.wait(g, [&] { return stop || !q.empty(); });
                    if (q.empty()) return;  // stop, nothing left
                    jobs.swap(q);
                }
                for (auto& f : jobs) f();
            }
        }
    };
    std::mutex mu;  // guards w's growth
    std::vector<std::unique_ptr<W>> w;
    void post(size_t i, std::function<void()> f) {
        W* x;
        {
            std::lock_guard<std::mutex> g(mu);
            while (w.size() <= i) w.emplace_back(new W());
            x = w[i].get();
            std::lock_guard<std::mutex> gx(x->mu);
            if (!x->th.joinable()) x->th = std::thread([x] {
                pthread_setname_np(pthread_self(), "sbft-share");
                x->loop();
            });
        }
        {
            std::lock_guard<std::mutex> gx(x->mu);
            x->q.push_back(std::move(f));
        }
        x->cv.notify_one();
    }
    ~Workers() {
        for (auto& x : w) {
            {
                std::lock_guard<std::mutex> g(x->mu);
                x->stop = true;
            }
            x->cv.notify_one();
            if (x->th.joinable()) x->th.join();
        }
    }
};

struct Workspace {
    void* ptr = nullptr;
    size_t cap = 0;
};

struct Slot {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    uint8_t* dbuf = nullptr;
    size_t dcap = 0;
    // verify workspaces of the device-resident entry points, one per caller stream (work on
    // one stream is ordered, so a stream never races with itself on its workspace)
    std::mutex ws_mu;
    std::map<hipStream_t, Workspace> ws;

    uint32_t* stream_workspace(hipStream_t st, size_t bytes) {
        if (sbft_fault_hit(SBFT_GV_FAULT_NOMEM)) return nullptr;
        std::lock_guard<std::mutex> g(ws_mu);
        Workspace& w = ws[st];
        if (w.cap < bytes) {
            if (w.ptr) {
                // the stream may still be using the old buffer
                if (hipStreamSynchronize(st) != hipSuccess) return nullptr;
                if (hipFree(w.ptr) != hipSuccess) return nullptr;
            }
            w.ptr = nullptr;
            w.cap = 0;
            const size_t want = std::max(bytes, (size_t)1 << 16);
            if (hipMalloc(&w.ptr, want) != hipSuccess) return nullptr;
            w.cap = want;
        }
        return (uint32_t*)w.ptr;
    }

    // registered-key comb tables (p256_keyed.hip): comb[id] is key id's table on this device,
    // comb[0] the generator's; d_keytab mirrors comb for the kernels. Tables never move; a
    // grown pointer array retires the old one only at destroy (kernels may still read it).
    std::vector<void*> comb;        // per key id (nullptr for an invalid key)
    std::vector<void*> comb_alloc;  // the allocations holding them (one per build batch)
    void** d_keytab = nullptr;
    size_t keytab_cap = 0;
    std::vector<void*> retired;
    // copy stream, second compute stream and per-sub-batch events of the pinned-input
    // pipeline (enqueue_verify_piped)
    hipStream_t copy_stream = nullptr;
    hipStream_t stream2 = nullptr;
    std::vector<hipEvent_t> sub_ev;
    int reserve_pipe(size_t subs) {
        if (!copy_stream && hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking) != hipSuccess) {
            copy_stream = nullptr;
            return SBFT_GV_EDEVICE;
        }
        if (!stream2 && hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking) != hipSuccess) {
            stream2 = nullptr;
            return SBFT_GV_EDEVICE;
        }
        while (sub_ev.size() < subs) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return SBFT_GV_EDEVICE;
            sub_ev.push_back(e);
        }
        return SBFT_GV_OK;
    }
    // pinned host staging for the small-batch (latency) path: one H2D and one D2H per call
    uint8_t* pin = nullptr;
    size_t pin_cap = 0;
    // mapped, coherent (fine-grained) host memory for the zero-copy keyed path: the kernel
    // reads its inputs and writes its verdicts here over PCIe (enqueue_keyed). Several lanes,
    // each with its own stream and buffer and lock, and none holds `mu`: concurrent small
    // batches (the consenter coalescer's back-to-back batches, quorum calls of different
    // decisions) run side by side on the device instead of queueing behind one another.
    struct ZcLane {
        std::mutex mu;
        hipStream_t stream = nullptr;
        // recorded after each launch; created with hipEventBlockingSync, so a caller that has
        // spun its budget waits for the kernel asleep (interrupt), not on a core
        hipEvent_t done = nullptr;
        uint8_t* host = nullptr;
        uint8_t* dev = nullptr;
        size_t cap = 0;
        // caller holds mu and has selected the slot's device
        int reserve(size_t bytes) {
            NOMEM_POINT();
            if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
                stream = nullptr;
                return SBFT_GV_EDEVICE;
            }
            if (!done && hipEventCreateWithFlags(&done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess) {
                done = nullptr;
                return SBFT_GV_EDEVICE;
            }
            if (bytes <= cap) return SBFT_GV_OK;
            if (host) {
                (void)hipStreamSynchronize(stream);  // the last kernel that read it has drained
                (void)hipHostFree(host);
            }
            host = dev = nullptr;
            cap = 0;
            size_t want = std::max(bytes, (size_t)1 << 18);
            want = (want + 4095) & ~(size_t)4095;
            if (hipHostMalloc((void**)&host, want, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
                host = nullptr;
                return SBFT_GV_ENOMEM;
            }
            if (hipHostGetDevicePointer((void**)&dev, host, 0) != hipSuccess) {
                (void)hipHostFree(host);
                host = nullptr;
                return SBFT_GV_EDEVICE;
            }
            cap = want;
            return SBFT_GV_OK;
        }
        void release() {
            if (stream) (void)hipStreamSynchronize(stream);
            if (host) (void)hipHostFree(host);
            if (done) (void)hipEventDestroy(done);
            done = nullptr;
            if (stream) (void)hipStreamDestroy(stream);
            host = dev = nullptr;
            stream = nullptr;
            cap = 0;
        }
    };
    // mapped, coherent host memory the VerifyProposal launches read their message offsets and
    // lengths from (sbft_gv_framed_overlapped; no copy, caller holds mu). Called while the helper
    // may still be queueing the payload copy on `stream`: when the buffer grows, the
    // synchronisation and hipHostFree below wait behind that copy, so the overlap holds only for
    // calls that do not grow it -- the buffer doubles, so after a proposal of a given size
    // every later one up to twice as large reuses it.
    uint8_t* vmap = nullptr;
    uint8_t* vmap_dev = nullptr;
    size_t vmap_cap = 0;
    int reserve_vmap(size_t bytes) {
        NOMEM_POINT();
        if (bytes <= vmap_cap) return SBFT_GV_OK;
        const size_t old_cap = vmap_cap;
        if (vmap) {
            (void)hipStreamSynchronize(stream);  // the last launches that read it have drained
            (void)hipHostFree(vmap);
        }
        vmap = vmap_dev = nullptr;
        vmap_cap = 0;
        size_t want = std::max(bytes, std::max((size_t)1 << 18, 2 * old_cap));
        want = (want + 4095) & ~(size_t)4095;
        if (hipHostMalloc((void**)&vmap, want, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            vmap = nullptr;
            return SBFT_GV_ENOMEM;
        }
        if (hipHostGetDevicePointer((void**)&vmap_dev, vmap, 0) != hipSuccess) {
            (void)hipHostFree(vmap);
            vmap = nullptr;
            return SBFT_GV_EDEVICE;
        }
        vmap_cap = want;
        return SBFT_GV_OK;
    }
    static constexpr int kZcLanes = 4;
    ZcLane zcl[kZcLanes];
    std::atomic<uint32_t> zc_rr{0};
    // A free lane (locked into lk), or, when all are busy, the next one in turn (waits for it).
    ZcLane& acquire_zc(std::unique_lock<std::mutex>& lk) {
        const uint32_t s = zc_rr.fetch_add(1, std::memory_order_relaxed);
        for (int i = 0; i < kZcLanes; ++i) {
            ZcLane& z = zcl[(s + i) % kZcLanes];
            std::unique_lock<std::mutex> t(z.mu, std::try_to_lock);
            if (t.owns_lock()) {
                lk = std::move(t);
                return z;
            }
        }
        ZcLane& z = zcl[s % kZcLanes];
        lk = std::unique_lock<std::mutex>(z.mu);
        return z;
    }
    // fixed-base comb table for u1*G of the generic verify (p256_verify.hip), built on first use
    std::mutex gcomb_mu;
    void* gcomb = nullptr;
    bool gcomb_ready = false;
    Slot* gcomb_owner = nullptr;  // the device's first slot, whose table every slot of it reads

    // The comb table, building it (synchronously, on the owner slot's stream) the first time.
    // The table is read-only once built, so the slots of one device (slots_per_device > 1)
    // share one copy (2.0 GB at 22-bit windows). Returns nullptr on failure.
    const void* gcomb_table() {
        if (gcomb_owner && gcomb_owner != this) return gcomb_owner->gcomb_table();
        std::lock_guard<std::mutex> g(gcomb_mu);
        if (gcomb_ready) return gcomb;
        const size_t bytes = sbft_gcomb_table_bytes();
        if (hipSetDevice(device) != hipSuccess) return nullptr;
        if (!gcomb && hipMalloc(&gcomb, bytes) != hipSuccess) {
            gcomb = nullptr;
            return nullptr;
        }
        if (sbft_launch_gcomb_build(gcomb, stream) || hipStreamSynchronize(stream) != hipSuccess) return nullptr;
        gcomb_ready = true;
        return gcomb;
    }

    int reserve_pinned(size_t bytes) {
        NOMEM_POINT();
        if (bytes <= pin_cap) return SBFT_GV_OK;
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        pin_cap = 0;
        size_t want = std::max(bytes, (size_t)1 << 20);
        want = (want + 4095) & ~(size_t)4095;
        if (hipHostMalloc((void**)&pin, want, hipHostMallocDefault) != hipSuccess) return SBFT_GV_ENOMEM;
        pin_cap = want;
        return SBFT_GV_OK;
    }

    // device copy of a whole payload for sbft_gv_framed_overlapped (kept apart from dbuf,
    // which that call grows after the copy has started)
    uint8_t* bbuf = nullptr;
    size_t bcap = 0;
    int reserve_blob(size_t bytes) {
        NOMEM_POINT();
        if (bytes <= bcap) return SBFT_GV_OK;
        if (bbuf) (void)hipFree(bbuf);
        bbuf = nullptr;
        bcap = 0;
        size_t want = std::max(bytes, (size_t)1 << 22);
        want = (want + 4095) & ~(size_t)4095;
        if (hipMalloc(&bbuf, want) != hipSuccess) return SBFT_GV_ENOMEM;
        bcap = want;
        return SBFT_GV_OK;
    }

    // double-buffered staging of the streamed hash + verify (sbft_gv_sha256_verify_p256_stream):
    // per window slot a device buffer, a pinned input and a pinned output buffer, and the
    // events that order them (H2D done on the copy stream, outputs landed on the main stream)
    struct StreamStage {
        uint8_t* dev = nullptr;
        size_t dev_cap = 0;
        uint8_t* pin_in = nullptr;
        size_t in_cap = 0;
        uint8_t* pin_out = nullptr;
        size_t out_cap = 0;
        hipEvent_t h2d_done = nullptr, out_done = nullptr;
        hipStream_t cs = nullptr;  // the stage's compute stream
    };
    std::vector<StreamStage> stage;
    int reserve_stage(size_t b, size_t dev_bytes, size_t in_bytes, size_t out_bytes) {
        NOMEM_POINT();
        if (stage.size() <= b) stage.resize(b + 1);
        StreamStage& st = stage[b];
        if (!st.cs && hipStreamCreateWithFlags(&st.cs, hipStreamNonBlocking) != hipSuccess) {
            st.cs = nullptr;
            return SBFT_GV_EDEVICE;
        }
        if (!st.h2d_done && hipEventCreateWithFlags(&st.h2d_done, hipEventDisableTiming) != hipSuccess) {
            st.h2d_done = nullptr;
            return SBFT_GV_EDEVICE;
        }
        if (!st.out_done && hipEventCreateWithFlags(&st.out_done, hipEventDisableTiming) != hipSuccess) {
            st.out_done = nullptr;
            return SBFT_GV_EDEVICE;
        }
        auto grow = [](uint8_t*& p, size_t& cap, size_t want, bool pinned) -> int {
            if (want <= cap) return SBFT_GV_OK;
            if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
            p = nullptr;
            cap = 0;
            want = ((want + ((size_t)1 << 20) - 1) >> 20) << 20;
            const hipError_t e = pinned ? hipHostMalloc((void**)&p, want, hipHostMallocDefault) : hipMalloc(&p, want);
            if (e != hipSuccess) {
                p = nullptr;
                return SBFT_GV_ENOMEM;
            }
            cap = want;
            return SBFT_GV_OK;
        };
        int rc = grow(st.dev, st.dev_cap, dev_bytes, false);
        if (!rc) rc = grow(st.pin_in, st.in_cap, in_bytes, true);
        if (!rc) rc = grow(st.pin_out, st.out_cap, out_bytes, true);
        return rc;
    }
    void free_stage() {
        for (StreamStage& st : stage) {
            if (st.cs) (void)hipStreamSynchronize(st.cs);
            if (st.dev) (void)hipFree(st.dev);
            if (st.pin_in) (void)hipHostFree(st.pin_in);
            if (st.pin_out) (void)hipHostFree(st.pin_out);
            if (st.h2d_done) (void)hipEventDestroy(st.h2d_done);
            if (st.out_done) (void)hipEventDestroy(st.out_done);
            if (st.cs) {
                (void)hipStreamSynchronize(st.cs);
                (void)hipStreamDestroy(st.cs);
            }
        }
        stage.clear();
    }

    uint64_t dgen = 0;  // dbuf allocations so far (a new one may reuse the old address)
    // dbuf reservations so far: a path that wants to know whether anyone else wrote dbuf since
    // its own last use compares this (enqueue_framed_share's fix-up counter)
    uint64_t duses = 0, share_clean_at = UINT64_MAX;
    int reserve(size_t bytes) {
        NOMEM_POINT();
        ++duses;
        if (bytes <= dcap) return SBFT_GV_OK;
        if (dbuf) (void)hipFree(dbuf);
        dbuf = nullptr;
        dcap = 0;
        size_t want = std::max(bytes, (size_t)1 << 20);
        want = (want + 4095) & ~(size_t)4095;
        if (hipMalloc(&dbuf, want) != hipSuccess) return SBFT_GV_ENOMEM;
        dcap = want;
        ++dgen;
        return SBFT_GV_OK;
    }
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// hash batches of at least this many messages (and no caller order) are taken longest first
// (sbft_launch_sha256_lpt_order: three small kernels, ~tens of us, against a tail of up to
// milliseconds when long messages are drawn last)
constexpr size_t kShaLptMin = 65536;

// signing batches up to this size take the wavefront-per-signature kernel (defined with the
// registered-key code below, which owns G's comb table)
constexpr size_t kSignWaveMax = 4096;
int sign_wave(sbft_gv_ctx* ctx, const uint8_t* d, const uint8_t* k, const uint8_t* digest, size_t n, uint8_t* qx,
              uint8_t* qy, uint8_t* r, uint8_t* s, uint8_t* status);
// registered-key tables [0, upto) on a slot's device (defined with the registered-key code)
int ensure_tables(Slot* sl, size_t upto);


}  // namespace

struct sbft_gv_ctx {
    // kernel timing (sbft_gv_kernel_timing): event pairs around each device-resident verify's
    // main kernel, read and released by sbft_gv_kernel_time
    std::atomic<bool> timing{false};
    std::mutex ev_mu;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    std::vector<Slot*> slots;
    uint32_t min_split = 65536;
    // batches (per device) of at most this many tuples use the two-lanes-per-tuple latency
    // kernel; 0 = never (sbft_gv_opts.pair_max)
    uint32_t pair_max = SBFT_GV_PAIR_MAX_DEFAULT;
    uint32_t half_max = SBFT_GV_HALF_MAX_DEFAULT;  // ... half-size scalars (sbft_gv_opts.half_max)
    uint32_t halfq_max = 0;  // ... their wide form (sbft_gv_opts.halfq_max; set by sbft_gv_init)
    std::atomic<uint32_t> rr{0};
    // verify kernel for a per-device batch of n: 4 = half-size scalars on quads (eight lanes per
    // tuple), 3 = half-size scalars (four lanes), 2 = pair kernel, 1 = throughput kernel
    int lanes_for(size_t n) const { return n <= halfq_max ? 4 : n <= half_max ? 3 : n <= pair_max ? 2 : 1; }
    // keyed batches (per device) of at most this many signatures take the zero-copy path
    // (enqueue_keyed); SBFT_KEYED_ZC_MAX overrides (0 = never)
    size_t keyed_zc_max = 1024;
    // ... and batches of at least this many the four-lane kernel (p256_verify_keyed_lanes_kernel,
    // batched s^-1) instead of a wavefront per signature; SBFT_KEYED_LANES_MIN overrides (0 = never)
    size_t keyed_lanes_min = 1025;
    // zero-copy keyed batches of at most this many signatures get s^-1 from the host (a batched
    // inversion: one safegcd and ~4 products mod n per signature, ~7 us for a 67-signature quorum)
    // instead of the kernel's second wavefront (~15 us: the divstep table and the wave-parallel
    // safegcd); SBFT_KEYED_HOST_SINV_MAX overrides (0 = always on the device)
    size_t keyed_host_sinv_max = 96;
    // registered public keys (x || y big-endian); index = key id, entry 0 = the generator
    std::mutex keys_mu;
    std::vector<std::array<uint8_t, 64>> keys;
    std::vector<uint8_t> key_valid;  // 1 if keys[i] is a point on the curve
    struct KeyHash {
        size_t operator()(const std::array<uint8_t, 64>& k) const {
            uint64_t a, b;
            std::memcpy(&a, k.data() + 24, 8);  // low words of x and y: uniformly distributed
            std::memcpy(&b, k.data() + 56, 8);
            return (size_t)(a * 0x9E3779B97F4A7C15ull ^ b);
        }
    };
    std::unordered_map<std::array<uint8_t, 64>, uint32_t, KeyHash> key_index;
    std::atomic<uint32_t> nkeys{1};
    // client-key budget (sbft_gv_register_client_keys): bytes of client comb tables allowed per
    // device (0 = 1/8 of the device's memory) and the client keys that hold tables (under keys_mu)
    uint64_t client_cap = 0;
    size_t client_keys = 0;
    Helper helper;    // host work overlapped with a caller's copies (sbft_gv_framed_overlapped)
    Workers workers;  // host threads driving shares 1.. of a split batch (for_each_device)
};

// the generator G, x || y big-endian (key id 0)
static const std::array<uint8_t, 64> kGXY = {
    0x6b, 0x17, 0xd1, 0xf2, 0xe1, 0x2c, 0x42, 0x47, 0xf8, 0xbc, 0xe6, 0xe5, 0x63, 0xa4, 0x40, 0xf2,
    0x77, 0x03, 0x7d, 0x81, 0x2d, 0xeb, 0x33, 0xa0, 0xf4, 0xa1, 0x39, 0x45, 0xd8, 0x98, 0xc2, 0x96,
    0x4f, 0xe3, 0x42, 0xe2, 0xfe, 0x1a, 0x7f, 0x9b, 0x8e, 0xe7, 0xeb, 0x4a, 0x7c, 0x0f, 0x9e, 0x16,
    0x2b, 0xce, 0x33, 0x57, 0x6b, 0x31, 0x5e, 0xce, 0xcb, 0xb6, 0x40, 0x68, 0x37, 0xbf, 0x51, 0xf5};

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return SBFT_GV_EDEVICE; \
    } while (0)

#include "p256_post_vectors.inc"

// Power-on self-test (sbft_gv_init, every device; SBFT_GV_SELFTEST=0 skips it): 72 known-answer
// tuples (tools/gen_post_vectors.py: four of every golden-fixture category, including R = infinity
// and Shamir-exceptional ones for the fix-up kernel) through the throughput kernel and both
// latency kernels, and six SHA-256 known answers at unaligned offsets. The radix-2^29 field code
// relies on the compiler not seeing its limb ranges (p256_f29.hpp: ROCm 7.2 miscompiled the
// range-visible form): a toolchain or driver that breaks it makes the context refuse to start
// (SBFT_GV_ESELFTEST) instead of returning wrong verdicts.
static int power_on_selftest(Slot* sl) {
    // SBFT_POST_TRACE=1: report the failing step on stderr (diagnostics)
    static const bool trace = getenv("SBFT_POST_TRACE") != nullptr;
#define POSTCHK(x, what)                                                                                  \
    do {                                                                                                  \
        const hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                           \
            if (trace) fprintf(stderr, "sbft POST: %s failed: %s (lanes %d)\n", what, hipGetErrorString(e_), cur); \
            return SBFT_GV_EDEVICE;                                                                       \
        }                                                                                                 \
    } while (0)
    int cur = 0;
    POSTCHK(hipSetDevice(sl->device), "set device");
    const size_t n = SBFT_POST_N;
    const size_t f = align_up(32 * n, 256), fo = align_up(n, 256);
    int rc = sl->reserve(5 * f + fo + sbft_verify_work_bytes(n));
    if (rc) return rc;
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    std::vector<uint8_t> h(5 * f, 0), ok(n);
    for (size_t k = 0; k < n; ++k)
        for (int fld = 0; fld < 5; ++fld) std::memcpy(&h[fld * f + 32 * k], kPostVectors[k] + 32 * fld, 32);
    uint8_t* base = sl->dbuf;
    uint32_t* work = (uint32_t*)(base + 5 * f + fo);
    POSTCHK(hipMemcpyAsync(base, h.data(), 5 * f, hipMemcpyHostToDevice, sl->stream), "tuple copy");
    // every verify kernel on the same workspace, back to back, the exact fixup net last (0): it
    // serves the others' flagged tuples, and in rounds 4-5 it had faulted unseen because nothing
    // reached it
    for (int lanes : {1, 2, 3, 4, 0}) {
        cur = lanes;
        POSTCHK(hipMemsetAsync(base + 5 * f, 0xEE, n, sl->stream), "verdict memset");
        if (sbft_launch_p256_verify(base, base + f, base + 2 * f, base + 3 * f, base + 4 * f, base + 5 * f, (uint32_t)n,
                                    work, gcomb, sl->stream, nullptr, nullptr, lanes))
            return SBFT_GV_ELAUNCH;
        POSTCHK(hipMemcpyAsync(ok.data(), base + 5 * f, n, hipMemcpyDeviceToHost, sl->stream), "verdict copy");
        POSTCHK(hipStreamSynchronize(sl->stream), "verify");
        for (size_t k = 0; k < n; ++k)
            if (ok[k] != kPostVectors[k][160]) {
                if (trace) fprintf(stderr, "sbft POST: lanes %d: tuple %zu verdict %d, expected %d\n", lanes, k, ok[k], kPostVectors[k][160]);
                return SBFT_GV_ESELFTEST;
            }
    }
    // SHA-256: blob (+ the kernel's over-read pad) | off | len | counter | digests
    const size_t m = SBFT_POST_SHA_N, fb = align_up(SBFT_POST_SHA_BLOB + SBFT_GV_SHA_BLOB_PAD, 256);
    if ((rc = sl->reserve(fb + 3 * 256 + 32 * m))) return rc;
    uint8_t* b = sl->dbuf;
    std::vector<uint8_t> blob(fb, 0);
    std::memcpy(blob.data(), kPostShaBlob, SBFT_POST_SHA_BLOB);
    uint64_t off[SBFT_POST_SHA_N];
    uint32_t len[SBFT_POST_SHA_N];
    for (size_t k = 0; k < m; ++k) {
        off[k] = kPostShaOff[k];
        len[k] = kPostShaLen[k];
    }
    uint8_t dig[SBFT_POST_SHA_N][32];
    HIPCHK(hipMemcpyAsync(b, blob.data(), fb, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(b + fb, off, sizeof off, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(b + fb + 256, len, sizeof len, hipMemcpyHostToDevice, sl->stream));
    if (sbft_launch_sha256(b, (const uint64_t*)(b + fb), (const uint32_t*)(b + fb + 256), nullptr, b + fb + 768,
                           (uint32_t)m, (uint32_t*)(b + fb + 512), sl->stream))
        return SBFT_GV_ELAUNCH;
    cur = 0;
    POSTCHK(hipMemcpyAsync(dig, b + fb + 768, sizeof dig, hipMemcpyDeviceToHost, sl->stream), "digest copy");
    POSTCHK(hipStreamSynchronize(sl->stream), "sha256");
    return std::memcmp(dig, kPostShaDigest, sizeof dig) == 0 ? SBFT_GV_OK : SBFT_GV_ESELFTEST;
}
#undef POSTCHK

extern "C" {

int sbft_gv_inject_fault(int kind, int count) {
    if (kind < SBFT_GV_FAULT_OFF || kind > SBFT_GV_FAULT_SYNC) return SBFT_GV_EINVAL;
    g_fault_kind.store(SBFT_GV_FAULT_OFF);
    g_fault_left.store(kind == SBFT_GV_FAULT_OFF ? 0 : count);
    g_fault_kind.store(kind);
    if (kind != SBFT_GV_FAULT_OFF)  // loud: an armed fault makes engine calls fail (fail-stop in Go)
        fprintf(stderr, "sbft_gpuverify: TEST FAULT INJECTION ARMED (kind %d, count %d): engine calls will fail\n",
                kind, count);
    return SBFT_GV_OK;
}

const char* sbft_gv_strerror(int code) {
    switch (code) {
    case SBFT_GV_OK: return "ok";
    case SBFT_GV_EINVAL: return "invalid argument";
    case SBFT_GV_ENODEV: return "no usable GPU";
    case SBFT_GV_ENOMEM: return "allocation failed";
    case SBFT_GV_ELAUNCH: return "kernel launch failed";
    case SBFT_GV_EDEVICE: return "HIP runtime error";
    case SBFT_GV_ESELFTEST: return "device failed the known-answer self-test";
    default: return "unknown error";
    }
}

int sbft_gv_init(const sbft_gv_opts* opts, sbft_gv_ctx** out) {
    if (!out) return SBFT_GV_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SBFT_GV_ENODEV;
    const uint32_t mask = (opts && opts->device_mask) ? opts->device_mask : 0xffffffffu;
    auto* ctx = new (std::nothrow) sbft_gv_ctx();
    if (!ctx) return SBFT_GV_ENOMEM;
    if (opts && (opts->reserved0 || opts->reserved1)) {  // reserved fields must be 0 (a retired field's
        delete ctx;                                      // old meaning is never read as a new one)
        return SBFT_GV_EINVAL;
    }
    if (opts && opts->pair_max) ctx->pair_max = opts->pair_max < 0 ? 0u : (uint32_t)opts->pair_max;
    // pair_max < 0 means "no latency kernel": the half kernel too, unless half_max asks for it
    if (opts && opts->pair_max < 0 && !opts->half_max) ctx->half_max = 0;
    if (opts && opts->half_max) ctx->half_max = opts->half_max < 0 ? 0u : (uint32_t)opts->half_max;
    if (const char* e = getenv("SBFT_GV_HALF_MAX")) {
        const long v = strtol(e, nullptr, 10);
        ctx->half_max = v < 0 ? 0u : (uint32_t)v;
    }
    {
        // the wide half kernel: one 24-tuple workgroup per CU of the first selected device (its
        // three verify wavefronts and the helper on the CU's four SIMDs); off with the half kernel
        int dev0 = 0, cus = 0;
        while (dev0 < ndev && !(mask & (1u << dev0))) ++dev0;
        if (dev0 >= ndev || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev0) != hipSuccess ||
            cus <= 0)
            cus = 256;
        ctx->halfq_max = ctx->half_max ? 24u * (uint32_t)cus : 0u;
        if (opts && opts->halfq_max) ctx->halfq_max = opts->halfq_max < 0 ? 0u : (uint32_t)opts->halfq_max;
        if (const char* e = getenv("SBFT_GV_HALFQ_MAX")) {
            const long v = strtol(e, nullptr, 10);
            ctx->halfq_max = v < 0 ? 0u : (uint32_t)v;
        }
    }
    // min_split: a batch the wide kernel cannot take whole is split when there are devices to
    // split it over (a 10k proposal over 2-8 GPUs: shares of <= halfq_max, each on the wide kernel)
    ctx->min_split = opts && opts->min_split ? opts->min_split : ctx->halfq_max ? ctx->halfq_max + 1 : 65536u;
    if (opts) ctx->client_cap = opts->client_table_bytes;
    if (const char* e = getenv("SBFT_GV_CLIENT_TABLE_BYTES")) ctx->client_cap = strtoull(e, nullptr, 10);
    if (const char* e = getenv("SBFT_KEYED_ZC_MAX")) ctx->keyed_zc_max = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("SBFT_KEYED_LANES_MIN")) ctx->keyed_lanes_min = (size_t)strtoull(e, nullptr, 10);
    if (const char* e = getenv("SBFT_KEYED_HOST_SINV_MAX"))
        ctx->keyed_host_sinv_max = (size_t)strtoull(e, nullptr, 10);
    // slots per device (sbft_gv_opts.slots_per_device, SBFT_GV_SLOTS_PER_DEVICE): > 1 runs the
    // multi-device split on one GPU, each slot standing in for a device of its own
    uint32_t spd = opts && opts->slots_per_device ? opts->slots_per_device : 1u;
    if (const char* e = getenv("SBFT_GV_SLOTS_PER_DEVICE")) spd = (uint32_t)strtoul(e, nullptr, 10);
    if (spd == 0 || spd > 64) {
        delete ctx;
        return SBFT_GV_EINVAL;
    }
    for (int d = 0; d < ndev && d < 32; ++d) {
        if (!(mask & (1u << d))) continue;
        Slot* first = nullptr;
        for (uint32_t k = 0; k < spd; ++k) {
            auto* s = new Slot();
            s->device = d;
            s->gcomb_owner = first ? first : s;
            if (hipSetDevice(d) != hipSuccess ||
                hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
                delete s;
                break;
            }
            ctx->slots.push_back(s);
            if (!first) first = s;
        }
    }
    if (ctx->slots.empty()) {
        delete ctx;
        return SBFT_GV_ENODEV;
    }
    // key id 0: the generator G (its comb table serves u1*G on the keyed path)
    ctx->keys.push_back(kGXY);
    ctx->key_valid.push_back(1);
    // The self-test (which also builds each device's 2 GB G comb, ~0.43 s) runs on every slot at
    // once, one host thread per slot: an 8-GPU node starts in one device's time, not eight.
    // Slots of one device share its comb (built once, under the owner's lock).
    const char* st = getenv("SBFT_GV_SELFTEST");
    if (!st || std::strcmp(st, "0") != 0) {
        std::vector<int> rcs(ctx->slots.size(), SBFT_GV_OK);
        std::vector<std::thread> th;
        try {
            for (size_t i = 1; i < ctx->slots.size(); ++i)
                th.emplace_back([&, i] { rcs[i] = power_on_selftest(ctx->slots[i]); });
        } catch (...) {  // no thread: the remaining slots are tested on this one
            for (size_t i = th.size() + 1; i < ctx->slots.size(); ++i) rcs[i] = power_on_selftest(ctx->slots[i]);
        }
        rcs[0] = power_on_selftest(ctx->slots[0]);
        for (auto& t : th) t.join();
        for (int rc : rcs)
            if (rc) {
                sbft_gv_destroy(ctx);
                return rc;
            }
    }
    // SBFT_GV_FAULT=nomem|launch|sync[:count] (tests): armed once the self-test has passed
#ifdef SBFT_FAULT_INJECTION  // test builds only: a stray variable must not stop a deployment
    if (const char* e = getenv("SBFT_GV_FAULT")) {
        const int kind = !std::strncmp(e, "nomem", 5) ? SBFT_GV_FAULT_NOMEM
                         : !std::strncmp(e, "launch", 6) ? SBFT_GV_FAULT_LAUNCH
                         : !std::strncmp(e, "sync", 4) ? SBFT_GV_FAULT_SYNC : SBFT_GV_FAULT_OFF;
        const char* c = std::strchr(e, ':');
        (void)sbft_gv_inject_fault(kind, c ? std::atoi(c + 1) : -1);
    }
#endif
    *out = ctx;
    return SBFT_GV_OK;
}

void sbft_gv_destroy(sbft_gv_ctx* ctx) {
    if (!ctx) return;
    uint64_t nl;
    double ms;
    (void)sbft_gv_kernel_time(ctx, &nl, &ms);  // releases pending timing events
    // drain every device first: a slot's launches (on its streams or a caller's) may read
    // tables another slot of the device owns (the shared G comb)
    uint32_t drained = 0;
    for (Slot* s : ctx->slots)
        if (!(drained & (1u << s->device))) {
            drained |= 1u << s->device;
            (void)hipSetDevice(s->device);
            (void)hipDeviceSynchronize();
        }
    for (Slot* s : ctx->slots) {
        (void)hipSetDevice(s->device);
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->dbuf) (void)hipFree(s->dbuf);
        if (s->bbuf) (void)hipFree(s->bbuf);
        for (void* t : s->comb_alloc) (void)hipFree(t);
        if (s->d_keytab) (void)hipFree(s->d_keytab);
        for (void* t : s->retired) (void)hipFree(t);
        if (s->pin) (void)hipHostFree(s->pin);
        for (auto& z : s->zcl) z.release();
        if (s->vmap) (void)hipHostFree(s->vmap);
        if (s->gcomb) (void)hipFree(s->gcomb);
        for (auto& kv : s->ws) {
            (void)hipStreamSynchronize(kv.first);
            if (kv.second.ptr) (void)hipFree(kv.second.ptr);
        }
        for (hipEvent_t e : s->sub_ev) (void)hipEventDestroy(e);
        s->free_stage();
        for (hipStream_t st : {s->copy_stream, s->stream2}) {
            if (!st) continue;
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
    }
    delete ctx;
}

size_t sbft_gv_verify_workspace_bytes(size_t n) { return sbft_verify_work_bytes(n); }

int sbft_gv_host_alloc(size_t bytes, void** out) {
    if (!out) return SBFT_GV_EINVAL;
    *out = nullptr;
    if (bytes == 0) return SBFT_GV_OK;
    if (hipHostMalloc(out, bytes, hipHostMallocPortable) != hipSuccess) {
        *out = nullptr;
        return SBFT_GV_ENOMEM;
    }
    return SBFT_GV_OK;
}

void sbft_gv_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
namespace {
// sbft_gv_kernel_timing for the latency paths (the fused VerifyProposal launch, the keyed
// launches): HIP events around one launch on its stream, handed to ctx->events for
// sbft_gv_kernel_time. Inert unless timing is on.
struct LaunchTimer {
    sbft_gv_ctx* ctx;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    LaunchTimer(sbft_gv_ctx* c, hipStream_t s) : ctx(c && c->timing.load() ? c : nullptr), st(s) {
        if (!ctx) return;
        if (hipEventCreate(&a) != hipSuccess || hipEventRecord(a, st) != hipSuccess) {
            if (a) (void)hipEventDestroy(a);
            a = nullptr;
            ctx = nullptr;
        }
    }
    void end() {
        if (!ctx) return;
        if (hipEventCreate(&b) != hipSuccess || hipEventRecord(b, st) != hipSuccess) {
            (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
        } else {
            std::lock_guard<std::mutex> g(ctx->ev_mu);
            ctx->events.emplace_back(a, b);
        }
        ctx = nullptr;
    }
    ~LaunchTimer() {
        if (ctx && a) (void)hipEventDestroy(a);
    }
};
}  // namespace
extern "C" {

int sbft_gv_kernel_timing(sbft_gv_ctx* ctx, int enable) {
    if (!ctx) return SBFT_GV_EINVAL;
    ctx->timing = enable != 0;
    return SBFT_GV_OK;
}

int sbft_gv_kernel_time(sbft_gv_ctx* ctx, uint64_t* launches, double* ms) {
    if (!ctx || !launches || !ms) return SBFT_GV_EINVAL;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
    {
        std::lock_guard<std::mutex> g(ctx->ev_mu);
        evs.swap(ctx->events);
    }
    *launches = 0;
    *ms = 0.0;
    int rc = SBFT_GV_OK;
    for (auto& e : evs) {
        float t = 0.f;
        if (rc == SBFT_GV_OK &&
            (hipEventSynchronize(e.second) != hipSuccess || hipEventElapsedTime(&t, e.first, e.second) != hipSuccess))
            rc = SBFT_GV_EDEVICE;
        if (rc == SBFT_GV_OK) {
            *ms += t;
            ++*launches;
        }
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    return rc;
}

int sbft_gv_device_count(const sbft_gv_ctx* ctx) { return ctx ? (int)ctx->slots.size() : 0; }

size_t sbft_gv_plan_split(size_t n, size_t n_devices, size_t min_split, size_t* begin, size_t* count) {
    if (n_devices == 0 || !begin || !count) return 0;
    if (n < (min_split ? min_split : 65536) || n_devices == 1) {
        begin[0] = 0;
        count[0] = n;
        return 1;
    }
    // contiguous shares that differ by at most one tuple; a device with none is left out
    size_t parts = 0;
    for (size_t d = 0; d < n_devices; ++d) {
        const size_t b = n * d / n_devices, e = n * (d + 1) / n_devices;
        if (e > b) {
            begin[parts] = b;
            count[parts] = e - b;
            ++parts;
        }
    }
    return parts;
}

void sbft_gv_normalize_hash(const uint8_t* hash, size_t len, uint8_t out32[32]) {
    // Go hashToNat (crypto/internal/fips140/ecdsa): the leftmost N.Size() = 32 bytes; a
    // shorter hash is the same integer, i.e. left-padded with zeros.
    std::memset(out32, 0, 32);
    if (!hash || len == 0) return;
    if (len >= 32) std::memcpy(out32, hash, 32);
    else std::memcpy(out32 + (32 - len), hash, len);
}

int sbft_gv_normalize_scalar(const uint8_t* be, size_t len, uint8_t out32[32]) {
    std::memset(out32, 0, 32);
    size_t i = 0;
    while (i < len && be[i] == 0) ++i;  // big.Int.Bytes() has no leading zeros; accept them anyway
    const size_t m = len - i;
    if (m > 32) return 0;
    if (m) std::memcpy(out32 + (32 - m), be + i, m);
    return 1;
}

// ---------------------------------------------------------------- device-resident
static Slot* slot_for(sbft_gv_ctx* ctx, int device) {
    for (Slot* s : ctx->slots)
        if (s->device == device) return s;
    return nullptr;
}

int sbft_gv_verify_p256_dev(sbft_gv_ctx* ctx, int device, const void* d_digest, const void* d_r,
                            const void* d_s, const void* d_qx, const void* d_qy, size_t n,
                            void* d_ok, void* stream) {
    if (!ctx || (n && (!d_digest || !d_r || !d_s || !d_qx || !d_qy || !d_ok))) return SBFT_GV_EINVAL;
    if (n > 0xffffffffu) return SBFT_GV_EINVAL;
    Slot* sl = slot_for(ctx, device);
    if (!sl) return SBFT_GV_ENODEV;
    if (n == 0) return SBFT_GV_OK;
    if (hipSetDevice(device) != hipSuccess) return SBFT_GV_EDEVICE;
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    uint32_t* work = sl->stream_workspace((hipStream_t)stream, sbft_verify_work_bytes(n));
    if (!work) return SBFT_GV_ENOMEM;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (ctx->timing.load()) {
        if (hipEventCreate(&ev0) != hipSuccess) return SBFT_GV_EDEVICE;
        if (hipEventCreate(&ev1) != hipSuccess) {
            (void)hipEventDestroy(ev0);
            return SBFT_GV_EDEVICE;
        }
        std::lock_guard<std::mutex> g(ctx->ev_mu);
        ctx->events.emplace_back(ev0, ev1);
    }
    return sbft_launch_p256_verify((const uint8_t*)d_digest, (const uint8_t*)d_r, (const uint8_t*)d_s,
                                   (const uint8_t*)d_qx, (const uint8_t*)d_qy, (uint8_t*)d_ok,
                                   (uint32_t)n, work, gcomb, (hipStream_t)stream, ev0, ev1, ctx->lanes_for(n))
               ? SBFT_GV_ELAUNCH
               : SBFT_GV_OK;
}

int sbft_gv_sha256_dev(sbft_gv_ctx* ctx, int device, const void* d_blob, const void* d_off,
                       const void* d_len, const void* d_order, size_t n, void* d_dig, void* stream) {
    if (!ctx || (n && (!d_blob || !d_off || !d_len || !d_dig))) return SBFT_GV_EINVAL;
    if (n > 0xffffffffu) return SBFT_GV_EINVAL;
    Slot* sl = slot_for(ctx, device);
    if (!sl) return SBFT_GV_ENODEV;
    if (n == 0) return SBFT_GV_OK;
    if (hipSetDevice(device) != hipSuccess) return SBFT_GV_EDEVICE;
    // the stream's workspace: work counter | longest-first sort scratch | order
    const bool lpt = !d_order && n >= kShaLptMin;
    const size_t o_ws = 256, o_ord = 256 + align_up(sbft_sha256_lpt_ws_bytes(), 256);
    uint32_t* ws = sl->stream_workspace((hipStream_t)stream, lpt ? o_ord + 4 * n : 256);
    if (!ws) return SBFT_GV_ENOMEM;
    uint32_t* ord = (uint32_t*)((uint8_t*)ws + o_ord);
    if (lpt && sbft_launch_sha256_lpt_order((const uint32_t*)d_len, (uint32_t)n, (uint32_t*)((uint8_t*)ws + o_ws),
                                            ord, (hipStream_t)stream))
        return SBFT_GV_ELAUNCH;
    return sbft_launch_sha256((const uint8_t*)d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len,
                              lpt ? ord : (const uint32_t*)d_order, (uint8_t*)d_dig, (uint32_t)n, ws,
                              (hipStream_t)stream)
               ? SBFT_GV_ELAUNCH
               : SBFT_GV_OK;
}

int sbft_gv_sha256_verify_p256_dev(sbft_gv_ctx* ctx, int device, const void* d_blob,
                                   const void* d_off, const void* d_len, const void* d_order,
                                   const void* d_r, const void* d_s, const void* d_qx,
                                   const void* d_qy, size_t n, void* d_ok, void* d_dig,
                                   void* stream) {
    if (!d_dig) return SBFT_GV_EINVAL;  // the digest scratch is caller-provided here
    int rc = sbft_gv_sha256_dev(ctx, device, d_blob, d_off, d_len, d_order, n, d_dig, stream);
    if (rc) return rc;
    return sbft_gv_verify_p256_dev(ctx, device, d_dig, d_r, d_s, d_qx, d_qy, n, d_ok, stream);
}

int sbft_gv_sign_p256_dev(sbft_gv_ctx* ctx, int device, const void* d_d, const void* d_k,
                          const void* d_digest, size_t n, void* d_qx, void* d_qy, void* d_r,
                          void* d_s, void* d_status, void* stream) {
    if (!ctx || (n && (!d_d || !d_k || !d_digest || !d_qx || !d_qy || !d_r || !d_s || !d_status)))
        return SBFT_GV_EINVAL;
    if (n > 0xffffffffu) return SBFT_GV_EINVAL;
    if (!slot_for(ctx, device)) return SBFT_GV_ENODEV;
    if (hipSetDevice(device) != hipSuccess) return SBFT_GV_EDEVICE;
    return sbft_launch_p256_sign((const uint8_t*)d_d, (const uint8_t*)d_k, (const uint8_t*)d_digest,
                                 (uint8_t*)d_qx, (uint8_t*)d_qy, (uint8_t*)d_r, (uint8_t*)d_s,
                                 (uint8_t*)d_status, (uint32_t)n, (hipStream_t)stream)
               ? SBFT_GV_ELAUNCH
               : SBFT_GV_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- host buffers
namespace {

struct Chunk {
    Slot* slot;
    size_t begin, count;
    size_t out_off = 0;  // keyed path: verdict offset inside the slot's pinned staging
    int lanes = 1;       // verify kernel: 1 lane per tuple, or the 2 / 4-lane latency kernel
};

std::vector<Chunk> plan(sbft_gv_ctx* ctx, size_t n) {
    std::vector<Chunk> out;
    const size_t nd = ctx->slots.size();
    std::vector<size_t> begin(nd), count(nd);
    const size_t parts = sbft_gv_plan_split(n, nd, ctx->min_split, begin.data(), count.data());
    if (parts == 1) {
        // one device: round-robin, so concurrent small calls spread over the GPUs
        const uint32_t k = ctx->rr.fetch_add(1) % nd;
        out.push_back({ctx->slots[k], 0, n, 0, ctx->lanes_for(n)});
        return out;
    }
    for (size_t d = 0; d < parts; ++d)
        out.push_back({ctx->slots[d], begin[d], count[d], 0, ctx->lanes_for(count[d])});
    return out;
}

// Run f(i) for i in [0, m): i = 0 on the calling thread, the others on the context's persistent
// workers (worker i drives share i), so each device's pageable H2D copies and its synchronisation are
// driven independently instead of one device after another. Returns the first non-zero rc.
// Nothing escapes as an exception (the callers are C entry points): a share that throws reports
// SBFT_GV_ENOMEM (bad_alloc) or SBFT_GV_EDEVICE, a share whose post fails runs on the calling
// thread, and the frame (rc, mu, cv, left, f) outlives every posted job: the wait below runs
// whatever share 0 does.
template <class F>
int for_each_device(sbft_gv_ctx* ctx, size_t m, F&& f) {
    auto run = [&f](size_t i) noexcept -> int {
        try {
            return f(i);
        } catch (const std::bad_alloc&) {
            return SBFT_GV_ENOMEM;
        } catch (...) {
            return SBFT_GV_EDEVICE;
        }
    };
    if (m == 1) return run((size_t)0);
    std::vector<int> rc;
    try {
        rc.assign(m, SBFT_GV_OK);
    } catch (...) {
        return SBFT_GV_ENOMEM;
    }
    std::mutex mu;
    std::condition_variable cv;
    size_t left = 0;  // posted shares still running
    for (size_t i = 1; i < m; ++i) {
        {
            std::lock_guard<std::mutex> g(mu);
            ++left;
        }
        try {
            ctx->workers.post(i, [&, i] {
                const int r = run(i);
                std::lock_guard<std::mutex> g(mu);
                rc[i] = r;
                if (--left == 0) cv.notify_one();
            });
        } catch (...) {  // not queued (Workers::post throws before the push): run it here
            {
                std::lock_guard<std::mutex> g(mu);
                --left;
            }
            rc[i] = run(i);
        }
    }
    rc[0] = run((size_t)0);
    {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return left == 0; });
    }
    for (int r : rc)
        if (r) return r;
    return SBFT_GV_OK;
}

// Enqueue verify of tuples [c.begin, c.begin+c.count) on c.slot. Layout of the slot
// buffer: digest | r | s | qx | qy | ok, each array 256-byte aligned.
int enqueue_verify(const Chunk& c, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                   const uint8_t* qx, const uint8_t* qy, uint8_t* ok_out) {
    Slot* sl = c.slot;
    const size_t f = align_up(32 * c.count, 256);
    HIPCHK(hipSetDevice(sl->device));
    const size_t fo = align_up(c.count, 256);
    int rc = sl->reserve(5 * f + fo + sbft_verify_work_bytes(c.count));
    if (rc) return rc;
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    uint8_t* base = sl->dbuf;
    uint32_t* work = (uint32_t*)(base + 5 * f + fo);
    const uint8_t* src[5] = {digest, r, s, qx, qy};
    for (int k = 0; k < 5; ++k)
        HIPCHK(hipMemcpyAsync(base + k * f, src[k] + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice,
                              sl->stream));
    if (sbft_launch_p256_verify(base, base + f, base + 2 * f, base + 3 * f, base + 4 * f, base + 5 * f,
                                (uint32_t)c.count, work, gcomb, sl->stream, nullptr, nullptr, c.lanes))
        return SBFT_GV_ELAUNCH;
    HIPCHK(hipMemcpyAsync(ok_out + c.begin, base + 5 * f, c.count, hipMemcpyDeviceToHost, sl->stream));
    return SBFT_GV_OK;
}

// True if p is page-locked host memory (sbft_gv_host_alloc / hipHostMalloc / registered).
bool is_pinned(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error here; clear it
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// One device round of the one-lane verify kernel (256 CUs x 4 SIMDs x 4 waves x 64 lanes).
// The pipelined path cuts its batch into a small first sub-batch (its copy is the only one
// exposed) and then sub-batches of one round each.
constexpr size_t kPipeSub = 262144;
// 64k first sub-batch (10 MB, ~0.2 ms exposed); measured (profiles/r01k_pipe_sweep.txt) against
// 16k-256k first sub-batches and one compute stream
constexpr size_t kPipeFirst = 65536;

// enqueue_verify for pinned inputs: the H2D copies run on the slot's copy stream, one event
// per sub-batch; each sub-batch's verify waits on its event and runs on one of two compute
// streams (alternating, each with its own workspace), so a partly filled launch overlaps
// the next one. Same device layout, so the verdicts are byte-identical to enqueue_verify's.
int enqueue_verify_piped(const Chunk& c, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                         const uint8_t* qx, const uint8_t* qy, uint8_t* ok_out) {
    Slot* sl = c.slot;
    const size_t f = align_up(32 * c.count, 256);
    HIPCHK(hipSetDevice(sl->device));
    const size_t fo = align_up(c.count, 256);
    const size_t wb = align_up(sbft_verify_work_bytes(kPipeSub), 256);
    int rc = sl->reserve(5 * f + fo + 2 * wb);
    if (rc) return rc;
    std::vector<size_t> cut{0};
        for (size_t b = std::min(kPipeFirst, c.count); b < c.count; b = std::min(b + kPipeSub, c.count)) cut.push_back(b);
    cut.push_back(c.count);
    const size_t subs = cut.size() - 1;
    if ((rc = sl->reserve_pipe(subs + 2))) return rc;
    hipStream_t cs[2] = {sl->stream, sl->stream2};
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    uint8_t* base = sl->dbuf;
    const uint8_t* src[5] = {digest, r, s, qx, qy};
    // pageable inputs: each sub-batch is first gathered into page-locked staging by four host
    // threads (~60 GB/s, far ahead of the ~10 GB/s the kernels consume), so its DMA runs at the
    // pinned rate while earlier sub-batches verify
    const bool stage = !(is_pinned(digest) && is_pinned(r) && is_pinned(s) && is_pinned(qx) && is_pinned(qy));
    uint8_t* hst = nullptr;
    if (stage) {
        if ((rc = sl->reserve_pinned(5 * f))) return rc;
        hst = sl->pin;
    }
    hipEvent_t ev_start = sl->sub_ev[subs], ev_join = sl->sub_ev[subs + 1];
    // the copy stream and the second compute stream start after earlier work on the slot's
    // stream (which may still read dbuf)
    HIPCHK(hipEventRecord(ev_start, sl->stream));
    // From here on work may be queued on the copy stream and stream2, which the caller does not
    // synchronise (run_chunks waits on sl->stream only): a failure drains both before it
    // returns, so no copy or kernel is still writing dbuf when the next call reallocates it.
    auto body = [&]() -> int {
        HIPCHK(hipStreamWaitEvent(sl->copy_stream, ev_start, 0));
        HIPCHK(hipStreamWaitEvent(sl->stream2, ev_start, 0));
        for (size_t i = 0; i < subs; ++i) {
            const size_t b = cut[i], m = cut[i + 1] - b;
            if (stage) {
                auto part = [&](size_t lo, size_t hi) {
                    for (int k = 0; k < 5; ++k)
                        std::memcpy(hst + k * f + 32 * (b + lo), src[k] + 32 * (c.begin + b + lo), 32 * (hi - lo));
                };
                std::thread th[3];
                for (int t = 1; t < 4; ++t) th[t - 1] = std::thread(part, m * t / 4, m * (t + 1) / 4);
                part(0, m / 4);
                for (auto& x : th) x.join();
            }
            for (int k = 0; k < 5; ++k)
                HIPCHK(hipMemcpyAsync(base + k * f + 32 * b, stage ? hst + k * f + 32 * b : src[k] + 32 * (c.begin + b),
                                      32 * m, hipMemcpyHostToDevice, sl->copy_stream));
            HIPCHK(hipEventRecord(sl->sub_ev[i], sl->copy_stream));
        }
        for (size_t i = 0; i < subs; ++i) {
            const size_t b = cut[i], m = cut[i + 1] - b;
            hipStream_t st = cs[i & 1];
            uint32_t* work = (uint32_t*)(base + 5 * f + fo + (i & 1) * wb);
            HIPCHK(hipStreamWaitEvent(st, sl->sub_ev[i], 0));
            if (sbft_launch_p256_verify(base + 32 * b, base + f + 32 * b, base + 2 * f + 32 * b,
                                        base + 3 * f + 32 * b, base + 4 * f + 32 * b, base + 5 * f + b,
                                        (uint32_t)m, work, gcomb, st, nullptr, nullptr, 1))
                return SBFT_GV_ELAUNCH;
        }
        HIPCHK(hipEventRecord(ev_join, sl->stream2));
        HIPCHK(hipStreamWaitEvent(sl->stream, ev_join, 0));
        HIPCHK(hipMemcpyAsync(ok_out + c.begin, base + 5 * f, c.count, hipMemcpyDeviceToHost, sl->stream));
        return SBFT_GV_OK;
    };
    rc = body();
    if (rc) {
        (void)hipStreamSynchronize(sl->copy_stream);
        (void)hipStreamSynchronize(sl->stream2);
    }
    return rc;
}

// Framed verify batches on the small-batch kernels hash inside the verify launch
// (sbft_launch_p256_verify_framed). SBFT_VP_FUSED=0: gather + hash + verify kernels (A/B only).
bool framed_fused_on() {
    static const bool on = [] {
        const char* e = getenv("SBFT_VP_FUSED");
        return !e || e[0] != '0';
    }();
    return on;
}

// Hash (and optionally verify) messages [c.begin, +c.count). Offsets are rebased to the
// chunk's first message so each device receives only its slice of the blob.
// framed: verify inputs are gathered on the device from the blob itself (r || s at message
// end + sig_rel, x || y at message end + pub_rel) instead of copied from r, s, qx, qy.
// kid (optional): registered client key id per message (all non-zero); a share of at least
// keyed_min messages then takes the keyed launch over the clients' comb tables
// (sbft_launch_p256_verify_keyed_framed, hash on a fifth wavefront), as the one-slot
// VerifyProposal path does.
struct Framing {
    bool on = false;
    int32_t sig_rel = 0, pub_rel = 0;
    const uint32_t* kid = nullptr;
    uint32_t nkeys = 0;
    size_t keyed_min = 0;
};
int enqueue_hash(const Chunk& c, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                 const uint32_t* len, const uint8_t* r, const uint8_t* s, const uint8_t* qx,
                 const uint8_t* qy, uint8_t* ok_out, uint8_t* dig_out, std::vector<uint64_t>& rebased,
                 Framing fr = Framing()) {
    Slot* sl = c.slot;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t k = c.begin; k < c.begin + c.count; ++k) {
        if (off[k] + len[k] > blob_len || off[k] + len[k] < off[k]) return SBFT_GV_EINVAL;
        lo = std::min(lo, off[k]);
        hi = std::max(hi, off[k] + len[k]);
        if (fr.on) {
            const int64_t end = (int64_t)(off[k] + len[k]);
            for (int32_t rel : {fr.sig_rel, fr.pub_rel}) {
                const int64_t a = end + rel;
                if (a < 0 || (uint64_t)a + 64 > blob_len) return SBFT_GV_EINVAL;
                lo = std::min(lo, (uint64_t)a);
                hi = std::max(hi, (uint64_t)a + 64);
            }
        }
    }
    if (c.count == 0) return SBFT_GV_OK;
    rebased.resize(c.count);
    for (size_t k = 0; k < c.count; ++k) rebased[k] = off[c.begin + k] - lo;
    const size_t span = hi - lo;
    const size_t fb = align_up(span + SBFT_GV_SHA_BLOB_PAD, 256);  // the hash kernel's over-read
    const size_t fo = align_up(8 * c.count, 256), fl = align_up(4 * c.count, 256);
    const size_t fd = align_up(32 * c.count, 256);
    const bool verify = ok_out != nullptr;
    if (fr.on && verify && fr.kid && fr.keyed_min && c.count >= fr.keyed_min) {
        // registered clients: blob | off | len | key ids | ok (caller holds sl->mu)
        HIPCHK(hipSetDevice(sl->device));
        const size_t fk = align_up(4 * c.count, 256);
        int rc = ensure_tables(sl, fr.nkeys);
        if (!rc) rc = sl->reserve(fb + fo + fl + fk + align_up(c.count, 256));
        if (rc) return rc;
        uint8_t* b = sl->dbuf;
        uint8_t *d_blob = b, *d_off = b + fb, *d_len = d_off + fo, *d_kid = d_len + fl, *d_ok = d_kid + fk;
        HIPCHK(hipMemcpyAsync(d_blob, blob + lo, span, hipMemcpyHostToDevice, sl->stream));
        HIPCHK(hipMemcpyAsync(d_off, rebased.data(), 8 * c.count, hipMemcpyHostToDevice, sl->stream));
        HIPCHK(hipMemcpyAsync(d_len, len + c.begin, 4 * c.count, hipMemcpyHostToDevice, sl->stream));
        HIPCHK(hipMemcpyAsync(d_kid, fr.kid + c.begin, 4 * c.count, hipMemcpyHostToDevice, sl->stream));
        if (sbft_launch_p256_verify_keyed_framed(d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len, fr.sig_rel,
                                                 (const uint32_t*)d_kid, (const void* const*)sl->d_keytab, fr.nkeys,
                                                 d_ok, (uint32_t)c.count, sl->stream))
            return SBFT_GV_ELAUNCH;
        HIPCHK(hipMemcpyAsync(ok_out + c.begin, d_ok, c.count, hipMemcpyDeviceToHost, sl->stream));
        return SBFT_GV_OK;
    }
    // blob | off | len | work counter | digests [| r | s | qx | qy | ok | verify workspace]
    // [| longest-first sort scratch | order]
    const bool lpt = c.count >= kShaLptMin;
    const size_t f_lpt = lpt ? align_up(sbft_sha256_lpt_ws_bytes(), 256) + align_up(4 * c.count, 256) : 0;
    const size_t need = fb + fo + fl + 256 + fd +
                        (verify ? 4 * fd + align_up(c.count, 256) + sbft_verify_work_bytes(c.count) : 0) + f_lpt;
    HIPCHK(hipSetDevice(sl->device));
    int rc = sl->reserve(need);
    if (rc) return rc;
    uint8_t* b = sl->dbuf;
    uint8_t *d_blob = b, *d_off = b + fb, *d_len = d_off + fo, *d_ctr = d_len + fl, *d_dig = d_ctr + 256;
    HIPCHK(hipMemcpyAsync(d_blob, blob + lo, span, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(d_off, rebased.data(), 8 * c.count, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(d_len, len + c.begin, 4 * c.count, hipMemcpyHostToDevice, sl->stream));
    // `rebased` is owned by the caller until the stream is synchronised
    const bool fused = fr.on && verify && !dig_out && c.lanes >= 2 && framed_fused_on();
    uint32_t* ord = nullptr;
    if (lpt && !fused) {
        uint8_t* w = b + need - f_lpt;
        ord = (uint32_t*)(w + align_up(sbft_sha256_lpt_ws_bytes(), 256));
        if (sbft_launch_sha256_lpt_order((const uint32_t*)d_len, (uint32_t)c.count, (uint32_t*)w, ord, sl->stream))
            return SBFT_GV_ELAUNCH;
    }
    if (!fused && sbft_launch_sha256(d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len, ord, d_dig,
                                     (uint32_t)c.count, (uint32_t*)d_ctr, sl->stream))
        return SBFT_GV_ELAUNCH;
    if (fused) {
        uint8_t* v = d_dig + fd;
        uint8_t* d_ok = v + 4 * fd;
        uint32_t* work = (uint32_t*)(d_ok + align_up(c.count, 256));
        const void* gcomb = sl->gcomb_table();
        if (!gcomb) return SBFT_GV_ENOMEM;
        if (hipMemsetAsync(work, 0, sizeof(uint32_t), sl->stream) != hipSuccess ||
            sbft_launch_p256_verify_framed(d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len,
                                           (uint32_t)c.count, fr.sig_rel, fr.pub_rel, d_dig, v, v + fd, v + 2 * fd,
                                           v + 3 * fd, d_ok, work, gcomb, sl->stream, c.lanes))
            return SBFT_GV_ELAUNCH;
        HIPCHK(hipMemcpyAsync(ok_out + c.begin, d_ok, c.count, hipMemcpyDeviceToHost, sl->stream));
    } else if (verify) {
        uint8_t* v = d_dig + fd;
        if (fr.on) {
            if (sbft_launch_gather_framed(d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len,
                                          (uint32_t)c.count, fr.sig_rel, fr.pub_rel, v, v + fd, v + 2 * fd,
                                          v + 3 * fd, sl->stream))
                return SBFT_GV_ELAUNCH;
        } else {
            const uint8_t* src[4] = {r, s, qx, qy};
            for (int k = 0; k < 4; ++k)
                HIPCHK(hipMemcpyAsync(v + k * fd, src[k] + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice,
                                      sl->stream));
        }
        uint8_t* d_ok = v + 4 * fd;
        uint32_t* work = (uint32_t*)(d_ok + align_up(c.count, 256));
        const void* gcomb = sl->gcomb_table();
        if (!gcomb) return SBFT_GV_ENOMEM;
        if (sbft_launch_p256_verify(d_dig, v, v + fd, v + 2 * fd, v + 3 * fd, d_ok, (uint32_t)c.count,
                                    work, gcomb, sl->stream, nullptr, nullptr, c.lanes))
            return SBFT_GV_ELAUNCH;
        HIPCHK(hipMemcpyAsync(ok_out + c.begin, d_ok, c.count, hipMemcpyDeviceToHost, sl->stream));
    }
    if (dig_out)
        HIPCHK(hipMemcpyAsync(dig_out + 32 * c.begin, d_dig, 32 * c.count, hipMemcpyDeviceToHost,
                              sl->stream));
    // the rebased offsets are read by the async H2D: keep them alive until the sync
    return SBFT_GV_OK;
}

// Sign tuples [c.begin, +c.count): inputs d | k | digest, outputs qx | qy | r | s | status.
int enqueue_sign(const Chunk& c, const uint8_t* d, const uint8_t* k, const uint8_t* digest, uint8_t* qx,
                 uint8_t* qy, uint8_t* r, uint8_t* s, uint8_t* status) {
    Slot* sl = c.slot;
    const size_t f = align_up(32 * c.count, 256);
    HIPCHK(hipSetDevice(sl->device));
    int rc = sl->reserve(7 * f + align_up(c.count, 256));
    if (rc) return rc;
    uint8_t* b = sl->dbuf;
    const uint8_t* src[3] = {d, k, digest};
    for (int i = 0; i < 3; ++i)
        HIPCHK(hipMemcpyAsync(b + i * f, src[i] + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice,
                              sl->stream));
    if (sbft_launch_p256_sign(b, b + f, b + 2 * f, b + 3 * f, b + 4 * f, b + 5 * f, b + 6 * f, b + 7 * f,
                              (uint32_t)c.count, sl->stream))
        return SBFT_GV_ELAUNCH;
    uint8_t* dst[4] = {qx, qy, r, s};
    for (int i = 0; i < 4; ++i)
        HIPCHK(hipMemcpyAsync(dst[i] + 32 * c.begin, b + (3 + i) * f, 32 * c.count, hipMemcpyDeviceToHost,
                              sl->stream));
    HIPCHK(hipMemcpyAsync(status + c.begin, b + 7 * f, c.count, hipMemcpyDeviceToHost, sl->stream));
    return SBFT_GV_OK;
}

int enqueue_selftest(const Chunk& c, int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
    Slot* sl = c.slot;
    const size_t f = align_up(32 * c.count, 256);
    HIPCHK(hipSetDevice(sl->device));
    int rc = sl->reserve(3 * f);
    if (rc) return rc;
    uint8_t* d = sl->dbuf;
    HIPCHK(hipMemcpyAsync(d, a + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(d + f, b + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice, sl->stream));
    if (sbft_launch_selftest(op, d, d + f, d + 2 * f, (uint32_t)c.count, sl->stream)) return SBFT_GV_ELAUNCH;
    HIPCHK(hipMemcpyAsync(out + 32 * c.begin, d + 2 * f, 32 * c.count, hipMemcpyDeviceToHost, sl->stream));
    return SBFT_GV_OK;
}

// Each device chunk is enqueued and synchronised by its own host thread (for_each_device);
// a chunk's slot is locked by the thread that drives it.
// One device's share of a split VerifyProposal (the multi-device branch of
// sbft_gv_framed_overlapped) in the one-slot path's form: the share's offsets and lengths and its
// verdicts live in the slot's mapped host memory (no copies of them), the payload slice is the
// one DMA, and the fused hash + verify launch is followed by the fix-up kernel only when the
// kernel raised the mapped flag. The fix-up counter at dbuf's start is cleared only when another
// path used dbuf since this path's last call, or that call flagged a tuple (a clean call leaves it
// 0). Synchronous. The caller holds the slot's lock.
int enqueue_framed_share(const Chunk& c, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                         const uint32_t* len, int32_t sig_rel, int32_t pub_rel, uint8_t* ok_out) {
    Slot* sl = c.slot;
    const size_t n = c.count, b = c.begin;
    if (n == 0) return SBFT_GV_OK;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t k = b; k < b + n; ++k) {
        if (off[k] + len[k] > blob_len || off[k] + len[k] < off[k]) return SBFT_GV_EINVAL;
        lo = std::min(lo, off[k]);
        hi = std::max(hi, off[k] + len[k]);
        const int64_t end = (int64_t)(off[k] + len[k]);
        for (int32_t rel : {sig_rel, pub_rel}) {
            const int64_t a = end + rel;
            if (a < 0 || (uint64_t)a + 64 > blob_len) return SBFT_GV_EINVAL;
            lo = std::min(lo, (uint64_t)a);
            hi = std::max(hi, (uint64_t)a + 64);
        }
    }
    const size_t span = hi - lo;
    const size_t fw = align_up(sbft_verify_work_bytes(n), 256);
    const size_t fb = align_up(span + SBFT_GV_SHA_BLOB_PAD, 256);  // + the hash's over-read
    const size_t fd = align_up(32 * n, 256), fo = align_up(8 * n, 256), fl = align_up(4 * n, 256);
    HIPCHK(hipSetDevice(sl->device));
    const uint64_t gen0 = sl->dgen;
    const bool clean = sl->share_clean_at == sl->duses;  // nobody used dbuf since our clean call
    int rc = sl->reserve(fw + fb + 5 * fd);  // work | blob | digests | r | s | qx | qy
    if (!rc) rc = sl->reserve_vmap(fo + fl + align_up(n, 256) + 256);
    if (rc) return rc;
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    sl->share_clean_at = UINT64_MAX;
    uint8_t* d = sl->dbuf;
    uint8_t *d_work = d, *d_blob = d + fw, *d_dig = d_blob + fb, *v = d_dig + fd;
    uint64_t* ho = (uint64_t*)sl->vmap;
    uint32_t* hl = (uint32_t*)(sl->vmap + fo);
    for (size_t k = 0; k < n; ++k) {
        ho[k] = off[b + k] - lo;
        hl[k] = len[b + k];
    }
    uint8_t* const h_ok = sl->vmap + fo + fl;
    const uint8_t* vd = sl->vmap_dev;
    uint8_t* const d_hok = sl->vmap_dev + fo + fl;
    volatile uint32_t* const flag = (volatile uint32_t*)(h_ok + align_up(n, 256));
    *flag = 0;
    if ((!clean || sl->dgen != gen0) && hipMemsetAsync(d_work, 0, sizeof(uint32_t), sl->stream) != hipSuccess)
        return SBFT_GV_EDEVICE;
    HIPCHK(hipMemcpyAsync(d_blob, blob + lo, span, hipMemcpyHostToDevice, sl->stream));
    if (sbft_launch_p256_verify_framed(d_blob, (const uint64_t*)vd, (const uint32_t*)(vd + fo), (uint32_t)n, sig_rel,
                                       pub_rel, d_dig, v, v + fd, v + 2 * fd, v + 3 * fd, d_hok, (uint32_t*)d_work,
                                       gcomb, sl->stream, c.lanes, (uint32_t*)(d_hok + align_up(n, 256))))
        return SBFT_GV_ELAUNCH;
    HIPCHK(stream_sync(sl->stream));
    if (*flag) {
        if (sbft_launch_p256_verify_fixup(d_dig, v, v + fd, v + 2 * fd, v + 3 * fd, d_hok, (const uint32_t*)d_work,
                                          (uint32_t)n, sl->stream))
            return SBFT_GV_ELAUNCH;
        HIPCHK(stream_sync(sl->stream));
    } else {
        sl->share_clean_at = sl->duses;  // the counter stays 0 for the next share call
    }
    std::memcpy(ok_out + b, h_ok, n);
    return SBFT_GV_OK;
}

template <class F>
int run_chunks(sbft_gv_ctx* ctx, size_t n, F&& enqueue) {
    std::vector<Chunk> chunks = plan(ctx, n);
    return for_each_device(ctx, chunks.size(), [&](size_t i) {
        const Chunk& c = chunks[i];
        std::lock_guard<std::mutex> lk(c.slot->mu);
        int rc = enqueue(c, i);
        (void)hipSetDevice(c.slot->device);
        if (stream_sync(c.slot->stream) != hipSuccess && rc == SBFT_GV_OK) rc = SBFT_GV_EDEVICE;
        return rc;
    });
}

}  // namespace

extern "C" {

int sbft_gv_verify_p256(sbft_gv_ctx* ctx, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                        const uint8_t* qx, const uint8_t* qy, size_t n, uint8_t* ok_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!digest || !r || !s || !qx || !qy || !ok_out || n > 0xffffffffu) return SBFT_GV_EINVAL;
    // Large chunks are cut into sub-batches whose copies (copy stream) overlap the verify of
    // the earlier ones; pageable inputs are gathered into page-locked staging first (handing
    // the runtime pageable pointers measured no overlap: 51.2 vs 52.2 M verifies/s; staged: 53.0-53.8,
    // profiles/r02c_host_pipe_ab.txt). SBFT_PIPE_PAGEABLE=0 keeps pageable inputs unpipelined.
    static const bool pipe_pageable = getenv("SBFT_PIPE_PAGEABLE") ? atoi(getenv("SBFT_PIPE_PAGEABLE")) != 0 : true;
    const bool pipe = n >= 2 * kPipeSub &&
                      (pipe_pageable || (is_pinned(digest) && is_pinned(r) && is_pinned(s) && is_pinned(qx) &&
                                         is_pinned(qy)));
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) {
        if (pipe && c.lanes == 1 && c.count >= 2 * kPipeSub)
            return enqueue_verify_piped(c, digest, r, s, qx, qy, ok_out);
        return enqueue_verify(c, digest, r, s, qx, qy, ok_out);
    });
}

int sbft_gv_verify_p256_kernel(sbft_gv_ctx* ctx, int kernel, const uint8_t* digest, const uint8_t* r,
                               const uint8_t* s, const uint8_t* qx, const uint8_t* qy, size_t n, uint8_t* ok_out) {
    if (!ctx || kernel < SBFT_GV_KERNEL_EXACT || kernel > SBFT_GV_KERNEL_HALF_WIDE) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!digest || !r || !s || !qx || !qy || !ok_out || n > 0xffffffffu) return SBFT_GV_EINVAL;
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) {
        Chunk k = c;
        k.lanes = kernel;
        return enqueue_verify(k, digest, r, s, qx, qy, ok_out);
    });
}

int sbft_gv_sign_p256(sbft_gv_ctx* ctx, const uint8_t* d, const uint8_t* k, const uint8_t* digest,
                      size_t n, uint8_t* qx, uint8_t* qy, uint8_t* r, uint8_t* s, uint8_t* status) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!d || !k || !digest || !r || !s || !status || !qx != !qy || n > 0xffffffffu) return SBFT_GV_EINVAL;
    // latency path (api.Signer: one signature per call): two wavefronts per signature over G's
    // comb table instead of one lane running two scalar multiplications alone
    if (n <= kSignWaveMax) return sign_wave(ctx, d, k, digest, n, qx, qy, r, s, status);
    std::vector<uint8_t> qtmp;  // the one-lane kernel always derives Q
    if (!qx) {
        qtmp.resize(64 * n);
        qx = qtmp.data();
        qy = qtmp.data() + 32 * n;
    }
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) {
        return enqueue_sign(c, d, k, digest, qx, qy, r, s, status);
    });
}

int sbft_gv_selftest_field(sbft_gv_ctx* ctx, int op, const uint8_t* a, const uint8_t* b, size_t n,
                           uint8_t* out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!a || !b || !out || op < 0 || op > 30 || n > 0xffffffffu) return SBFT_GV_EINVAL;
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) { return enqueue_selftest(c, op, a, b, out); });
}

int sbft_gv_sha256(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                   const uint32_t* len, size_t n, uint8_t* dig_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if ((!blob && blob_len) || !off || !len || !dig_out || n > 0xffffffffu) return SBFT_GV_EINVAL;
    std::vector<std::vector<uint64_t>> rebased(ctx->slots.size() + 1);
    return run_chunks(ctx, n, [&](const Chunk& c, size_t i) {
        return enqueue_hash(c, blob, blob_len, off, len, nullptr, nullptr, nullptr, nullptr, nullptr,
                            dig_out, rebased[i]);
    });
}

int sbft_gv_sha256_verify_p256(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len,
                               const uint64_t* off, const uint32_t* len, const uint8_t* r,
                               const uint8_t* s, const uint8_t* qx, const uint8_t* qy, size_t n,
                               uint8_t* ok_out, uint8_t* dig_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if ((!blob && blob_len) || !off || !len || !r || !s || !qx || !qy || !ok_out || n > 0xffffffffu)
        return SBFT_GV_EINVAL;
    std::vector<std::vector<uint64_t>> rebased(ctx->slots.size() + 1);
    return run_chunks(ctx, n, [&](const Chunk& c, size_t i) {
        return enqueue_hash(c, blob, blob_len, off, len, r, s, qx, qy, ok_out, dig_out, rebased[i]);
    });
}

int sbft_gv_sha256_verify_p256_framed(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len,
                                      const uint64_t* off, const uint32_t* len, size_t n, int32_t sig_rel,
                                      int32_t pub_rel, uint8_t* ok_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!blob || !off || !len || !ok_out || n > 0xffffffffu) return SBFT_GV_EINVAL;
    std::vector<std::vector<uint64_t>> rebased(ctx->slots.size() + 1);
    Framing fr;
    fr.on = true;
    fr.sig_rel = sig_rel;
    fr.pub_rel = pub_rel;
    return run_chunks(ctx, n, [&](const Chunk& c, size_t i) {
        if (framed_fused_on() && c.lanes >= 2)  // the fused launch, offsets and verdicts in mapped memory
            return enqueue_framed_share(c, blob, blob_len, off, len, sig_rel, pub_rel, ok_out);
        return enqueue_hash(c, blob, blob_len, off, len, nullptr, nullptr, nullptr, nullptr, ok_out, nullptr,
                            rebased[i], fr);
    });
}

}  // extern "C"

int sbft_gv_framed_overlapped(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len, int32_t sig_rel,
                              int32_t pub_rel,
                              const std::function<int(std::vector<uint64_t>&, std::vector<uint32_t>&)>& prepare,
                              std::vector<uint8_t>& ok, const std::function<void()>& during,
                              const std::vector<uint32_t>* kid) {
    if (!ctx || (!blob && blob_len)) return SBFT_GV_EINVAL;
    // this thread's scratch, bound to references: a lambda running on the helper thread must
    // see these objects, not the helper's own thread_local instances
    thread_local std::vector<uint64_t> off_tl;
    thread_local std::vector<uint32_t> len_tl;
    std::vector<uint64_t>& off = off_tl;
    std::vector<uint32_t>& len = len_tl;
    off.clear();
    len.clear();
    static const bool trace = getenv("SBFT_VP_TRACE") != nullptr;  // diagnostics
    using TC = std::chrono::steady_clock;
    const auto t0 = TC::now();
    Slot* sl = ctx->slots[ctx->rr.fetch_add(1) % ctx->slots.size()];
    std::unique_lock<std::mutex> lk(sl->mu);
    HIPCHK(hipSetDevice(sl->device));
    int rc = sl->reserve_blob(blob_len + SBFT_GV_SHA_BLOB_PAD);  // + the hash kernel's over-read
    if (rc) return rc;
    // the helper stages the payload for the DMA (a pageable copy runs on the CPU) while this
    // thread parses: the parse is a chain of dependent loads through the payload, fastest on
    // the caller's core, whose caches typically hold it; the copy streams it from anywhere
    hipError_t ce = hipSuccess;
    const int dev = sl->device;
    // the fused launch's fixup counter (d_work's first word, at a fixed offset of the device
    // buffer): cleared ahead of the payload copy, so no fill sits between the parse and the
    // verify launch (cleared again below only if the buffer is reallocated)
    uint8_t* const pre_dbuf = sl->dbuf;
    const uint64_t pre_gen = sl->dgen;
    if (pre_dbuf && hipMemsetAsync(pre_dbuf + 256, 0, sizeof(uint32_t), sl->stream) != hipSuccess)
        return SBFT_GV_EDEVICE;
    TC::time_point tcs{}, tce{};  // the payload copy's start and return (SBFT_VP_TRACE)
    auto copy = [&] {
        if (trace) tcs = TC::now();
        if (blob_len && (ce = hipSetDevice(dev)) == hipSuccess)
            ce = hipMemcpyAsync(sl->bbuf, blob, blob_len, hipMemcpyHostToDevice, sl->stream);
        if (trace) tce = TC::now();
    };
    // A batch that may be split over the slots copies per share (each device its own slice): the
    // whole-payload copy to this slot would be wasted, and the split path waits for it. Each framed
    // message spans at least 128 bytes of the blob (a 64-byte key inside it, r || s after it), so
    // with blob_len < 128 min_split no split is possible and the copy overlaps the parse as before.
    const bool may_split = ctx->slots.size() > 1 && blob_len / 128 >= ctx->min_split;
    bool async = false;
    // SBFT_VP_COPY_FIRST=1 (diagnostics): the copy on this thread before the parse, not beside it
    static const bool copy_first = [] {
        const char* e = getenv("SBFT_VP_COPY_FIRST");
        return e && e[0] == '1';
    }();
    if (!may_split) {
        async = !copy_first && ctx->helper.try_submit(copy);
        if (!async) copy();
    }
    const auto t1 = TC::now();
    const int prc = prepare(off, len);
    const auto t2 = TC::now();
    // While the helper still stages the payload copy (it ends ~20 us after the parse): check the
    // parsed offsets and put them into the mapped host memory the launches below read -- all
    // that needs only the parse (~7 us of a 10k-request call). Errors are returned after the
    // helper has finished (its job holds references to this frame).
    const size_t n = off.size();
    const bool split = n >= ctx->min_split && ctx->slots.size() > 1;
    if (may_split && !split && !prc) copy();  // not split after all: the copy the parse did not overlap
    const size_t fo = align_up(8 * n, 256), fl = align_up(4 * n, 256);
    int src = SBFT_GV_OK;
    if (!prc && n > 0 && !split) {
        if (len.size() != n || n > 0xffffffffu) src = SBFT_GV_EINVAL;
        for (size_t k = 0; !src && k < n; ++k) {
            if (off[k] + len[k] > blob_len || off[k] + len[k] < off[k]) src = SBFT_GV_EINVAL;
            const int64_t end = (int64_t)(off[k] + len[k]);
            for (int32_t rel : {sig_rel, pub_rel})
                if (end + rel < 0 || (uint64_t)(end + rel) + 64 > blob_len) src = SBFT_GV_EINVAL;
        }
        // room for both layouts: offsets | lengths | key ids | verdicts (registered) and
        // offsets | lengths | verdicts | fix-up flag (generic)
        if (!src) src = sl->reserve_vmap(fo + 2 * fl + align_up(n, 256) + 256);
        if (!src) {
            std::memcpy(sl->vmap, off.data(), 8 * n);
            std::memcpy(sl->vmap + fo, len.data(), 4 * n);
        }
    }
    if (async) ctx->helper.wait();
    // No stream synchronisation here: the launches below queue behind the payload copy on the
    // same stream, so the verify starts as the DMA ends instead of one host round trip later
    // (a pageable copy returns once its source is staged: the caller's buffer is free). A DMA
    // fault surfaces at the closing synchronisation. SBFT_VP_SYNC=1: wait here (A/B only).
    static const bool sync_after_copy = [] {
        const char* e = getenv("SBFT_VP_SYNC");
        return e && e[0] == '1';
    }();
    const int sync_rc = (!sync_after_copy || stream_sync(sl->stream) == hipSuccess) && ce == hipSuccess
                            ? SBFT_GV_OK
                            : SBFT_GV_EDEVICE;
    const auto t3 = TC::now();
    // From here the payload copy may still be in flight (possibly a DMA from the caller's
    // page-locked buffer): every return drains this slot's stream first, so the caller's buffer
    // is free and a copy fault is reported by this call, not by the slot's next user. (The
    // launch paths end in a synchronisation of their own and disarm it.)
    struct Drain {
        hipStream_t st;
        bool armed;
        ~Drain() {
            if (armed) (void)hipStreamSynchronize(st);
        }
    } drain{sl->stream, true};
    struct Tr {
        bool on;
        TC::time_point a, b, c, d, e, f;  // e: offsets staged, f: launch returned (fused path)
        bool async;
        const TC::time_point *cs, *ce;  // the copy's start and return
        ~Tr() {
            if (!on) return;
            auto us = [](TC::time_point x, TC::time_point y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
            const TC::time_point z = TC::now();
            if (f == TC::time_point{}) e = f = d;
            const bool cp = *cs != TC::time_point{} && *ce != TC::time_point{};
            fprintf(stderr, "vp async=%d submit=%.1f parse=%.1f copy_wait_sync=%.1f stage=%.1f launch=%.1f rest=%.1f us"
                    " copy=%.1f,%.1f\n",
                    (int)async, us(a, b), us(b, c), us(c, d), us(d, e), us(e, f), us(f, z), cp ? us(a, *cs) : -1.0,
                    cp ? us(a, *ce) : -1.0);
        }
    } tr{trace, t0, t1, t2, t3, {}, {}, async, &tcs, &tce};
    if (prc) return prc;
    if (sync_rc) return sync_rc;
    ok.assign(n, 0);
    if (n == 0) return SBFT_GV_OK;
    if (len.size() != n || n > 0xffffffffu) return SBFT_GV_EINVAL;
    if (split) {  // large: the multi-device split path
        // each share copies its own slice of the payload (this slot made no copy of the whole)
        drain.armed = false;
        if (!may_split && stream_sync(sl->stream) != hipSuccess) return SBFT_GV_EDEVICE;
        lk.unlock();
        Framing fr;
        fr.on = true;
        fr.sig_rel = sig_rel;
        fr.pub_rel = pub_rel;
        if (kid && kid->size() == n) {
            fr.kid = kid->data();
            fr.nkeys = (uint32_t)ctx->nkeys.load();
            fr.keyed_min = ctx->keyed_lanes_min;
        }
        std::vector<std::vector<uint64_t>> rebased(ctx->slots.size() + 1);
        // The shares run on the context's workers (share i on worker i + 1) while this thread does
        // the caller's host work (`during`: the full format check and the RequestInfo records),
        // as the one-slot path does it under its launch.
        const std::vector<Chunk> chunks = plan(ctx, n);
        // SBFT_VP_TRACE: each share's pick-up and end on its worker, from the call's start
        std::vector<std::array<TC::time_point, 2>> sh(trace ? chunks.size() + 1 : 0);
        const TC::time_point ts = TC::now();
        struct ShareTrace {
            const std::vector<std::array<TC::time_point, 2>>& sh;
            TC::time_point t0, ts;
            ~ShareTrace() {
                if (sh.empty()) return;
                auto us = [](TC::time_point x, TC::time_point y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
                fprintf(stderr, "vp-split start=%.1f", us(t0, ts));
                for (size_t i = 0; i < sh.size(); ++i)
                    fprintf(stderr, " s%zu=%.1f,%.1f", i, us(t0, sh[i][0]), us(t0, sh[i][1]));
                fprintf(stderr, "\n");
            }
        } share_trace{sh, t0, ts};
        return for_each_device(ctx, chunks.size() + 1, [&](size_t i) -> int {
            if (!sh.empty()) sh[i][0] = TC::now();
            struct End {
                std::array<TC::time_point, 2>* e;
                ~End() {
                    if (e) (*e)[1] = TC::now();
                }
            } end{sh.empty() ? nullptr : &sh[i]};
            if (i == 0) {
                if (during) during();
                return SBFT_GV_OK;
            }
            const Chunk& c = chunks[i - 1];
            std::lock_guard<std::mutex> slk(c.slot->mu);
            int rc;
            // a share the fused hash + verify launch takes: the one-slot path's mapped-memory form
            if (framed_fused_on() && c.lanes >= 2 && !(fr.kid && fr.keyed_min && c.count >= fr.keyed_min))
                rc = enqueue_framed_share(c, blob, blob_len, off.data(), len.data(), sig_rel, pub_rel, ok.data());
            else
                rc = enqueue_hash(c, blob, blob_len, off.data(), len.data(), nullptr, nullptr, nullptr, nullptr,
                                  ok.data(), nullptr, rebased[i - 1], fr);
            (void)hipSetDevice(c.slot->device);
            if (stream_sync(c.slot->stream) != hipSuccess && rc == SBFT_GV_OK) rc = SBFT_GV_EDEVICE;
            return rc;
        });
    }
    if (src) return src;  // the bounds checks and the offsets' staging above
    // Every request signed by a registered client key (kid[k] != 0 for all k, filled by
    // prepare): the keyed four-lane kernel over the clients' comb tables, hashing on a fifth
    // wavefront per workgroup and reading r || s from the payload; key ids beside the offsets
    // in mapped host memory. Smaller batches go through the caller's other paths.
    if (kid && kid->size() == n && ctx->keyed_lanes_min && n >= ctx->keyed_lanes_min) {
        const uint32_t nkeys = (uint32_t)ctx->nkeys.load();
        rc = ensure_tables(sl, nkeys);
        if (!rc) rc = sl->reserve(align_up(n, 256));
        if (rc) return rc;
        std::memcpy(sl->vmap + fo + fl, kid->data(), 4 * n);  // offsets, lengths: staged above
        const uint8_t* vd = sl->vmap_dev;
        // verdicts straight to mapped host memory (no device-to-host copy after the launch)
        LaunchTimer kt(ctx, sl->stream);
        if (sbft_launch_p256_verify_keyed_framed(sl->bbuf, (const uint64_t*)vd, (const uint32_t*)(vd + fo), sig_rel,
                                                 (const uint32_t*)(vd + fo + fl), (const void* const*)sl->d_keytab,
                                                 nkeys, sl->vmap_dev + fo + 2 * fl, (uint32_t)n, sl->stream))
            return SBFT_GV_ELAUNCH;
        kt.end();
        if (during) during();  // the caller's host work that does not need the verdicts
        HIPCHK(stream_sync(sl->stream));
        drain.armed = false;
        std::memcpy(ok.data(), sl->vmap + fo + 2 * fl, n);
        return SBFT_GV_OK;
    }
    // Device: hash counter (256) | verify workspace | digests | r | s | qx | qy | ok. The
    // offsets and lengths stay in mapped host memory that the gather and hash kernels read
    // over PCIe, and the gather launch (first on the stream) zeroes both counters: no copy and
    // no memset launch between the parse and the hash (a pageable copy each and two memsets
    // cost ~40 us of the ~1 ms call, one pinned copy still ~25 us with its engine hand-off).
    const size_t fd = align_up(32 * n, 256);
    const size_t fw = align_up(sbft_verify_work_bytes(n), 256);
    rc = sl->reserve(256 + fw + 5 * fd + align_up(n, 256));
    if (rc) return rc;
    uint8_t* b = sl->dbuf;
    uint8_t *d_ctr = b, *d_work = d_ctr + 256, *d_dig = d_work + fw;
    uint8_t* v = d_dig + fd;
    uint8_t* d_ok = v + 4 * fd;
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    const uint64_t* d_off = (const uint64_t*)sl->vmap_dev;
    const uint32_t* d_len = (const uint32_t*)(sl->vmap_dev + fo);
    // Small batches (lanes 2 / 4) hash inside the verify launch, on a second wavefront per
    // workgroup that runs while the first builds its Q tables: no gather or hash kernel in
    // front (~37 us of a 10k-tuple call).
    const int lanes = ctx->lanes_for(n);
    if (framed_fused_on() && lanes >= 2) {
        // the verdicts go straight to mapped host memory (n bytes over PCIe from the kernels'
        // stores): no device-to-host copy and no copy-engine hand-off after the verify
        if (trace) tr.e = TC::now();
        uint8_t* const h_ok = sl->vmap + fo + fl;
        uint8_t* const d_hok = sl->vmap_dev + fo + fl;
        // the fixup kernel (the exact net for flagged tuples, which the in-place repair leaves
        // none of in practice) runs only if the verify kernel raised this mapped flag
        volatile uint32_t* const flag = (volatile uint32_t*)(h_ok + align_up(n, 256));
        *flag = 0;
        if ((!pre_dbuf || sl->dgen != pre_gen) && hipMemsetAsync(d_work, 0, sizeof(uint32_t), sl->stream) != hipSuccess)
            return SBFT_GV_ELAUNCH;
        LaunchTimer kt(ctx, sl->stream);  // sbft_gv_kernel_timing: the fused hash + verify kernel
        if (sbft_launch_p256_verify_framed(sl->bbuf, d_off, d_len, (uint32_t)n, sig_rel, pub_rel, d_dig, v, v + fd,
                                           v + 2 * fd, v + 3 * fd, d_hok, (uint32_t*)d_work, gcomb, sl->stream, lanes,
                                           (uint32_t*)(d_hok + align_up(n, 256))))
            return SBFT_GV_ELAUNCH;
        kt.end();
        if (trace) tr.f = TC::now();
        if (during) during();
        HIPCHK(stream_sync(sl->stream));
        if (*flag) {
            if (sbft_launch_p256_verify_fixup(d_dig, v, v + fd, v + 2 * fd, v + 3 * fd, d_hok, (const uint32_t*)d_work,
                                              (uint32_t)n, sl->stream))
                return SBFT_GV_ELAUNCH;
            HIPCHK(stream_sync(sl->stream));
        }
        drain.armed = false;
        std::memcpy(ok.data(), h_ok, n);
        return SBFT_GV_OK;
    } else if (sbft_launch_gather_framed(sl->bbuf, d_off, d_len, (uint32_t)n, sig_rel, pub_rel, v, v + fd,
                                         v + 2 * fd, v + 3 * fd, sl->stream, (uint32_t*)d_ctr, (uint32_t*)d_work) ||
               sbft_launch_sha256(sl->bbuf, d_off, d_len, nullptr, d_dig, (uint32_t)n, (uint32_t*)d_ctr, sl->stream,
                                  1) ||
               sbft_launch_p256_verify(d_dig, v, v + fd, v + 2 * fd, v + 3 * fd, d_ok, (uint32_t)n,
                                       (uint32_t*)d_work, gcomb, sl->stream, nullptr, nullptr, lanes, 1)) {
        return SBFT_GV_ELAUNCH;
    }
    // the caller's host work that does not need the verdicts, under the launch: before the
    // verdict copy, which (into pageable memory) returns only once the kernel has finished
    if (during) during();
    HIPCHK(hipMemcpyAsync(ok.data(), d_ok, n, hipMemcpyDeviceToHost, sl->stream));
    HIPCHK(stream_sync(sl->stream));
    drain.armed = false;
    return SBFT_GV_OK;
}

// ---------------------------------------------------------------- streamed hash + verify
namespace {

constexpr size_t kStreamWindowDefault = (size_t)256 << 20;  // payload bytes per window
// windows in flight per device. Hashing is serial within a message (a 64 KiB message is 1,024
// dependent compressions), so one window of a few hundred long messages occupies a few CUs for
// milliseconds: several windows run concurrently, each on its stage's compute stream.
constexpr size_t kStreamStages = 6;
constexpr size_t kStreamWindowMsgs = 65536;                 // messages per window, at most
constexpr unsigned kStageThreads = 4;                       // host threads gathering a window

// Copy n items with f(i) on up to kStageThreads threads (contiguous index ranges).
template <class F>
void parallel_ranges(size_t n, size_t bytes, F&& f) {
    const unsigned t = bytes >= ((size_t)8 << 20) ? kStageThreads : 1;
    if (t == 1 || n < 2 * t) {
        f((size_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned k = 1; k < t; ++k) th.emplace_back([&, k] { f(n * k / t, n * (k + 1) / t); });
    f((size_t)0, n / t);
    for (auto& x : th) x.join();
}

struct StreamArgs {
    const uint8_t* blob;
    size_t blob_len;
    const uint64_t* off;
    const uint32_t* len;
    const uint8_t *r, *s, *qx, *qy;
    uint8_t* ok_out;
    uint8_t* dig_out;
    size_t window_bytes;
    bool blob_pinned;
};

// One device's share [c.begin, c.begin + c.count), streamed in windows through the slot's K
// stage buffers (kStreamStages). Window w (stage b = w mod K):
//   host    : wait for window w-K's outputs on stage b (out_done), hand them to the caller;
//             write window w's rebased offsets, lengths and tuple fields into the pinned
//             input of stage b; the messages are DMA'd straight from the caller's blob when
//             the window's span is dense (from pageable memory the runtime stages the copy
//             and this thread waits for it), else gathered into the stage first
//   copy    : H2D of the stage -> device buffer b; record h2d_done
//   compute : on the stage's own stream: wait h2d_done; SHA-256 -> verify (digests stay on
//             the device) -> D2H of the verdicts (+ digests) into the stage's pinned output;
//             record out_done
// so up to K windows hash and verify concurrently while the copy stream moves the next.
int stream_chunk(sbft_gv_ctx* ctx, const Chunk& c, const StreamArgs& a) {
    Slot* sl = c.slot;
    HIPCHK(hipSetDevice(sl->device));
    int rc = sl->reserve_pipe(0);  // the copy stream
    if (rc) return rc;
    const void* gcomb = sl->gcomb_table();
    if (!gcomb) return SBFT_GV_ENOMEM;
    // window boundaries (message index ranges)
    std::vector<size_t> cut{c.begin};
    {
        size_t bytes = 0, msgs = 0;
        for (size_t k = c.begin; k < c.begin + c.count; ++k) {
            if (a.off[k] + a.len[k] > a.blob_len || a.off[k] + a.len[k] < a.off[k]) return SBFT_GV_EINVAL;
            if (msgs && (bytes + a.len[k] > a.window_bytes || msgs == kStreamWindowMsgs)) {
                cut.push_back(k);
                bytes = msgs = 0;
            }
            bytes += a.len[k];
            ++msgs;
        }
        cut.push_back(c.begin + c.count);
    }
    const size_t W = cut.size() - 1;
    // per window: payload bytes, span [lo, hi) in the caller's blob, and whether the span is
    // DMA'd in place (page-locked blob, messages laid out densely) or gathered on the host
    std::vector<uint64_t> lo(W, UINT64_MAX), hi(W, 0), bytes(W, 0);
    std::vector<uint8_t> direct(W);
    size_t m = 0, dev_blob = 0, pin_blob = 0;
    for (size_t w = 0; w < W; ++w) {
        for (size_t k = cut[w]; k < cut[w + 1]; ++k) {
            lo[w] = std::min(lo[w], a.off[k]);
            hi[w] = std::max(hi[w], a.off[k] + a.len[k]);
            bytes[w] += a.len[k];
        }
        const uint64_t span = hi[w] - lo[w];
        // dense: DMA'd in place (from pageable memory through the runtime's own staging,
        // which runs at the PCIe rate; a host gather into our staging is the fallback for
        // windows whose messages are scattered over the blob)
        direct[w] = span <= bytes[w] + bytes[w] / 8 + 4096;
        m = std::max(m, cut[w + 1] - cut[w]);
        dev_blob = std::max<size_t>(dev_blob, direct[w] ? span : bytes[w]);
        if (!direct[w]) pin_blob = std::max<size_t>(pin_blob, bytes[w]);
    }
    // stage layouts (256-B aligned regions; m = the largest window's message count):
    //   pinned in : blob gather area (pb) | off (8 m) | len (4 m) | r | s | qx | qy (32 m each)
    //   device    : blob (fb)             | off | len | r | s | qx | qy | hash counter (256) |
    //               digests (32 m) | ok (m) | verify workspace
    //   pinned out: ok (m) | digests (32 m)
    // The hash kernel reads up to SBFT_GV_SHA_BLOB_PAD B past a message: the device blob region has that spare.
    const size_t fb = align_up(dev_blob + SBFT_GV_SHA_BLOB_PAD, 256), pb = pin_blob ? align_up(pin_blob, 256) : 0;
    const size_t fo = align_up(8 * m, 256), fl = align_up(4 * m, 256), fd = align_up(32 * m, 256),
                 fk = align_up(m, 256);
    const size_t meta = fo + fl + 4 * fd;
    const size_t dev_bytes = fb + meta + 256 + fd + fk + align_up(sbft_verify_work_bytes(m), 256);
    const size_t K = std::min(kStreamStages, W);
    for (size_t b = 0; b < K; ++b)
        if ((rc = sl->reserve_stage(b, dev_bytes, pb + meta, fk + fd))) return rc;
    auto collect = [&](size_t w) -> int {  // outputs of window w (stage w % K) -> caller
        Slot::StreamStage& st = sl->stage[w % K];
        // poll: a blocking event wait can sleep past the event by a scheduler tick or more,
        // once per window
        hipError_t q;
        while ((q = hipEventQuery(st.out_done)) == hipErrorNotReady) std::this_thread::yield();
        if (q != hipSuccess) return SBFT_GV_EDEVICE;
        const size_t b = cut[w], mw = cut[w + 1] - b;
        std::memcpy(a.ok_out + b, st.pin_out, mw);
        if (a.dig_out) std::memcpy(a.dig_out + 32 * b, st.pin_out + fk, 32 * mw);
        return SBFT_GV_OK;
    };
    static const bool trace = getenv("SBFT_STREAM_TRACE") != nullptr;  // diagnostics
    const auto t_start = std::chrono::steady_clock::now();
    auto us = [&] {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_start).count();
    };
    for (size_t w = 0; w < W; ++w) {
        Slot::StreamStage& st = sl->stage[w % K];
        const double t0 = trace ? us() : 0;
        if (w >= K && (rc = collect(w - K))) return rc;
        const double t1 = trace ? us() : 0;
        const size_t b = cut[w], mw = cut[w + 1] - b;
        uint8_t* in = st.pin_in;
        uint64_t* off_h = (uint64_t*)(in + pb);
        uint32_t* len_h = (uint32_t*)(in + pb + fo);
        uint8_t* tup = in + pb + fo + fl;
        if (direct[w]) {
            for (size_t k = 0; k < mw; ++k) off_h[k] = a.off[b + k] - lo[w];
        } else {
            uint64_t at = 0;
            for (size_t k = 0; k < mw; ++k) {
                off_h[k] = at;
                at += a.len[b + k];
            }
            parallel_ranges(mw, bytes[w], [&](size_t k0, size_t k1) {
                for (size_t k = k0; k < k1; ++k)
                    if (a.len[b + k]) std::memcpy(in + off_h[k], a.blob + a.off[b + k], a.len[b + k]);
            });
        }
        std::memcpy(len_h, a.len + b, 4 * mw);
        const uint8_t* src4[4] = {a.r, a.s, a.qx, a.qy};
        for (int f = 0; f < 4; ++f) std::memcpy(tup + f * fd, src4[f] + 32 * b, 32 * mw);
        uint8_t* d = st.dev;
        if (direct[w])
            HIPCHK(hipMemcpyAsync(d, a.blob + lo[w], hi[w] - lo[w], hipMemcpyHostToDevice, sl->copy_stream));
        else if (bytes[w])
            HIPCHK(hipMemcpyAsync(d, in, bytes[w], hipMemcpyHostToDevice, sl->copy_stream));
        HIPCHK(hipMemcpyAsync(d + fb, in + pb, meta, hipMemcpyHostToDevice, sl->copy_stream));
        HIPCHK(hipEventRecord(st.h2d_done, sl->copy_stream));
        HIPCHK(hipStreamWaitEvent(st.cs, st.h2d_done, 0));
        uint8_t* d_tup = d + fb + fo + fl;
        uint8_t* d_ctr = d + fb + meta;
        uint8_t* d_dig = d_ctr + 256;
        uint8_t* d_ok = d_dig + fd;
        uint32_t* work = (uint32_t*)(d_ok + fk);
        if (sbft_launch_sha256(d, (const uint64_t*)(d + fb), (const uint32_t*)(d + fb + fo), nullptr, d_dig,
                               (uint32_t)mw, (uint32_t*)d_ctr, st.cs) ||
            sbft_launch_p256_verify(d_dig, d_tup, d_tup + fd, d_tup + 2 * fd, d_tup + 3 * fd, d_ok, (uint32_t)mw,
                                    work, gcomb, st.cs, nullptr, nullptr, ctx->lanes_for(mw)))
            return SBFT_GV_ELAUNCH;
        HIPCHK(hipMemcpyAsync(st.pin_out, d_ok, mw, hipMemcpyDeviceToHost, st.cs));
        if (a.dig_out) HIPCHK(hipMemcpyAsync(st.pin_out + fk, d_dig, 32 * mw, hipMemcpyDeviceToHost, st.cs));
        HIPCHK(hipEventRecord(st.out_done, st.cs));
        if (trace)
            fprintf(stderr, "stream dev %d window %zu: msgs %zu bytes %llu direct %d | collect %.0f us, stage+enqueue %.0f us\n",
                    sl->device, w, mw, (unsigned long long)bytes[w], (int)direct[w], t1 - t0, us() - t1);
    }
    for (size_t w = W >= K ? W - K : 0; w < W; ++w)
        if ((rc = collect(w))) return rc;
    return SBFT_GV_OK;
}

}  // namespace

extern "C" int sbft_gv_sha256_verify_p256_stream(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len,
                                                 const uint64_t* off, const uint32_t* len, const uint8_t* r,
                                                 const uint8_t* s, const uint8_t* qx, const uint8_t* qy, size_t n,
                                                 size_t window_bytes, uint8_t* ok_out, uint8_t* dig_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if ((!blob && blob_len) || !off || !len || !r || !s || !qx || !qy || !ok_out || n > 0xffffffffu)
        return SBFT_GV_EINVAL;
    StreamArgs a{blob, blob_len, off, len, r, s, qx, qy, ok_out, dig_out,
                 window_bytes ? window_bytes : kStreamWindowDefault, blob && is_pinned(blob)};
    // a message longer than the window gets a window of its own
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) {
        const int rc = stream_chunk(ctx, c, a);
        if (rc) {  // drain the copy and stage streams too (run_chunks waits on the main stream only)
            (void)hipStreamSynchronize(c.slot->copy_stream);
            for (auto& st : c.slot->stage)
                if (st.cs) (void)hipStreamSynchronize(st.cs);
        }
        return rc;
    });
}

// ---------------------------------------------------------------- registered keys
namespace {

// Build the comb tables of keys [sl->comb.size(), upto) on sl's device in one launch (one
// allocation for the batch) and refresh its device pointer array. Caller holds sl->mu.
// status_out (optional) receives one validity byte per built key.
int build_tables(Slot* sl, const std::vector<std::array<uint8_t, 64>>& keys, size_t upto,
                 std::vector<uint8_t>* status_out) {
    HIPCHK(hipSetDevice(sl->device));
    const size_t have = sl->comb.size();
    if (status_out) status_out->clear();
    if (have >= upto) return SBFT_GV_OK;
    const size_t nk = upto - have, tb = sbft_comb_table_bytes();
    void* block = nullptr;
    if (hipMalloc(&block, nk * tb) != hipSuccess) return SBFT_GV_ENOMEM;
    uint8_t* tmp = nullptr;  // qx[nk] | qy[nk] | status[nk]
    if (hipMalloc(&tmp, nk * 68) != hipSuccess) {
        (void)hipFree(block);
        return SBFT_GV_ENOMEM;
    }
    std::vector<uint8_t> h(nk * 64);
    for (size_t i = 0; i < nk; ++i) {
        std::memcpy(&h[32 * i], keys[have + i].data(), 32);
        std::memcpy(&h[32 * (nk + i)], keys[have + i].data() + 32, 32);
    }
    std::vector<uint32_t> st(nk);
    int rc = SBFT_GV_OK;
    if (hipMemcpyAsync(tmp, h.data(), nk * 64, hipMemcpyHostToDevice, sl->stream) != hipSuccess ||
        sbft_launch_comb_build(tmp, tmp + 32 * nk, block, (uint32_t*)(tmp + 64 * nk), (uint32_t)nk, sl->stream) ||
        hipMemcpyAsync(st.data(), tmp + 64 * nk, 4 * nk, hipMemcpyDeviceToHost, sl->stream) != hipSuccess ||
        hipStreamSynchronize(sl->stream) != hipSuccess)
        rc = SBFT_GV_EDEVICE;
    (void)hipFree(tmp);
    if (rc) {
        (void)hipFree(block);
        return rc;
    }
    sl->comb_alloc.push_back(block);
    for (size_t i = 0; i < nk; ++i)
        sl->comb.push_back(st[i] == 1 ? (void*)((uint8_t*)block + i * tb) : nullptr);
    if (status_out)
        for (uint32_t v : st) status_out->push_back(v == 1 ? 1 : 0);
    if (sl->keytab_cap < sl->comb.size()) {
        if (sl->d_keytab) sl->retired.push_back(sl->d_keytab);
        sl->d_keytab = nullptr;
        const size_t cap = std::max<size_t>(64, 2 * sl->comb.size());
        HIPCHK(hipMalloc((void**)&sl->d_keytab, cap * sizeof(void*)));
        sl->keytab_cap = cap;
    }
    HIPCHK(hipMemcpyAsync(sl->d_keytab, sl->comb.data(), sl->comb.size() * sizeof(void*), hipMemcpyHostToDevice,
                          sl->stream));
    HIPCHK(stream_sync(sl->stream));
    return SBFT_GV_OK;
}

// Small-batch keyed verify on one device. Staging layout (all 256-B aligned):
// r | s | key | (digest | blob+pad, off, len) | ok. Messages (blob != null) are hashed in the
// launch; otherwise digest holds 32-byte digests.
//   zc = false: pinned staging, one H2D, one launch, one D2H (the caller synchronises the stream).
//   zc = true: the staging is the slot's mapped coherent buffer; the kernel reads it and writes
//     each verdict | 2 straight into it, and this call returns once every verdict byte has
//     landed: no copies and no stream synchronisation on the latency path (~20 us of a ~70 us
//     commit-quorum call). A fault is caught by polling the stream now and then.
int enqueue_keyed(Chunk& c, const uint8_t* digest, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                  const uint32_t* len, const uint8_t* r, const uint8_t* s, const uint32_t* key, uint32_t nkeys,
                  void** keytab, Slot::ZcLane* zl, uint8_t* ok_out, size_t lanes_min, size_t host_sinv_max,
                  sbft_gv_ctx* tctx = nullptr) {
    Slot* sl = c.slot;
    const bool zc = zl != nullptr;
    hipStream_t st = zc ? zl->stream : sl->stream;  // (the lane's stream is created by its reserve)
    const size_t n = c.count, b = c.begin;
    static const bool trace = getenv("SBFT_KEYED_TRACE") != nullptr;  // diagnostics
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t lo = UINT64_MAX, hi = 0;
    if (blob) {
        for (size_t k = b; k < b + n; ++k) {
            if (off[k] + len[k] > blob_len) return SBFT_GV_EINVAL;
            lo = std::min(lo, off[k]);
            hi = std::max(hi, off[k] + len[k]);
        }
        if (n == 0 || hi < lo) lo = hi = 0;
    }
    const size_t span = blob ? hi - lo : 0;
    const size_t f32 = align_up(32 * n, 256), fk = align_up(4 * n, 256);
    const size_t fblob = align_up(span + SBFT_GV_SHA_BLOB_PAD, 256);  // + the hash kernel's over-read
    const size_t fmsg = blob ? fblob + align_up(8 * n, 256) + fk : f32;
    const size_t fok = align_up(n, 256);
    // large batches: the four-lane kernel, with digests from the hash kernel (counter | digests)
    const bool lanes = !zc && lanes_min && n >= lanes_min;
    // s^-1 from the host (modn::sinv_batch_mont) for small wavefront-kernel batches: | w after the messages
    const bool host_sinv = !lanes && n > 0 && n <= host_sinv_max;
    const size_t fw = host_sinv ? f32 : 0;
    const size_t in_bytes = 2 * f32 + fk + fmsg + fw;
    const size_t fextra = lanes ? 256 + f32 : 0;
    HIPCHK(hipSetDevice(sl->device));
    int rc;
    uint8_t *h, *d;
    if (zc) {
        rc = zl->reserve(in_bytes + fok);
        if (rc) return rc;
        st = zl->stream;
        h = zl->host;
        d = zl->dev;
    } else {
        rc = sl->reserve(in_bytes + fok + fextra);
        if (rc) return rc;
        rc = sl->reserve_pinned(in_bytes + fok);
        if (rc) return rc;
        h = sl->pin;
        d = sl->dbuf;
    }
    std::memcpy(h, r + 32 * b, 32 * n);
    std::memcpy(h + f32, s + 32 * b, 32 * n);
    std::memcpy(h + 2 * f32, key + b, 4 * n);
    uint8_t* m = h + 2 * f32 + fk;
    if (blob) {
        std::memcpy(m, blob + lo, span);
        std::memset(m + span, 0, fblob - span);
        uint64_t* o = (uint64_t*)(m + fblob);
        for (size_t k = 0; k < n; ++k) o[k] = off[b + k] - lo;
        std::memcpy((uint8_t*)o + align_up(8 * n, 256), len + b, 4 * n);
    } else {
        std::memcpy(m, digest + 32 * b, 32 * n);
    }
    if (host_sinv) sbft::modn::sinv_batch_mont(s + 32 * b, n, (uint32_t*)(h + 2 * f32 + fk + fmsg));
    volatile uint8_t* okh = h + in_bytes;
    if (zc) {
        std::memset((void*)okh, 0, n);
        std::atomic_thread_fence(std::memory_order_seq_cst);
    } else {
        HIPCHK(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st));
    }
    const uint8_t* dm = d + 2 * f32 + fk;
    const uint8_t* d_blob = blob ? dm : nullptr;
    const uint64_t* d_off = blob ? (const uint64_t*)(dm + fblob) : nullptr;
    const uint32_t* d_len = blob ? (const uint32_t*)((const uint8_t*)d_off + align_up(8 * n, 256)) : nullptr;
    uint8_t* d_ok = d + in_bytes;
    const auto t1 = std::chrono::steady_clock::now();
    LaunchTimer kt(tctx, st);  // sbft_gv_kernel_timing: the keyed kernel (and its hash kernel, if any)
    if (lanes) {
        uint8_t* x = d + in_bytes + fok;  // hash counter | digests
        const uint8_t* dig = dm;
        if (blob) {
            if (sbft_launch_sha256(d_blob, d_off, d_len, nullptr, x + 256, (uint32_t)n, (uint32_t*)x, st))
                return SBFT_GV_ELAUNCH;
            dig = x + 256;
        }
        if (sbft_launch_p256_verify_keyed_lanes(dig, d, d + f32, (const uint32_t*)(d + 2 * f32),
                                                (const void* const*)keytab, nkeys, d_ok, (uint32_t)n,
                                                st))
            return SBFT_GV_ELAUNCH;
    } else if (sbft_launch_p256_verify_keyed(blob ? nullptr : dm, d_blob, d_off, d_len, d, d + f32,
                                             (const uint32_t*)(d + 2 * f32), (const void* const*)keytab, nkeys,
                                             d_ok, (uint32_t)n, zc ? 2 : 0,
                                             host_sinv ? (const uint32_t*)(d + 2 * f32 + fk + fmsg) : nullptr, st)) {
        return SBFT_GV_ELAUNCH;
    }
    kt.end();
    if (!zc) {
        HIPCHK(hipMemcpyAsync(h + in_bytes, d_ok, n, hipMemcpyDeviceToHost, st));
        c.out_off = in_bytes;
        return SBFT_GV_OK;
    }
    if (hipEventRecord(zl->done, st) != hipSuccess) {
        (void)hipStreamSynchronize(st);  // the kernel still writes into the lane's buffer: drain it
        return SBFT_GV_EDEVICE;
    }
    const auto t2 = std::chrono::steady_clock::now();
    auto t3 = t2;
    size_t seen = 0;
    // Spin on the verdict bytes for at most the spin budget (the keyed kernel of a quorum takes
    // ~45 us, so a healthy call never leaves the spin), then sleep on the blocking event: a caller
    // stuck behind other work, or a core-starved host, stops burning the job's CPU quota
    // (VERDICT r04 #3). SBFT_ZC_SPIN_US overrides the budget (0 = block at once).
    static const long spin_us = [] {
        const char* e = getenv("SBFT_ZC_SPIN_US");
        return e ? std::max(0L, std::atol(e)) : 120L;
    }();
    const auto spin_end = t2 + std::chrono::microseconds(spin_us);
    for (uint32_t spin = 1; seen < n; ++spin) {
        if (okh[seen]) {
            if (seen == 0) t3 = std::chrono::steady_clock::now();
            ++seen;
            continue;
        }
        cpu_relax();
        if ((spin & 63u) == 0 && std::chrono::steady_clock::now() >= spin_end) {
            // the budget is spent: wait for the kernel asleep; it has then written every verdict
            // it will, so any byte still zero is a launch that failed or ended short
            if (hipEventSynchronize(zl->done) != hipSuccess) return SBFT_GV_EDEVICE;
            std::atomic_thread_fence(std::memory_order_seq_cst);
            for (; seen < n && okh[seen]; ++seen) {
            }
            if (seen < n) return SBFT_GV_EDEVICE;
            if (seen && t3 == t2) t3 = std::chrono::steady_clock::now();
            break;
        }
    }
    if (sbft_fault_hit(SBFT_GV_FAULT_SYNC)) return SBFT_GV_EDEVICE;  // the kernel has finished
    for (size_t k = 0; k < n; ++k) ok_out[b + k] = okh[k] & 1u;
    if (trace) {
        const auto t4 = std::chrono::steady_clock::now();
        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
            return std::chrono::duration<double, std::micro>(z - a).count();
        };
        fprintf(stderr, "keyed_zc n=%zu stage=%.1f launch=%.1f first=%.1f all=%.1f us\n", n, us(t0, t1), us(t1, t2),
                us(t2, t3), us(t3, t4));
    }
    return SBFT_GV_OK;
}

// Tables of keys [0, upto) on sl's device, upto <= the published key count. A registration
// builds its keys on every device before publishing them, so the only table a device can lack
// here is G's (key 0, built on first use). No key snapshot, no keys_mu (registration takes
// keys_mu before a slot's mu; this runs under sl->mu). Caller holds sl->mu.
int ensure_tables(Slot* sl, size_t upto) {
    if (sl->comb.size() >= upto) return SBFT_GV_OK;
    if (sl->comb.empty()) {
        const std::vector<std::array<uint8_t, 64>> g(1, kGXY);
        const int rc = build_tables(sl, g, 1, nullptr);
        if (rc) return rc;
    }
    return sl->comb.size() >= upto ? SBFT_GV_OK : SBFT_GV_EDEVICE;
}

int run_keyed(sbft_gv_ctx* ctx, const uint8_t* digest, const uint8_t* blob, size_t blob_len, const uint64_t* off,
              const uint32_t* len, const uint8_t* r, const uint8_t* s, const uint32_t* key, size_t n,
              uint8_t* ok_out) {
    const uint32_t nkeys = (uint32_t)ctx->nkeys.load();  // published keys
    std::vector<Chunk> chunks = plan(ctx, n);
    return for_each_device(ctx, chunks.size(), [&](size_t i) {
        Chunk& c = chunks[i];
        if (c.count <= ctx->keyed_zc_max) {
            // zero-copy: the slot lock only for the tables, then a lane of its own
            void** keytab;
            {
                std::lock_guard<std::mutex> lk(c.slot->mu);
                const int rc = ensure_tables(c.slot, nkeys);
                if (rc) return rc;
                keytab = c.slot->d_keytab;  // entries [0, nkeys) never change; old arrays are retired
            }
            std::unique_lock<std::mutex> zlk;
            Slot::ZcLane& zl = c.slot->acquire_zc(zlk);
            return enqueue_keyed(c, digest, blob, blob_len, off, len, r, s, key, nkeys, keytab, &zl, ok_out, 0,
                                 ctx->keyed_host_sinv_max, ctx);
        }
        std::lock_guard<std::mutex> lk(c.slot->mu);
        int rc = ensure_tables(c.slot, nkeys);
        if (rc == SBFT_GV_OK)
            rc = enqueue_keyed(c, digest, blob, blob_len, off, len, r, s, key, nkeys, c.slot->d_keytab, nullptr,
                               ok_out, ctx->keyed_lanes_min, ctx->keyed_host_sinv_max, ctx);
        (void)hipSetDevice(c.slot->device);
        if (stream_sync(c.slot->stream) != hipSuccess && rc == SBFT_GV_OK) rc = SBFT_GV_EDEVICE;
        // the verdicts sit in the slot's pinned staging, which the lock still protects
        if (rc == SBFT_GV_OK) std::memcpy(ok_out + c.begin, c.slot->pin + c.out_off, c.count);
        return rc;
    });
}

// Small signing batches on one device: one H2D of d | k | digest through pinned staging, the
// wave kernel over G's comb table (slot 0, built on first use), one D2H of qx | qy | r | s | status.
int sign_wave(sbft_gv_ctx* ctx, const uint8_t* d, const uint8_t* k, const uint8_t* digest, size_t n, uint8_t* qx,
              uint8_t* qy, uint8_t* r, uint8_t* s, uint8_t* status) {
    std::vector<Chunk> chunks = plan(ctx, n);  // n < min_split: one device
    Slot* sl = chunks[0].slot;
    std::lock_guard<std::mutex> lk(sl->mu);
    int rc = ensure_tables(sl, 1);  // G's table
    if (rc) return rc;
    const size_t f = align_up(32 * n, 256), fs = align_up(n, 256);
    const size_t in_bytes = 3 * f, out_bytes = 4 * f + fs;
    HIPCHK(hipSetDevice(sl->device));
    rc = sl->reserve(in_bytes + out_bytes);
    if (rc) return rc;
    rc = sl->reserve_pinned(in_bytes + out_bytes);
    if (rc) return rc;
    uint8_t* h = sl->pin;
    std::memcpy(h, d, 32 * n);
    std::memcpy(h + f, k, 32 * n);
    std::memcpy(h + 2 * f, digest, 32 * n);
    uint8_t* b = sl->dbuf;
    HIPCHK(hipMemcpyAsync(b, h, in_bytes, hipMemcpyHostToDevice, sl->stream));
    uint8_t* o = b + in_bytes;
    const bool want_q = qx != nullptr;
    if (sbft_launch_p256_sign_wave(b, b + f, b + 2 * f, (const void* const*)sl->d_keytab, want_q ? o : nullptr,
                                   want_q ? o + f : nullptr, o + 2 * f, o + 3 * f, o + 4 * f, (uint32_t)n, sl->stream))
        return SBFT_GV_ELAUNCH;
    HIPCHK(hipMemcpyAsync(h + in_bytes, o, out_bytes, hipMemcpyDeviceToHost, sl->stream));
    HIPCHK(stream_sync(sl->stream));
    const uint8_t* ho = h + in_bytes;
    if (want_q) {
        std::memcpy(qx, ho, 32 * n);
        std::memcpy(qy, ho + f, 32 * n);
    }
    std::memcpy(r, ho + 2 * f, 32 * n);
    std::memcpy(s, ho + 3 * f, 32 * n);
    std::memcpy(status, ho + 4 * f, n);
    return SBFT_GV_OK;
}

// New client keys whose tables still fit (caller holds keys_mu): the client budget per device
// (ctx->client_cap, default 1/8 of the device's memory) and, on every device, the memory above
// the staging reserve. A device with k slots pays k tables per key.
// Client keys that still fit every device's budget, or SBFT_GV_EDEVICE in *rc when a device's
// memory cannot be queried (an engine failure, never reported as a spent budget). The calling
// thread's current device is restored.
size_t client_key_room(sbft_gv_ctx* ctx, int* rc) {
    *rc = SBFT_GV_OK;
    const size_t tb = sbft_comb_table_bytes();
    std::map<int, size_t> spd;
    for (Slot* sl : ctx->slots) ++spd[sl->device];
    size_t room = SIZE_MAX;
    int prev = -1;
    const bool have_prev = hipGetDevice(&prev) == hipSuccess;
    struct Restore {
        bool on;
        int dev;
        ~Restore() {
            if (on) (void)hipSetDevice(dev);
        }
    } restore{have_prev, prev};
    for (const auto& [dev, k] : spd) {
        size_t free_b = 0, total = 0;
        if (hipSetDevice(dev) != hipSuccess || hipMemGetInfo(&free_b, &total) != hipSuccess) {
            *rc = SBFT_GV_EDEVICE;
            return 0;
        }
        const uint64_t cap = ctx->client_cap ? ctx->client_cap : total / 8;
        const uint64_t used = (uint64_t)ctx->client_keys * tb * k;
        const size_t by_cap = used >= cap ? 0 : (size_t)((cap - used) / (tb * k));
        const uint64_t reserve = std::max<uint64_t>(SBFT_GV_HBM_RESERVE, total / 32);
        const size_t by_free = free_b <= reserve ? 0 : (size_t)((free_b - reserve) / (tb * k));
        room = std::min(room, std::min(by_cap, by_free));
    }
    return room;
}

// sbft_gv_register_keys with at most max_new keys added (the rest: id 0, not added)
int register_keys(sbft_gv_ctx* ctx, const uint8_t* qx, const uint8_t* qy, size_t n, uint32_t* key_ids,
                  bool client, size_t* registered) {
    if (!ctx || (n && (!qx || !qy || !key_ids)) || n > 0xffffffu) return SBFT_GV_EINVAL;
    std::lock_guard<std::mutex> g(ctx->keys_mu);
    const size_t before = ctx->keys.size();
    int room_rc = SBFT_GV_OK;
    const size_t max_new = client ? client_key_room(ctx, &room_rc) : SIZE_MAX;
    if (room_rc) return room_rc;
    std::vector<size_t> pending;  // positions i whose key is new in this call
    std::vector<uint8_t> held(n, 1);  // 0: past the budget (id 0)
    for (size_t i = 0; i < n; ++i) {
        std::array<uint8_t, 64> k;
        std::memcpy(k.data(), qx + 32 * i, 32);
        std::memcpy(k.data() + 32, qy + 32 * i, 32);
        auto it = ctx->key_index.find(k);
        if (it != ctx->key_index.end()) {
            key_ids[i] = it->second;  // resolved below for keys added by this call
            continue;
        }
        if (pending.size() >= max_new) {
            key_ids[i] = 0;
            held[i] = 0;
            continue;
        }
        const uint32_t id = (uint32_t)ctx->keys.size();
        ctx->key_index.emplace(k, id);
        ctx->keys.push_back(k);
        ctx->key_valid.push_back(0);
        key_ids[i] = id;
        pending.push_back(i);
    }
    const size_t upto = ctx->keys.size();
    int rc = SBFT_GV_OK;
    std::vector<uint8_t> st;
    for (size_t si = 0; si < ctx->slots.size() && rc == SBFT_GV_OK; ++si) {
        Slot* sl = ctx->slots[si];
        std::lock_guard<std::mutex> lk(sl->mu);
        std::vector<uint8_t> sst;
        // G's table first, in a block of its own: concurrent zero-copy batches may already read it
        // (run_keyed needs only key 0 to be built), so the rollback below must never free it
        rc = ensure_tables(sl, 1);
        if (rc == SBFT_GV_OK) rc = build_tables(sl, ctx->keys, upto, &sst);
        // a device that had not built G's table yet built [0, upto): keep this call's tail
        if (rc == SBFT_GV_OK && sl->comb.size() == upto && sst.size() >= upto - before)
            st.assign(sst.end() - (upto - before), sst.end());
    }
    if (rc == SBFT_GV_OK && st.size() != upto - before && upto > before) rc = SBFT_GV_EDEVICE;
    if (rc) {
        // forget this call's keys everywhere. Their tables share one block per slot, which holds
        // nothing else (G's table was built apart, above), and no other call can reach them: key
        // ids >= before are published only on success (ctx->nkeys), so the zero-copy lanes, which
        // run outside sl->mu, never read this block.
        for (Slot* sl : ctx->slots) {
            std::lock_guard<std::mutex> lk(sl->mu);
            if (sl->comb.size() > before && before >= 1) {
                (void)hipSetDevice(sl->device);
                (void)hipStreamSynchronize(sl->stream);  // the build kernel ran on the slot's stream
                (void)hipFree(sl->comb_alloc.back());
                sl->comb_alloc.pop_back();
                sl->comb.resize(before);
            }
        }
        for (size_t id = before; id < upto; ++id) ctx->key_index.erase(ctx->keys[id]);
        ctx->keys.resize(before);
        ctx->key_valid.resize(before);
        return rc;
    }
    for (size_t id = before; id < upto; ++id) ctx->key_valid[id] = st[id - before];
    ctx->nkeys = (uint32_t)upto;
    if (client) ctx->client_keys += upto - before;
    size_t got = 0;
    for (size_t i = 0; i < n; ++i) {
        if (held[i] && !ctx->key_valid[key_ids[i]]) key_ids[i] = 0;
        got += key_ids[i] != 0;
    }
    if (registered) *registered = got;
    return SBFT_GV_OK;
}

}  // namespace

extern "C" {

int sbft_gv_register_keys(sbft_gv_ctx* ctx, const uint8_t* qx, const uint8_t* qy, size_t n, uint32_t* key_ids) {
    return register_keys(ctx, qx, qy, n, key_ids, false, nullptr);
}

int sbft_gv_register_client_keys(sbft_gv_ctx* ctx, const uint8_t* qx, const uint8_t* qy, size_t n,
                                 uint32_t* key_ids, size_t* registered) {
    return register_keys(ctx, qx, qy, n, key_ids, true, registered);
}

int sbft_gv_register_key(sbft_gv_ctx* ctx, const uint8_t qx[32], const uint8_t qy[32], uint32_t* key_id) {
    if (!ctx || !qx || !qy || !key_id) return SBFT_GV_EINVAL;
    const int rc = sbft_gv_register_keys(ctx, qx, qy, 1, key_id);
    if (rc) return rc;
    return *key_id ? SBFT_GV_OK : SBFT_GV_EINVAL;
}

int sbft_gv_verify_p256_keyed(sbft_gv_ctx* ctx, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                              const uint32_t* key_id, size_t n, uint8_t* ok_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!digest || !r || !s || !key_id || !ok_out || n > 0xffffffffu) return SBFT_GV_EINVAL;
    return run_keyed(ctx, digest, nullptr, 0, nullptr, nullptr, r, s, key_id, n, ok_out);
}

int sbft_gv_sha256_verify_p256_keyed(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                                     const uint32_t* len, const uint8_t* r, const uint8_t* s, const uint32_t* key_id,
                                     size_t n, uint8_t* ok_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if ((!blob && blob_len) || !off || !len || !r || !s || !key_id || !ok_out || n > 0xffffffffu)
        return SBFT_GV_EINVAL;
    static const uint8_t empty = 0;
    return run_keyed(ctx, nullptr, blob ? blob : &empty, blob_len, off, len, r, s, key_id, n, ok_out);
}

}  // extern "C"
