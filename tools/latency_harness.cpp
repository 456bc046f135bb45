// latency_harness.cpp — per-call latency of BASELINE configs 3 and 4 as the library drives them,
// on the GPU path (through the C ABI of libsbft_gpuverify.so) and on a CPU baseline (OpenSSL
// libcrypto ECDSA_do_verify; Go is absent on both machines, so OpenSSL's ecp_nistz256 assembly
// is the stand-in for Go's crypto/ecdsa). Measurement tooling for bench.py, not product code.
//
//   quorum-gpu  CALLERS DECISIONS COALESCE_MAX COALESCE_WAIT_US
//       view.go:537-541: one goroutine per commit vote, each calling VerifyConsenterSig
//       (:834). CALLERS threads of a persistent pool are released at once per decision; each
//       makes ONE sbft_verifier_verify_consenter_sig call on its own vote. Latency = release ->
//       the last call returned. COALESCE_MAX <= 1 is the stock behaviour (a launch per call).
//       Every 10th decision carries one bad signature (vote 7): its caller must get
//       SBFT_V_EVERIFY with the reference's text, everyone else 0.
//   quorum-batch VOTES DECISIONS
//       the batch hook: one sbft_verifier_verify_consenter_sigs call per decision.
//   quorum-hook VOTERS NEED DECISIONS INFLIGHT
//       the processCommits batch hook with arriving votes (go/patches/internal_bft_commits.patch),
//       at most INFLIGHT (default 2) batch calls in flight.
//   quorum-pipe CHANNELS DECISIONS gpu|cpu|cpu-batched
//       pipelined decisions: CHANNELS consensus instances on one node, each deciding back to
//       back (prev-commit batch, then the commit votes), all in flight at once; cpu-batched is
//       the CPU plugin under the same patched call sequence as gpu (prev-commit batch over the cores).
//   sign CALLS
//       one signature at a time from one thread: sbft_signer_sign (RFC 6979, and with the
//       pre-signature pool of 1,024) vs OpenSSL ECDSA_do_sign.
//   quorum-cpu  CALLERS DECISIONS THREADS
//       the same fan-out with the verify on the CPU: CALLERS votes verified by THREADS
//       workers (one thread per vote when THREADS >= CALLERS), SHA-256(Msg) + ECDSA_do_verify
//       each, keys pre-materialised.
//   quorum-vote-cpu VOTERS NEED DECISIONS THREADS
//       quorum-hook's scenario on the CPU: VOTERS votes released per decision, each verified as
//       it arrives (one thread per vote, or a pool of THREADS), NEED valid ones close it; every
//       10th decision has a bad vote, as in quorum-hook.
//   proposal-cpu REQUESTS DECISIONS THREADS
//   proposal-gpu REQUESTS DECISIONS
//   proposal-phases REQUESTS CALLS REGISTERED   (where a VerifyProposal call's time goes)
//   parse-cpu    REQUESTS ITERS
//       VerifyProposal (view.go:555) on the CPU: REQUESTS signed requests (distinct keys,
//       64-256 B bodies) verified by THREADS workers pulling indices from an atomic counter:
//       SHA-256(body) + ECDSA_do_verify each, keys pre-materialised (favours the CPU: a real
//       plugin also decodes each request's key).
// Prints one JSON object.
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>
#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <dirent.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <climits>

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
#include <string>
#include <thread>
#include <vector>

#include "../include/sbft_verifier.h"

using Clock = std::chrono::steady_clock;
static int64_t now_ns() { return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count(); }

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    if (v.empty()) return 0;
    size_t i = (size_t)(p / 100.0 * (v.size() - 1) + 0.5);
    return v[std::min(i, v.size() - 1)];
}

// A pool of `n` threads released together once per round; run(i, round) is thread i's work.
// Returns per-round wall times (release -> last thread done), microseconds. Release and
// completion go through futexes and atomics, not a mutex: a mutex makes the n wake-ups (and
// the n completions) queue one behind another, which would add ~2-4 us per thread to every
// round (Go's goroutines, which this emulates, do not pay that). The release is a wake-up tree
// (the main thread wakes two, every woken thread two more): one FUTEX_WAKE of all n runs the n
// wake-ups serially inside one system call (~1-1.5 us each), slower than the Go runtime
// starting n goroutines on its GOMAXPROCS threads.
static long futex(std::atomic<int>* a, int op, int val) {
    return syscall(SYS_futex, reinterpret_cast<int*>(a), op, val, nullptr, nullptr, 0);
}
// A blocking wait with a bounded spin, as a Go select parks its goroutine: spin up to spin_us for
// ready(), then sleep on a futex that notify() (the producers: arriving votes, finished batches)
// bumps. No lost wake-up: the waiter reads ev, announces itself, re-checks ready(), and only then
// sleeps on ev's old value; a producer publishes its data, bumps ev, then wakes a sleeper.
struct Waker {
    std::atomic<int> ev{0}, sleeping{0};
    long spin_us = 20;
    void notify() {
        ev.fetch_add(1, std::memory_order_seq_cst);
        if (sleeping.load(std::memory_order_seq_cst)) futex(&ev, FUTEX_WAKE_PRIVATE, 1);
    }
    template <class Ready>
    void wait(Ready ready) {
        const auto t0 = Clock::now();
        while (!ready()) {
            if (Clock::now() - t0 < std::chrono::microseconds(spin_us)) {
                __builtin_ia32_pause();
                continue;
            }
            const int e = ev.load(std::memory_order_seq_cst);
            sleeping.store(1, std::memory_order_seq_cst);
            if (!ready()) futex(&ev, FUTEX_WAIT_PRIVATE, e);
            sleeping.store(0, std::memory_order_relaxed);
        }
    }
};
static long env_long(const char* name, long dflt) {
    const char* e = std::getenv(name);
    return e ? std::atol(e) : dflt;
}
// cores this job may use: the affinity mask, capped by the cgroup v2 CPU quota (as bench.py's
// host_cores: the GPU box gives a 16-CPU quota inside a 256-CPU mask)
static unsigned host_cores() {
    cpu_set_t set;
    unsigned n = sched_getaffinity(0, sizeof set, &set) == 0 ? (unsigned)CPU_COUNT(&set) : 1u;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long period = 0;
        if (std::fscanf(f, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
            n = std::min(n, (unsigned)std::max(1L, (std::atol(q) + period - 1) / period));
        std::fclose(f);
    }
    return std::max(1u, n);
}
// this thread's CPU time, nanoseconds
static int64_t thread_cpu_ns() {
    timespec ts{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}
// CPU time of this process's threads by name (/proc/self/task/*/stat utime + stime), ms: the
// harness names its threads (voter, collector, batch worker), the engine its own (sbft-*), the
// HIP runtime's keep theirs
struct ThreadCpu {
    std::map<long, std::pair<std::string, double>> by_tid;
    static ThreadCpu now() {
        ThreadCpu t;
        const double tick_ms = 1000.0 / (double)sysconf(_SC_CLK_TCK);
        DIR* d = opendir("/proc/self/task");
        if (!d) return t;
        while (dirent* e = readdir(d)) {
            if (e->d_name[0] == '.') continue;
            char path[300], buf[1024];
            std::snprintf(path, sizeof path, "/proc/self/task/%s/stat", e->d_name);
            FILE* f = std::fopen(path, "r");
            if (!f) continue;
            const size_t got = std::fread(buf, 1, sizeof buf - 1, f);
            std::fclose(f);
            buf[got] = 0;
            char* l = std::strchr(buf, '(');
            char* r = std::strrchr(buf, ')');
            if (!l || !r) continue;
            std::string comm(l + 1, r);
            // fields after ')': state(3) ... utime(14) stime(15)
            unsigned long ut = 0, st = 0;
            int field = 3;
            for (char* p = std::strtok(r + 2, " "); p; p = std::strtok(nullptr, " "), ++field) {
                if (field == 14) ut = std::strtoul(p, nullptr, 10);
                if (field == 15) {
                    st = std::strtoul(p, nullptr, 10);
                    break;
                }
            }
            t.by_tid[std::atol(e->d_name)] = {comm, (ut + st) * tick_ms};
        }
        closedir(d);
        return t;
    }
    // per-name CPU ms between `before` and this snapshot (threads started since count whole)
    std::map<std::string, double> since(const ThreadCpu& before) const {
        std::map<std::string, double> out;
        for (const auto& [tid, v] : by_tid) {
            auto it = before.by_tid.find(tid);
            out[v.first] += v.second - (it != before.by_tid.end() ? it->second.second : 0.0);
        }
        return out;
    }
};
static std::string cpu_json(const std::map<std::string, double>& m, double per) {
    std::string s = "{";
    for (const auto& [k, v] : m) {
        if (v <= 0) continue;
        char b[160];
        std::snprintf(b, sizeof b, "%s\"%s\": %.3f", s.size() > 1 ? ", " : "", k.c_str(), v / per);
        s += b;
    }
    return s + "}";
}

static std::vector<double> fan_out(size_t n, int rounds, const std::function<void(size_t, int)>& run) {
    std::atomic<int> gen{-1}, remaining{0}, done_gen{-1};
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            int seen = -1;
            for (;;) {
                int g;
                bool slept = false;
                while ((g = gen.load(std::memory_order_acquire)) == seen && !stop.load()) {
                    futex(&gen, FUTEX_WAIT_PRIVATE, seen);
                    slept = true;
                }
                if (slept) futex(&gen, FUTEX_WAKE_PRIVATE, 2);  // the release is a wake-up tree
                if (stop.load()) return;
                seen = g;
                run(i, g);
                if (remaining.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                    done_gen.store(g, std::memory_order_release);
                    futex(&done_gen, FUTEX_WAKE_PRIVATE, 1);
                }
            }
        });
    std::vector<double> out;
    for (int r = 0; r < rounds; ++r) {
        remaining.store((int)n);
        const auto t0 = Clock::now();
        gen.store(r, std::memory_order_release);
        futex(&gen, FUTEX_WAKE_PRIVATE, 2);
        int d;
        while ((d = done_gen.load(std::memory_order_acquire)) != r) futex(&done_gen, FUTEX_WAIT_PRIVATE, d);
        out.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    stop.store(true);
    gen.fetch_add(1);
    futex(&gen, FUTEX_WAKE_PRIVATE, INT_MAX);
    for (auto& t : th) t.join();
    return out;
}

// The job's cgroup CPU accounting (cgroup v2 cpu.stat; zeros where absent): a quota-limited
// job whose threads spin can be throttled for the rest of the quota period, which shows up as
// multi-millisecond outliers in the fan-out latencies.
struct CgroupCpu {
    long long usage_us = 0, nr_throttled = 0, throttled_us = 0;
};
static CgroupCpu cgroup_cpu() {
    CgroupCpu c;
    FILE* f = std::fopen("/sys/fs/cgroup/cpu.stat", "r");
    if (!f) return c;
    char key[64];
    long long val;
    while (std::fscanf(f, "%63s %lld", key, &val) == 2) {
        if (!std::strcmp(key, "usage_usec")) c.usage_us = val;
        else if (!std::strcmp(key, "nr_throttled")) c.nr_throttled = val;
        else if (!std::strcmp(key, "throttled_usec")) c.throttled_us = val;
    }
    std::fclose(f);
    return c;
}

// this process's CPU time (user + system), microseconds
static double proc_cpu_us() {
    rusage ru{};
    getrusage(RUSAGE_SELF, &ru);
    return (ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) * 1e6 + ru.ru_utime.tv_usec + ru.ru_stime.tv_usec;
}

static void priv_of(uint64_t tag, uint8_t out[32]) {
    // deterministic private keys in [1, n-1]: SHA-256(tag) with the top bit cleared
    uint8_t in[16] = "sbft-harness";
    std::memcpy(in + 8, &tag, 8);
    SHA256_CTX c;
    SHA256_Init(&c);
    SHA256_Update(&c, in, sizeof in);
    SHA256_Final(out, &c);
    out[0] &= 0x7f;
    out[31] |= 1;
}

// quorum-batch VOTES DECISIONS: the patched library's batch hook, one
// sbft_verifier_verify_consenter_sigs call with all VOTES signatures per decision, from one
// thread; 8 proposals in rotation (the digest memo misses every call). Latency = the call.
static int quorum_batch(int votes, int decisions) {
    sbft_gv_ctx* ctx = nullptr;
    if (sbft_gv_init(nullptr, &ctx)) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    sbft_verifier* v = sbft_verifier_new(ctx, 1);
    std::vector<sbft_signer*> signers;
    for (int i = 1; i <= votes; ++i) {
        uint8_t d[32], pub[65];
        priv_of(1000 + i, d);
        signers.push_back(sbft_signer_new(ctx, i, d));
        sbft_signer_public_key(signers.back(), pub);
        sbft_verifier_add_consenter(v, i, pub);
    }
    const int NB = 8;
    std::vector<std::string> payloads(NB);
    std::vector<sbft_proposal> props(NB);
    std::vector<std::vector<std::vector<uint8_t>>> msgs(NB), vals(NB);
    std::vector<std::vector<sbft_signature>> sigs(NB);
    for (int b = 0; b < NB; ++b) {
        payloads[b] = std::string(1300, 'a' + b);
        props[b] = sbft_proposal{(const uint8_t*)payloads[b].data(), payloads[b].size(), (const uint8_t*)"h", 1,
                                 (const uint8_t*)"m", 1, 1};
        for (int i = 0; i < votes; ++i) {
            std::vector<uint8_t> m(256), sig(64);
            size_t ml = 0;
            sbft_signer_sign_proposal(signers[i], &props[b], nullptr, 0, m.data(), m.size(), &ml, sig.data());
            m.resize(ml);
            msgs[b].push_back(m);
            vals[b].push_back(sig);
        }
        for (int i = 0; i < votes; ++i)
            sigs[b].push_back(sbft_signature{(uint64_t)(i + 1), vals[b][i].data(), 64, msgs[b][i].data(), msgs[b][i].size()});
    }
    std::vector<int32_t> st(votes);
    int wrong = 0;
    std::vector<double> t;
    for (int g = -5; g < decisions; ++g) {
        const int b = (g + 8) % NB;
        const auto t0 = Clock::now();
        const int rc = sbft_verifier_verify_consenter_sigs(v, sigs[b].data(), votes, &props[b], st.data());
        const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        if (g >= 0) t.push_back(us);
        if (rc) wrong++;
        for (int i = 0; i < votes; ++i) wrong += st[i] != 0;
    }
    std::printf("{\"mode\": \"quorum-batch\", \"votes\": %d, \"decisions\": %d, \"p50_ms\": %.4f, \"p99_ms\": %.4f, "
                "\"wrong_verdicts\": %d}\n", votes, decisions, pct(t, 50) / 1e3, pct(t, 99) / 1e3, wrong);
    for (auto* s : signers) sbft_signer_free(s);
    sbft_verifier_free(v);
    sbft_gv_destroy(ctx);
    return wrong ? 2 : 0;
}

static int quorum_gpu(int callers, int decisions, int cmax, int cwait) {
    sbft_gv_ctx* ctx = nullptr;
    if (sbft_gv_init(nullptr, &ctx)) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    sbft_verifier* v = sbft_verifier_new(ctx, 1);
    const int voters = callers + 1;  // the node's own signature is not verified (view.go:851-858)
    std::vector<sbft_signer*> signers;
    for (int i = 1; i <= voters; ++i) {
        uint8_t d[32], pub[65];
        priv_of(1000 + i, d);
        signers.push_back(sbft_signer_new(ctx, i, d));
        sbft_signer_public_key(signers.back(), pub);
        sbft_verifier_add_consenter(v, i, pub);
    }
    // 8 blocks in rotation: every decision checks a proposal the digest memo does not hold
    const int NB = 8;
    std::vector<std::string> payloads(NB);
    std::vector<sbft_proposal> props(NB);
    std::vector<std::vector<std::vector<uint8_t>>> msgs(NB), vals(NB);
    for (int b = 0; b < NB; ++b) {
        payloads[b] = std::string(1300, 'a' + b);
        props[b] = sbft_proposal{(const uint8_t*)payloads[b].data(), payloads[b].size(), (const uint8_t*)"h", 1,
                                 (const uint8_t*)"m", 1, 1};
        for (int i = 0; i < callers; ++i) {
            std::vector<uint8_t> m(256), sig(64);
            size_t ml = 0;
            sbft_signer_sign_proposal(signers[i + 1], &props[b], nullptr, 0, m.data(), m.size(), &ml, sig.data());
            m.resize(ml);
            msgs[b].push_back(m);
            vals[b].push_back(sig);
        }
    }
    if (cmax > 1) sbft_verifier_coalesce_consenter_sigs(v, cmax, cwait);
    std::atomic<int> wrong{0};
    auto run = [&](size_t i, int g) {
        const int b = g % NB;
        std::vector<uint8_t> val = vals[b][i];
        const bool bad = g % 10 == 9 && i == 7;
        if (bad) val[40] ^= 1;
        sbft_signature s{(uint64_t)(i + 2), val.data(), val.size(), msgs[b][i].data(), msgs[b][i].size()};
        uint8_t aux[64];
        size_t alen = 0;
        char err[256] = {0};
        const int rc = sbft_verifier_verify_consenter_sig(v, &s, &props[b], aux, sizeof aux, &alen, err, sizeof err);
        if (bad ? (rc != SBFT_V_EVERIFY || !std::strstr(err, "invalid signature")) : rc != 0) wrong++;
    };
    fan_out(callers, 5, run);  // warm-up: tables, staging, memo
    uint64_t l0, c0, l1, c1;
    sbft_verifier_consenter_stats(v, &l0, &c0);
    const CgroupCpu cg0 = cgroup_cpu();
    auto t = fan_out(callers, decisions, run);
    const CgroupCpu cg1 = cgroup_cpu();
    sbft_verifier_consenter_stats(v, &l1, &c1);
    int over1ms = 0;
    for (double us : t) over1ms += us > 1000.0;
    std::printf("{\"mode\": \"quorum-gpu\", \"callers\": %d, \"decisions\": %d, \"coalesce_max\": %d, "
                "\"coalesce_wait_us\": %d, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"max_ms\": %.4f, "
                "\"decisions_over_1ms\": %d, \"launches_per_decision\": %.2f, \"cpu_ms_per_decision\": %.3f, "
                "\"cgroup_throttled\": %lld, \"cgroup_throttled_ms\": %.3f, \"wrong_verdicts\": %d}\n",
                callers, decisions, cmax, cwait, pct(t, 50) / 1e3, pct(t, 99) / 1e3, pct(t, 100) / 1e3, over1ms,
                (double)(l1 - l0) / decisions, (cg1.usage_us - cg0.usage_us) / 1e3 / decisions,
                cg1.nr_throttled - cg0.nr_throttled, (cg1.throttled_us - cg0.throttled_us) / 1e3, wrong.load());
    for (auto* s : signers) sbft_signer_free(s);
    sbft_verifier_free(v);
    sbft_gv_destroy(ctx);
    return wrong.load() ? 2 : 0;
}

// ---- the processCommits batch hook (go/patches/internal_bft_commits.patch) with arriving votes ----
// Shared by quorum-hook and quorum-pipe. A channel (one consensus instance: its View goroutine
// and the replicas voting in it) owns VOTERS voter threads that deliver one commit vote each per
// decision, released together (the votes arriving from the network), and BatchWorkers that run
// the hook's VerifyConsenterSigs calls as the patch's goroutines do, so the collector keeps
// taking arrivals while a batch is in flight.
struct BatchWorker {
    std::thread th;
    std::atomic<int> st{0};  // 0 idle, 1 posted, 2 done, 3 stop
    sbft_verifier* v = nullptr;
    const sbft_proposal* p = nullptr;
    std::vector<sbft_signature> batch;
    std::vector<int> who;
    std::vector<int32_t> res;
    int rc = 0;
    const std::atomic<int>* armed = nullptr;  // the channel's decision is collecting: stay awake
    Waker* done = nullptr;                    // the collector's wait, notified when a batch is done
    // phase stamps (ns, steady clock): the collector's at post time, the worker's around the call
    int64_t post_ns = 0, wake_ns = 0, last_arr_ns = 0, call0_ns = 0, call1_ns = 0;
    std::atomic<int64_t>* engine_ns = nullptr;  // CPU time spent inside the engine's calls
    long spin_us = 10;  // after a batch, spin this long for the next one (SBFT_HOOK_WORKER_SPIN_US)
    void start() {
        th = std::thread([this] {
            pthread_setname_np(pthread_self(), "h-bworker");
            for (;;) {
                int s;
                const auto t0 = Clock::now();
                while ((s = st.load(std::memory_order_acquire)) != 1 && s != 3) {
                    if ((armed && armed->load(std::memory_order_relaxed)) ||
                        Clock::now() - t0 < std::chrono::microseconds(spin_us)) {  // a batch follows
                        __builtin_ia32_pause();                                    // an arrival closely
                        continue;
                    }
                    futex(&st, FUTEX_WAIT_PRIVATE, s);
                }
                if (s == 3) return;
                res.assign(batch.size(), 0);
                const int64_t c0 = thread_cpu_ns();
                call0_ns = now_ns();
                rc = sbft_verifier_verify_consenter_sigs(v, batch.data(), batch.size(), p, res.data());
                call1_ns = now_ns();
                if (engine_ns) engine_ns->fetch_add(thread_cpu_ns() - c0, std::memory_order_relaxed);
                st.store(2, std::memory_order_release);
                if (done) done->notify();
            }
        });
    }
    void post() {
        st.store(1, std::memory_order_release);
        futex(&st, FUTEX_WAKE_PRIVATE, 1);
    }
    void stop() {
        st.store(3, std::memory_order_release);
        futex(&st, FUTEX_WAKE_PRIVATE, 1);
        th.join();
    }
};

struct HookChannel {
    int voters, need, inflight;
    // delivery threads: 0 = one per voter (quorum-hook: each vote arrives from its own thread);
    // D > 0 = D threads, thread j delivering votes j, j + D, ... in turn (quorum-pipe: the node's
    // Go runtime runs its network goroutines on GOMAXPROCS threads, not one OS thread per peer)
    int deliverers = 0;
    // SBFT_HOOK_ARM=1: the batch workers spin from the release of a decision's votes until its
    // quorum (one core each while collecting) instead of sleeping until a batch is posted; the
    // futex wake of a sleeping worker otherwise lies on every decision's critical path
    std::atomic<int> armed{0};
    bool arm = false;
    sbft_verifier* v;
    const std::vector<sbft_proposal>* props;
    const std::vector<std::vector<std::vector<uint8_t>>>*msgs, *vals, *bads;
    std::unique_ptr<std::atomic<int>[]> order;
    std::unique_ptr<int64_t[]> arr_ns;  // delivery time of arrival k (written before order[k])
    std::atomic<int> arrived{0}, gen{-1};
    // per decision, the batch that completed the quorum (quorum-hook's breakdown, microseconds):
    // release -> its last vote delivered | -> the collector awake for it | -> batch posted |
    // -> the worker in the engine call | the call | -> the View (collector) has the verdicts
    std::vector<double> ph_arrive, ph_wake, ph_post, ph_pickup, ph_call, ph_view;
    std::atomic<bool> stop_{false};
    std::vector<std::thread> th;
    std::vector<std::unique_ptr<BatchWorker>> w;
    int launches = 0, wrong = 0;
    // the collector (the View goroutine) blocks while nothing arrives, as processCommits' select
    // does (view.go:532-549); SBFT_HOOK_COLLECT_SPIN_US bounds its spin first (default 20 us)
    Waker waker;
    // arrivals that can change the collector's next step: it sleeps until arrived >= wake_at (the
    // count at which the quorum becomes reachable) or a batch finishes, so only that voter wakes
    // it (one futex wake per step instead of one per vote; the batches launched are the same)
    std::atomic<int> wake_at{0};
    std::atomic<int64_t> engine_ns{0};

    void start() {
        waker.spin_us = env_long("SBFT_HOOK_COLLECT_SPIN_US", 20);
        order.reset(new std::atomic<int>[voters]);
        arr_ns.reset(new int64_t[voters]);
        for (int i = 0; i < voters; ++i) order[i].store(0);
        const int nd = deliverers > 0 ? std::min(deliverers, voters) : voters;
        for (int j = 0; j < nd; ++j)
            th.emplace_back([this, j, nd] {
                pthread_setname_np(pthread_self(), "h-voter");
                int seen = -1;
                for (;;) {
                    int g;
                    bool slept = false;
                    while ((g = gen.load(std::memory_order_acquire)) == seen && !stop_.load()) {
                        futex(&gen, FUTEX_WAIT_PRIVATE, seen);
                        slept = true;
                    }
                    if (slept) futex(&gen, FUTEX_WAKE_PRIVATE, 2);  // the release is a wake-up tree
                    if (stop_.load()) return;
                    seen = g;
                    for (int i = j; i < voters; i += nd) {
                        const int k = arrived.fetch_add(1, std::memory_order_seq_cst);
                        arr_ns[k] = now_ns();
                        order[k].store(i + 1, std::memory_order_release);
                        if (k + 1 >= wake_at.load(std::memory_order_seq_cst)) waker.notify();
                    }
                }
            });
        const char* e = std::getenv("SBFT_HOOK_ARM");
        arm = e && std::atoi(e) != 0;
        for (int k = 0; k < std::max(1, inflight); ++k) {
            w.emplace_back(new BatchWorker());
            w.back()->v = v;
            w.back()->armed = &armed;
            w.back()->done = &waker;
            w.back()->engine_ns = &engine_ns;
            w.back()->spin_us = env_long("SBFT_HOOK_WORKER_SPIN_US", 10);
            w.back()->start();
        }
    }
    bool worker_done() const {
        for (auto& x : w)
            if (x->st.load(std::memory_order_acquire) == 2) return true;
        return false;
    }
    void finish() {
        stop_.store(true);
        gen.fetch_add(1);
        futex(&gen, FUTEX_WAKE_PRIVATE, INT_MAX);
        for (auto& x : th) x.join();
        for (auto& x : w) x->stop();
    }
    // One decision on proposal b (voter 7's vote is bad when bad_dec): release the votes, collect
    // NEED valid ones through the hook. Returns release -> quorum in microseconds.
    double decide(int g, int b, bool bad_dec) {
        for (int k = 0; k < voters; ++k) order[k].store(0, std::memory_order_relaxed);
        arrived.store(0, std::memory_order_release);
        const auto t0 = Clock::now();
        gen.store(g, std::memory_order_release);
        futex(&gen, FUTEX_WAKE_PRIVATE, 2);
        if (arm) {
            armed.store(1, std::memory_order_relaxed);
            for (auto& x : w) futex(&x->st, FUTEX_WAKE_PRIVATE, 1);
        }
        int valid = 0, consumed = 0, in_flight = 0, in_votes = 0;
        int64_t wake_ns = now_ns(), last_arr = 0;
        const int64_t t0_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count();
        std::vector<int> pending;
        auto harvest = [&](BatchWorker& x) {
            if (x.rc) wrong++;
            const bool short_before = valid < need;
            for (size_t k = 0; k < x.batch.size(); ++k) {
                const bool is_bad = bad_dec && x.who[k] == 7;
                if (is_bad != (x.res[k] != 0)) wrong++;
                if (!x.res[k] && valid < need) ++valid;
            }
            if (short_before && valid >= need) {  // this batch completed the quorum
                const int64_t h = now_ns();
                ph_arrive.push_back((x.last_arr_ns - t0_ns) / 1e3);
                ph_wake.push_back(std::max<int64_t>(0, x.wake_ns - x.last_arr_ns) / 1e3);
                ph_post.push_back((x.post_ns - std::max(x.wake_ns, x.last_arr_ns)) / 1e3);
                ph_pickup.push_back((x.call0_ns - x.post_ns) / 1e3);
                ph_call.push_back((x.call1_ns - x.call0_ns) / 1e3);
                ph_view.push_back((h - x.call1_ns) / 1e3);
            }
            in_flight--;
            in_votes -= (int)x.batch.size();
            x.st.store(0, std::memory_order_release);
        };
        while (valid < need) {
            bool progress = false;
            for (auto& x : w)
                if (x->st.load(std::memory_order_acquire) == 2) {
                    harvest(*x);
                    progress = true;
                }
            if (valid >= need) break;
            const int a = arrived.load(std::memory_order_acquire);
            for (; consumed < a; ++consumed) {
                int i;
                while ((i = order[consumed].load(std::memory_order_acquire)) == 0) __builtin_ia32_pause();
                pending.push_back(i - 1);
                last_arr = arr_ns[consumed];
                progress = true;
            }
            // the patch's canLaunch: quorum reachable, a batch slot free
            if (!pending.empty() && in_flight < inflight && valid + in_votes + (int)pending.size() >= need) {
                BatchWorker* x = nullptr;
                for (auto& y : w)
                    if (y->st.load(std::memory_order_acquire) == 0) x = y.get();
                x->p = &(*props)[b];
                x->batch.clear();
                x->who.clear();
                for (int i : pending) {
                    const auto& val = (bad_dec && i == 7) ? (*bads)[b][i] : (*vals)[b][i];
                    x->batch.push_back(
                        sbft_signature{(uint64_t)(i + 2), val.data(), 64, (*msgs)[b][i].data(), (*msgs)[b][i].size()});
                    x->who.push_back(i);
                }
                pending.clear();
                in_flight++;
                in_votes += (int)x->batch.size();
                ++launches;
                x->wake_ns = wake_ns;
                x->last_arr_ns = last_arr;
                x->post_ns = now_ns();
                x->post();
                progress = true;
            }
            if (!progress) {
                if (a == voters && in_flight == 0 && pending.empty()) break;  // all in, quorum short
                // nothing to do: sleep until enough votes arrive to make the quorum reachable, or
                // a batch finishes (the patch's select; view.go:532-549). With both batch slots
                // busy only a finished batch can change anything.
                const int short_by = need - valid - in_votes - (int)pending.size();
                const int want = in_flight < inflight ? consumed + std::max(1, short_by) : INT_MAX;
                wake_at.store(std::min(want, voters), std::memory_order_seq_cst);
                waker.wait([&] {
                    return arrived.load(std::memory_order_seq_cst) >= wake_at.load(std::memory_order_relaxed) ||
                           worker_done();
                });
                wake_at.store(0, std::memory_order_relaxed);
                wake_ns = now_ns();
            }
        }
        const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        armed.store(0, std::memory_order_relaxed);
        if (valid != need) wrong++;
        // drain: batches still in flight and the remaining arrivals (outside the latency)
        for (auto& x : w)
            while (x->st.load(std::memory_order_acquire) != 0) {
                if (x->st.load(std::memory_order_acquire) == 2) harvest(*x);
                else waker.wait([&] { return x->st.load(std::memory_order_acquire) != 1; });
            }
        wake_at.store(voters, std::memory_order_seq_cst);
        waker.wait([&] { return arrived.load(std::memory_order_seq_cst) >= voters; });
        wake_at.store(0, std::memory_order_relaxed);
        for (int k = 0; k < voters; ++k)
            while (order[k].load(std::memory_order_acquire) == 0) __builtin_ia32_pause();
        return us;
    }
};

// Signed commit votes of NB proposals by consenters 2..VOTERS+1 (and a corrupted copy of each).
struct VoteSet {
    static constexpr int NB = 8;
    std::vector<sbft_signer*> signers;
    std::vector<std::string> payloads;
    std::vector<sbft_proposal> props;
    std::vector<std::vector<std::vector<uint8_t>>> msgs, vals, bads;
    VoteSet(sbft_gv_ctx* ctx, sbft_verifier* v, int voters, uint64_t tag) : payloads(NB), props(NB), msgs(NB), vals(NB), bads(NB) {
        for (int i = 1; i <= voters + 1; ++i) {
            uint8_t d[32], pub[65];
            priv_of(tag + i, d);
            signers.push_back(sbft_signer_new(ctx, i, d));
            sbft_signer_public_key(signers.back(), pub);
            sbft_verifier_add_consenter(v, i, pub);
        }
        for (int b = 0; b < NB; ++b) {
            payloads[b] = std::string(1300, (char)('a' + b + (int)(tag % 7)));
            props[b] = sbft_proposal{(const uint8_t*)payloads[b].data(), payloads[b].size(), (const uint8_t*)"h", 1,
                                     (const uint8_t*)"m", 1, 1};
            for (int i = 0; i < voters; ++i) {
                std::vector<uint8_t> m(256), sig(64);
                size_t ml = 0;
                sbft_signer_sign_proposal(signers[i + 1], &props[b], nullptr, 0, m.data(), m.size(), &ml, sig.data());
                m.resize(ml);
                msgs[b].push_back(m);
                vals[b].push_back(sig);
                sig[40] ^= 1;
                bads[b].push_back(sig);
            }
        }
    }
    ~VoteSet() {
        for (auto* s : signers) sbft_signer_free(s);
    }
};

// quorum-hook VOTERS NEED DECISIONS INFLIGHT: the patched processCommits. VOTERS threads deliver one
// commit vote each per decision, released together; the collector (this thread, the View
// goroutine) takes them in arrival order and, once the valid votes so far plus the ones in flight
// and pending can complete the quorum, hands the pending ones to a batch worker (one
// sbft_verifier_verify_consenter_sigs call), with at most INFLIGHT calls in flight: votes that
// arrive during a call go out as the next one at once (INFLIGHT = 1: they wait for it, the round-3
// hook). Latency = release -> NEED valid votes collected. Every 10th decision carries one bad
// vote (voter 7), so VOTERS = NEED + 1 lets the spare vote complete that quorum, as a 67th
// replica's vote would at n = 100.
static int quorum_hook(int voters, int need, int decisions, int inflight) {
    sbft_gv_ctx* ctx = nullptr;
    if (sbft_gv_init(nullptr, &ctx)) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    sbft_verifier* v = sbft_verifier_new(ctx, 1);
    int wrong = 0, launches = 0;
    std::vector<double> t;
    std::string phases = "{}";
    uint64_t klaunch = 0;
    double kms = 0;
    {
        VoteSet vs(ctx, v, voters, 1000);
        HookChannel ch;
        ch.voters = voters;
        ch.need = need;
        ch.inflight = std::max(1, inflight);
        ch.v = v;
        ch.props = &vs.props;
        ch.msgs = &vs.msgs;
        ch.vals = &vs.vals;
        ch.bads = &vs.bads;
        ch.start();
        for (int g = -5; g < decisions; ++g) {
            if (g == 0) {
                ch.launches = 0;
                for (auto* ph : {&ch.ph_arrive, &ch.ph_wake, &ch.ph_post, &ch.ph_pickup, &ch.ph_call, &ch.ph_view})
                    ph->clear();
                (void)sbft_gv_kernel_timing(ctx, 1);  // HIP events around every keyed launch
                (void)sbft_gv_kernel_time(ctx, &klaunch, &kms);
            }
            const double us = ch.decide(g + 5, (g + 80) % VoteSet::NB, g % 10 == 9);
            if (g >= 0) t.push_back(us);
        }
        ch.finish();
        (void)sbft_gv_kernel_time(ctx, &klaunch, &kms);
        wrong = ch.wrong;
        launches = ch.launches;
        char buf[512];
        std::snprintf(buf, sizeof buf,
                      "{\"release_to_last_vote_us\": %.1f, \"collector_wake_us\": %.1f, \"batch_post_us\": %.1f, "
                      "\"worker_pickup_us\": %.1f, \"engine_call_us\": %.1f, \"view_wake_us\": %.1f, "
                      "\"keyed_kernel_us_mean\": %.1f, \"timed_launches\": %llu}",
                      pct(ch.ph_arrive, 50), pct(ch.ph_wake, 50), pct(ch.ph_post, 50), pct(ch.ph_pickup, 50),
                      pct(ch.ph_call, 50), pct(ch.ph_view, 50), klaunch ? kms * 1e3 / (double)klaunch : 0.0,
                      (unsigned long long)klaunch);
        phases = buf;
    }
    std::printf("{\"mode\": \"quorum-hook\", \"voters\": %d, \"need\": %d, \"decisions\": %d, \"inflight\": %d, "
                "\"p50_ms\": %.4f, \"p99_ms\": %.4f, \"max_ms\": %.4f, \"launches_per_decision\": %.2f, "
                "\"phases_p50\": %s, \"wrong_verdicts\": %d}\n",
                voters, need, decisions, std::max(1, inflight), pct(t, 50) / 1e3, pct(t, 99) / 1e3, pct(t, 100) / 1e3,
                (double)launches / decisions, phases.c_str(), wrong);
    sbft_verifier_free(v);
    sbft_gv_destroy(ctx);
    return wrong ? 2 : 0;
}

// SHA-256 through the low-level interface: OpenSSL 3's one-shot SHA256() fetches the digest
// from the library context on every call, which serialises threads on its lock
static void sha256_ll(const uint8_t* m, size_t n, uint8_t h[32]) {
    SHA256_CTX c;
    SHA256_Init(&c);
    SHA256_Update(&c, m, n);
    SHA256_Final(h, &c);
}

struct CpuTuple {
    std::vector<uint8_t> msg;
    EC_KEY* key;
    ECDSA_SIG* sig;
};

static std::vector<CpuTuple> cpu_tuples(int n, int min_len, int max_len) {
    std::vector<CpuTuple> out(n);
    EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    uint32_t x = 12345;
    for (int i = 0; i < n; ++i) {
        x = x * 1103515245u + 12345u;
        const int len = min_len + (int)(x % (uint32_t)(max_len - min_len + 1));
        out[i].msg.resize(len);
        for (int j = 0; j < len; ++j) out[i].msg[j] = (uint8_t)(i * 31 + j * 7);
        EC_KEY* k = EC_KEY_new();
        EC_KEY_set_group(k, grp);
        EC_KEY_generate_key(k);
        uint8_t h[32];
        sha256_ll(out[i].msg.data(), len, h);
        {
            // r, s re-imported as plain BIGNUMs (a signer's BIGNUMs carry flags such as
            // constant-time that would slow the verify down)
            ECDSA_SIG* sg = ECDSA_do_sign(h, 32, k);
            uint8_t rb[32], sb[32];
            BN_bn2binpad(ECDSA_SIG_get0_r(sg), rb, 32);
            BN_bn2binpad(ECDSA_SIG_get0_s(sg), sb, 32);
            ECDSA_SIG_free(sg);
            out[i].sig = ECDSA_SIG_new();
            ECDSA_SIG_set0(out[i].sig, BN_bin2bn(rb, 32, nullptr), BN_bin2bn(sb, 32, nullptr));
        }
        // the verifier's key is decoded from its SEC1 bytes (affine, public only), as a
        // plugin holds it; a generated key object carries a projective point that every
        // verify would convert again
        uint8_t oct[65];
        EC_POINT_point2oct(grp, EC_KEY_get0_public_key(k), POINT_CONVERSION_UNCOMPRESSED, oct, 65, nullptr);
        EC_KEY* pk = EC_KEY_new();
        EC_KEY_set_group(pk, grp);
        EC_KEY_oct2key(pk, oct, 65, nullptr);
        EC_KEY_free(k);
        out[i].key = pk;
    }
    EC_GROUP_free(grp);
    return out;
}

static bool cpu_verify(const CpuTuple& t) {
    uint8_t h[32];
    sha256_ll(t.msg.data(), t.msg.size(), h);
    return ECDSA_do_verify(h, 32, t.sig, t.key) == 1;
}

static int quorum_cpu(int callers, int decisions, int threads) {
    auto tup = cpu_tuples(callers, 128, 128);
    std::atomic<int> bad{0};
    const int nt = std::max(1, std::min(threads, callers));
    auto t = fan_out(nt, decisions, [&](size_t i, int) {
        for (int k = (int)i; k < callers; k += nt)
            if (!cpu_verify(tup[k])) bad++;
    });
    std::printf("{\"mode\": \"quorum-cpu\", \"callers\": %d, \"decisions\": %d, \"threads\": %d, \"p50_ms\": %.4f, "
                "\"p99_ms\": %.4f, \"rejected\": %d}\n",
                callers, decisions, nt, pct(t, 50) / 1e3, pct(t, 99) / 1e3, bad.load());
    return 0;
}

// quorum-vote-cpu VOTERS NEED DECISIONS THREADS: the stock processCommits with an OpenSSL plugin,
// under the same arrivals as quorum-hook: VOTERS votes released together per decision (a
// wake-up tree), every vote verified as it arrives (view.go:537-541: a goroutine per vote; with
// THREADS < VOTERS a pool of THREADS, thread j taking votes j, j + THREADS, ...), and the View
// continuing once NEED are valid. Every 10th decision carries one bad vote (voter 7), as in
// quorum-hook, so those decisions wait for the spare vote. Latency = release -> NEED valid.
static int quorum_vote_cpu(int voters, int need, int decisions, int threads) {
    auto votes = cpu_tuples(voters, 128, 128);
    const int nt = std::max(1, std::min(threads, voters));
    const int total = decisions + 5;
    std::unique_ptr<std::atomic<int>[]> valid(new std::atomic<int>[total]), done(new std::atomic<int>[total]);
    for (int k = 0; k < total; ++k) {
        valid[k].store(0);
        done[k].store(0);
    }
    std::atomic<int> gen{-1};
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    Waker wk;  // the View blocks until the quorum (or the last vote) is in, as the GPU collector
    wk.spin_us = env_long("SBFT_HOOK_COLLECT_SPIN_US", 20);
    for (int j = 0; j < nt; ++j)
        th.emplace_back([&, j] {
            int seen = -1;
            for (;;) {
                int g;
                bool slept = false;
                while ((g = gen.load(std::memory_order_acquire)) == seen && !stop.load()) {
                    futex(&gen, FUTEX_WAIT_PRIVATE, seen);
                    slept = true;
                }
                if (slept) futex(&gen, FUTEX_WAKE_PRIVATE, 2);  // the release is a wake-up tree
                if (stop.load()) return;
                for (int k = seen + 1; k <= g; ++k)
                    for (int i = j; i < voters; i += nt) {
                        const bool bad = k % 10 == 4 && i == 7;  // decisions 9, 19, ... after warm-up
                        const bool last_valid = cpu_verify(votes[i]) && !bad &&
                                                valid[k].fetch_add(1, std::memory_order_seq_cst) + 1 == need;
                        if (done[k].fetch_add(1, std::memory_order_seq_cst) + 1 == voters || last_valid) wk.notify();
                    }
                seen = g;
            }
        });
    std::vector<double> t;
    int wrong = 0;
    for (int g = 0; g < total; ++g) {
        const auto t0 = Clock::now();
        gen.store(g, std::memory_order_release);
        futex(&gen, FUTEX_WAKE_PRIVATE, 2);
        // all in with the quorum short ends it too
        wk.wait([&] {
            return valid[g].load(std::memory_order_seq_cst) >= need || done[g].load(std::memory_order_seq_cst) == voters;
        });
        const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        if (g >= 5) t.push_back(us);
        // drain the spare vote (outside the latency), as quorum-hook does
        wk.wait([&] { return done[g].load(std::memory_order_seq_cst) == voters; });
        if (valid[g].load() < need) wrong++;
    }
    stop.store(true);
    gen.fetch_add(1);
    futex(&gen, FUTEX_WAKE_PRIVATE, INT_MAX);
    for (auto& x : th) x.join();
    std::printf("{\"mode\": \"quorum-vote-cpu\", \"voters\": %d, \"need\": %d, \"decisions\": %d, \"threads\": %d, "
                "\"p50_ms\": %.4f, \"p99_ms\": %.4f, \"max_ms\": %.4f, \"wrong_verdicts\": %d}\n",
                voters, need, decisions, nt, pct(t, 50) / 1e3, pct(t, 99) / 1e3, pct(t, 100) / 1e3, wrong);
    return wrong ? 2 : 0;
}

// VerifyConsenterSigs on the CPU (the prev-commit batch hook with an OpenSSL plugin): the batch's
// signatures spread over the calling thread and `helpers` pool threads pulling indices from an
// atomic counter, as a Go plugin would fan them out over goroutines on GOMAXPROCS threads. The
// caller blocks (bounded spin, then a futex) until the last signature is verified.
struct CpuBatchPool {
    std::vector<std::thread> th;
    std::atomic<int> gen{0}, next{0}, left{0}, bad{0};
    std::atomic<bool> stop{false};
    const std::vector<CpuTuple>* job = nullptr;  // the same vector every call (one channel's batch)
    Waker done;
    void start(int helpers, const std::vector<CpuTuple>* batch) {
        job = batch;
        done.spin_us = env_long("SBFT_HOOK_COLLECT_SPIN_US", 20);
        for (int j = 0; j < helpers; ++j)
            th.emplace_back([this] {
                pthread_setname_np(pthread_self(), "h-cpubatch");
                int seen = 0;
                for (;;) {
                    int g;
                    while ((g = gen.load(std::memory_order_acquire)) == seen && !stop.load())
                        futex(&gen, FUTEX_WAIT_PRIVATE, seen);
                    if (stop.load()) return;
                    seen = g;
                    work();
                }
            });
    }
    void work() {
        const int n = (int)job->size();
        int i, mine = 0;
        while ((i = next.fetch_add(1, std::memory_order_acq_rel)) < n) {
            if (!cpu_verify((*job)[i])) bad.fetch_add(1, std::memory_order_relaxed);
            ++mine;
        }
        if (mine && left.fetch_sub(mine, std::memory_order_acq_rel) == mine) done.notify();
    }
    int verify_all() {  // failures in the batch
        bad.store(0, std::memory_order_relaxed);
        left.store((int)job->size(), std::memory_order_relaxed);
        next.store(0, std::memory_order_release);
        gen.fetch_add(1, std::memory_order_release);
        futex(&gen, FUTEX_WAKE_PRIVATE, INT_MAX);
        work();
        done.wait([&] { return left.load(std::memory_order_acquire) == 0; });
        return bad.load();
    }
    void finish() {
        stop.store(true);
        gen.fetch_add(1);
        futex(&gen, FUTEX_WAKE_PRIVATE, INT_MAX);
        for (auto& t : th) t.join();
    }
};

// quorum-pipe CHANNELS DECISIONS gpu|cpu|cpu-batched: pipelined decisions at n = 100 (config 4). CHANNELS
// consensus instances on one node (e.g. one SmartBFT orderer per channel, sharing the node's
// cores and GPU) each decide back to back, so CHANNELS decisions are always in flight. A
// decision is what the View verifies per block: the previous decision's 67 commit signatures
// (verifyPrevCommitSignatures, view.go:606-647), then 66 of the 67 arriving commit votes
// (processCommits, view.go:519-551; every 10th decision has a bad vote).
//   gpu: the patched library: one VerifyConsenterSigs call for the 67 prev-commit signatures,
//        the processCommits hook (quorum-hook, two batches in flight) for the votes.
//   cpu: the stock library with an OpenSSL plugin: the prev-commit loop verifies serially on
//        the View goroutine; every vote is verified by its own goroutine (a voter thread here),
//        and the View continues once 66 are valid.
//   cpu-batched: the patched library with an OpenSSL plugin (the fair CPU leg):
//        the prev-commit hook's VerifyConsenterSigs spreads the 67 signatures over the channel's
//        share of the job's cores (CpuBatchPool); votes as in cpu (each verified as it arrives).
// Reports decisions/s over all channels, p50/p99 per decision and CPU ms per decision (cgroup).
static int quorum_pipe(int channels, int decisions, bool gpu, bool batched = false) {
    const int voters = 67, need = 66;
    channels = std::max(1, channels);
    // the node's goroutines run on GOMAXPROCS threads: the job's cores, shared by the channels
    // (SBFT_PIPE_DELIVERERS per channel overrides; 0 = one OS thread per vote, the round-4 harness)
    const int deliverers = (int)env_long("SBFT_PIPE_DELIVERERS", std::max(1, (int)host_cores() / channels));
    std::vector<std::vector<double>> lat(channels);
    std::atomic<int> wrong{0};
    double wall_s = 0, cpu0 = 0, cpu1 = 0;
    CgroupCpu cg0, cg1;
    ThreadCpu tc0, tc1;
    std::atomic<int64_t> engine_ns{0};
    int launches = 0;
    if (gpu) {
        sbft_gv_ctx* ctx = nullptr;
        if (sbft_gv_init(nullptr, &ctx)) {
            std::fprintf(stderr, "no GPU\n");
            return 1;
        }
        std::vector<sbft_verifier*> vs;
        std::vector<std::unique_ptr<VoteSet>> sets;
        std::vector<std::unique_ptr<HookChannel>> chs;
        for (int c = 0; c < channels; ++c) {
            vs.push_back(sbft_verifier_new(ctx, 1));
            sets.emplace_back(new VoteSet(ctx, vs[c], voters, 5000 + 1000 * (uint64_t)c));
            chs.emplace_back(new HookChannel());
            HookChannel& ch = *chs.back();
            ch.voters = voters;
            ch.need = need;
            ch.inflight = 2;
            ch.deliverers = deliverers;
            ch.v = vs[c];
            ch.props = &sets[c]->props;
            ch.msgs = &sets[c]->msgs;
            ch.vals = &sets[c]->vals;
            ch.bads = &sets[c]->bads;
            ch.start();
        }
        auto run = [&](int c, int from, int to) {
            pthread_setname_np(pthread_self(), "h-collect");
            HookChannel& ch = *chs[c];
            VoteSet& s = *sets[c];
            std::vector<sbft_signature> prev(voters);
            std::vector<int32_t> st(voters);
            for (int g = from; g < to; ++g) {
                const int b = (g + 80) % VoteSet::NB, pb = (g + 79) % VoteSet::NB;
                const auto t0 = Clock::now();
                for (int i = 0; i < voters; ++i)  // the previous block's commit signatures
                    prev[i] = sbft_signature{(uint64_t)(i + 2), s.vals[pb][i].data(), 64, s.msgs[pb][i].data(),
                                             s.msgs[pb][i].size()};
                const int64_t c0 = thread_cpu_ns();
                if (sbft_verifier_verify_consenter_sigs(vs[c], prev.data(), voters, &s.props[pb], st.data())) wrong++;
                if (g >= 0) engine_ns.fetch_add(thread_cpu_ns() - c0, std::memory_order_relaxed);
                for (int i = 0; i < voters; ++i) wrong += st[i] != 0;
                ch.decide(g + 10, b, g % 10 == 9);
                if (g >= 0) lat[c].push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
            }
        };
        {  // warm-up
            std::vector<std::thread> th;
            for (int c = 0; c < channels; ++c) th.emplace_back(run, c, -5, 0);
            for (auto& t : th) t.join();
        }
        for (auto& ch : chs) {
            ch->launches = 0;
            ch->engine_ns = 0;
        }
        cg0 = cgroup_cpu();
        cpu0 = proc_cpu_us();
        tc0 = ThreadCpu::now();
        const auto t0 = Clock::now();
        {
            std::vector<std::thread> th;
            for (int c = 0; c < channels; ++c) th.emplace_back(run, c, 0, decisions);
            for (auto& t : th) t.join();
        }
        wall_s = std::chrono::duration<double>(Clock::now() - t0).count();
        tc1 = ThreadCpu::now();
        cpu1 = proc_cpu_us();
        cg1 = cgroup_cpu();
        for (auto& ch : chs) {
            ch->finish();
            wrong += ch->wrong;
            launches += ch->launches;
            engine_ns += ch->engine_ns.load();
        }
        sets.clear();
        for (auto* v : vs) sbft_verifier_free(v);
        sbft_gv_destroy(ctx);
    } else {
        // per channel: 67 prev-commit tuples (serial loop) and 67 vote tuples (one thread each)
        std::vector<std::vector<CpuTuple>> prev(channels), votes(channels);
        for (int c = 0; c < channels; ++c) {
            prev[c] = cpu_tuples(voters, 128, 128);
            votes[c] = cpu_tuples(voters, 128, 128);
        }
        const int total = decisions + 5;
        std::vector<std::unique_ptr<std::atomic<int>[]>> valid(channels);
        for (int c = 0; c < channels; ++c) {
            valid[c].reset(new std::atomic<int>[total]);
            for (int k = 0; k < total; ++k) valid[c][k].store(0);
        }
        std::vector<std::unique_ptr<std::atomic<int>>> gen;
        for (int c = 0; c < channels; ++c) gen.emplace_back(new std::atomic<int>(-1));
        // cpu-batched: each channel's View plus host_cores / channels - 1 pool threads
        std::vector<std::unique_ptr<CpuBatchPool>> pools;
        if (batched)
            for (int c = 0; c < channels; ++c) {
                pools.emplace_back(new CpuBatchPool());
                pools.back()->start(std::max(0, (int)host_cores() / channels - 1), &prev[c]);
            }
        std::atomic<bool> stop{false};
        std::vector<std::thread> vth;
        // the View blocks on the valid-vote channel as the GPU side's collector does (Waker)
        std::vector<std::unique_ptr<Waker>> wk;
        for (int c = 0; c < channels; ++c) {
            wk.emplace_back(new Waker());
            wk.back()->spin_us = env_long("SBFT_HOOK_COLLECT_SPIN_US", 20);
        }
        const int nd = deliverers > 0 ? std::min(deliverers, voters) : voters;
        for (int c = 0; c < channels; ++c)
            for (int j = 0; j < nd; ++j)
                vth.emplace_back([&, c, j, nd] {
                    pthread_setname_np(pthread_self(), "h-voter");
                    int seen = -1;
                    for (;;) {
                        int g;
                        while ((g = gen[c]->load(std::memory_order_acquire)) == seen && !stop.load())
                            futex(gen[c].get(), FUTEX_WAIT_PRIVATE, seen);
                        if (stop.load()) return;
                        for (int k = seen + 1; k <= g; ++k)  // every decision released since
                            for (int i = j; i < voters; i += nd) {  // a goroutine per vote, on nd threads
                                const bool bad = k % 10 == 4 && i == 7;
                                if (cpu_verify(votes[c][i]) && !bad &&
                                    valid[c][k].fetch_add(1, std::memory_order_seq_cst) + 1 == need)
                                    wk[c]->notify();  // the vote that completes the quorum wakes the View
                            }
                        seen = g;
                    }
                });
        auto run = [&](int c, int from, int to) {
            pthread_setname_np(pthread_self(), "h-collect");
            for (int g = from; g < to; ++g) {
                const auto t0 = Clock::now();
                if (batched) wrong += pools[c]->verify_all();  // the prev-commit hook, over the cores
                else
                    for (int i = 0; i < voters; ++i) wrong += !cpu_verify(prev[c][i]);  // serial (view.go:630-644)
                gen[c]->store(g, std::memory_order_release);
                futex(gen[c].get(), FUTEX_WAKE_PRIVATE, INT_MAX);
                wk[c]->wait([&] { return valid[c][g].load(std::memory_order_acquire) >= need; });
                if (g >= 5) lat[c].push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
            }
        };
        {
            std::vector<std::thread> th;
            for (int c = 0; c < channels; ++c) th.emplace_back(run, c, 0, 5);
            for (auto& t : th) t.join();
        }
        cg0 = cgroup_cpu();
        cpu0 = proc_cpu_us();
        tc0 = ThreadCpu::now();
        const auto t0 = Clock::now();
        {
            std::vector<std::thread> th;
            for (int c = 0; c < channels; ++c) th.emplace_back(run, c, 5, total);
            for (auto& t : th) t.join();
        }
        wall_s = std::chrono::duration<double>(Clock::now() - t0).count();
        tc1 = ThreadCpu::now();
        cpu1 = proc_cpu_us();
        cg1 = cgroup_cpu();
        stop.store(true);
        for (int c = 0; c < channels; ++c) {
            gen[c]->fetch_add(1);
            futex(gen[c].get(), FUTEX_WAKE_PRIVATE, INT_MAX);
        }
        for (auto& t : vth) t.join();
        for (auto& pl : pools) pl->finish();
        for (int c = 0; c < channels; ++c)
            for (int k = 5; k < total; ++k)
                if (valid[c][k].load() < need) wrong++;
    }
    std::vector<double> all;
    for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
    const double nd = (double)channels * decisions;
    std::printf("{\"mode\": \"quorum-pipe\", \"backend\": \"%s\", \"channels\": %d, \"decisions_per_channel\": %d, "
                "\"decisions_per_s\": %.1f, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"cpu_ms_per_decision\": %.3f, "
                "\"engine_call_cpu_ms_per_decision\": %.3f, \"cpu_ms_per_decision_by_thread\": %s, "
                "\"delivery_threads_per_channel\": %d, "
                "\"launches_per_decision\": %.2f, \"cgroup_throttled\": %lld, \"wrong_verdicts\": %d}\n",
                gpu ? "gpu" : batched ? "cpu-batched" : "cpu", channels, decisions, nd / wall_s, pct(all, 50) / 1e3, pct(all, 99) / 1e3,
                (cpu1 - cpu0) / 1e3 / nd, engine_ns.load() / 1e6 / nd, cpu_json(tc1.since(tc0), nd).c_str(),
                deliverers > 0 ? std::min(deliverers, voters) : voters,
                gpu ? 1.0 + (double)launches / nd : 0.0, cg1.nr_throttled - cg0.nr_throttled, wrong.load());
    return wrong.load() ? 2 : 0;
}

// sign CALLS: SignProposal's signing (view.go:481) one message at a time from one thread:
// sbft_signer_sign (RFC 6979 nonce on the host, the GPU latency-path kernel) against OpenSSL
// ECDSA_do_sign (ecp_nistz256, random nonce) on the same 128-byte messages.
static int sign_both(int calls) {
    sbft_gv_ctx* ctx = nullptr;
    if (sbft_gv_init(nullptr, &ctx)) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    uint8_t d[32];
    priv_of(4242, d);
    sbft_signer* sg = sbft_signer_new(ctx, 1, d);
    std::vector<uint8_t> msg(128, 7), sig(64);
    std::vector<double> tg, tc;
    int bad = 0;
    for (int i = -5; i < calls; ++i) {
        msg[0] = (uint8_t)i;
        msg[1] = (uint8_t)(i >> 8);
        const auto t0 = Clock::now();
        bad += sbft_signer_sign(sg, msg.data(), msg.size(), sig.data()) != 0;
        if (i >= 0) tg.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    // the pre-signature pool (sbft_signer_presign): refills of 1,024 included in the samples
    std::vector<double> tp;
    if (sbft_signer_presign(sg, 1024)) bad++;
    for (int i = 0; i < 3 * calls; ++i) {
        msg[0] = (uint8_t)i;
        msg[1] = (uint8_t)(i >> 8);
        const auto t0 = Clock::now();
        bad += sbft_signer_sign(sg, msg.data(), msg.size(), sig.data()) != 0;
        tp.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    EC_KEY* k = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
    EC_KEY_generate_key(k);
    for (int i = -5; i < calls; ++i) {
        msg[0] = (uint8_t)i;
        msg[1] = (uint8_t)(i >> 8);
        const auto t0 = Clock::now();
        uint8_t h[32];
        sha256_ll(msg.data(), msg.size(), h);
        ECDSA_SIG* s = ECDSA_do_sign(h, 32, k);
        if (i >= 0) tc.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
        bad += s == nullptr;
        ECDSA_SIG_free(s);
    }
    EC_KEY_free(k);
    double tp_mean = 0;
    for (double x : tp) tp_mean += x;
    tp_mean /= tp.empty() ? 1 : (double)tp.size();
    std::printf("{\"mode\": \"sign\", \"calls\": %d, \"gpu_rfc6979_p50_ms\": %.4f, \"gpu_rfc6979_p99_ms\": %.4f, "
                "\"gpu_pooled_p50_ms\": %.4f, \"gpu_pooled_p99_ms\": %.4f, \"gpu_pooled_mean_ms\": %.4f, "
                "\"openssl_1core_p50_ms\": %.4f, \"openssl_1core_p99_ms\": %.4f, \"failures\": %d}\n",
                calls, pct(tg, 50) / 1e3, pct(tg, 99) / 1e3, pct(tp, 50) / 1e3, pct(tp, 99) / 1e3, tp_mean / 1e3,
                pct(tc, 50) / 1e3, pct(tc, 99) / 1e3, bad);
    sbft_signer_free(sg);
    sbft_gv_destroy(ctx);
    return bad ? 2 : 0;
}

static int proposal_cpu(int requests, int decisions, int threads) {
    auto tup = cpu_tuples(requests, 64 + 150, 256 + 150);  // body = ids + payload + key
    std::atomic<int> bad{0};
    const int nt = std::max(1, threads);
    // one pool; per decision the workers pull request indices from that decision's counter
    std::unique_ptr<std::atomic<int>[]> next(new std::atomic<int>[decisions]);
    for (int g = 0; g < decisions; ++g) next[g] = 0;
    auto t = fan_out(nt, decisions, [&](size_t, int g) {
        for (;;) {
            const int k = next[g].fetch_add(1);
            if (k >= requests) break;
            if (!cpu_verify(tup[k])) bad++;
        }
    });
    std::printf("{\"mode\": \"proposal-cpu\", \"requests\": %d, \"decisions\": %d, \"threads\": %d, "
                "\"p50_ms\": %.4f, \"p99_ms\": %.4f, \"rejected\": %d}\n",
                requests, decisions, nt, pct(t, 50) / 1e3, pct(t, 99) / 1e3, bad.load());
    return 0;
}

// proposal-gpu REQUESTS DECISIONS: VerifyProposal through the C ABI on proposals of REQUESTS
// signed requests (distinct client keys), each decision rotating over: the honest proposal
// (generic path), one with a bad signature at a varying index, one truncated (malformed), and
// the honest one again with every client registered (keyed path). Checks every verdict, count
// and reported index; reports the honest generic call's p50/p99.
// proposal-phases REQUESTS CALLS REGISTERED: where a VerifyProposal call's time goes (VERDICT r05
// #4). The engine's SBFT_VP_TRACE split of every call (submit | parse | copy wait | staging |
// launch | the rest: kernel, verdicts, return), captured from its stderr, and HIP events around
// the call's one kernel (sbft_gv_kernel_timing: p256_verify_half_kernel<true> generic, the keyed
// lanes kernel with the clients registered). Reports medians over all calls and over the calls
// above the 95th percentile (the tail), with the kernel's time in each.
static int proposal_phases(int requests, int calls, int registered) {
    setenv("SBFT_VP_TRACE", "1", 1);  // before the engine's first VerifyProposal reads it
    char tpath[] = "/tmp/sbft_vp_traceXXXXXX";
    const int tfd = mkstemp(tpath);
    if (tfd < 0) return 1;
    std::fflush(stderr);
    const int saved = dup(2);
    dup2(tfd, 2);
    sbft_gv_ctx* ctx = nullptr;
    if (sbft_gv_init(nullptr, &ctx)) {
        dup2(saved, 2);
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    sbft_verifier* v = sbft_verifier_new(ctx, 0);
    std::vector<uint8_t> payload(4), keys;
    uint32_t cnt = (uint32_t)requests;
    std::memcpy(payload.data(), &cnt, 4);
    for (int i = 0; i < requests; ++i) {
        uint8_t d[32], pub[65], buf[1024];
        priv_of(50'000 + i, d);
        sbft_signer* c = sbft_signer_new(ctx, 1, d);
        sbft_signer_public_key(c, pub);
        keys.insert(keys.end(), pub, pub + 65);
        std::string body(64 + i % 193, (char)('a' + i % 26));
        const std::string cid = "client" + std::to_string(i), rid = "tx" + std::to_string(i);
        const int64_t len = sbft_make_request(c, cid.c_str(), rid.c_str(), (const uint8_t*)body.data(), body.size(), buf,
                                              sizeof buf);
        sbft_signer_free(c);
        if (len <= 0) return 3;
        const uint32_t l = (uint32_t)len;
        payload.insert(payload.end(), (const uint8_t*)&l, (const uint8_t*)&l + 4);
        payload.insert(payload.end(), buf, buf + len);
    }
    if (registered) sbft_verifier_add_clients(v, keys.data(), (size_t)requests);
    std::vector<char> infos((size_t)requests * 40);
    char err[256];
    sbft_proposal p{payload.data(), payload.size(), (const uint8_t*)"h", 1, (const uint8_t*)"m", 1, 0};
    int wrong = 0;
    for (int g = 0; g < 5; ++g) {  // warm-up
        size_t count = 0;
        int64_t bad = -1;
        wrong += sbft_verifier_verify_proposal(v, &p, infos.data(), infos.size(), &count, &bad, err, sizeof err) != 0;
    }
    (void)sbft_gv_kernel_timing(ctx, 1);
    uint64_t nl = 0;
    double kms = 0;
    (void)sbft_gv_kernel_time(ctx, &nl, &kms);
    std::fflush(stderr);
    const off_t mark = lseek(tfd, 0, SEEK_END);
    std::vector<double> tot, kern;
    for (int g = 0; g < calls; ++g) {
        size_t count = 0;
        int64_t bad = -1;
        const auto t0 = Clock::now();
        const int rc = sbft_verifier_verify_proposal(v, &p, infos.data(), infos.size(), &count, &bad, err, sizeof err);
        tot.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
        wrong += rc != 0 || count != (size_t)requests;
        (void)sbft_gv_kernel_time(ctx, &nl, &kms);
        kern.push_back(nl == 1 ? kms * 1e3 : -1.0);
    }
    std::fflush(stderr);
    dup2(saved, 2);
    // the calls' trace lines, in call order (the engine prints one per call)
    std::vector<std::array<double, 8>> ph;  // + the payload copy's start and return (from the call's start)
    {
        FILE* f = std::fopen(tpath, "r");
        if (f) {
            std::fseek(f, (long)mark, SEEK_SET);
            char line[512];
            while (std::fgets(line, sizeof line, f)) {
                int a = 0;
                std::array<double, 8> x{};
                x[6] = x[7] = -1;
                if (std::sscanf(line, "vp async=%d submit=%lf parse=%lf copy_wait_sync=%lf stage=%lf launch=%lf rest=%lf",
                                &a, &x[0], &x[1], &x[2], &x[3], &x[4], &x[5]) == 7) {
                    const char* cp = std::strstr(line, "copy=");
                    if (cp) (void)std::sscanf(cp, "copy=%lf,%lf", &x[6], &x[7]);
                    ph.push_back(x);
                }
            }
            std::fclose(f);
        }
        unlink(tpath);
        close(tfd);
    }
    const double p95 = pct(tot, 95);
    auto med = [&](bool tail, int field) {  // field -1: the kernel
        std::vector<double> v;
        for (size_t i = 0; i < tot.size(); ++i)
            if (!tail || tot[i] > p95) {
                if (field < 0) {
                    if (kern[i] >= 0) v.push_back(kern[i]);
                } else if (i < ph.size() && ph[i][field] >= 0) {
                    v.push_back(ph[i][field]);
                }
            }
        return pct(v, 50);
    };
    auto group = [&](bool tail) {
        char b[512];
        std::snprintf(b, sizeof b,
                      "{\"submit_us\": %.1f, \"parse_us\": %.1f, \"copy_wait_us\": %.1f, \"stage_us\": %.1f, "
                      "\"launch_us\": %.1f, \"kernel_verdicts_return_us\": %.1f, \"kernel_us\": %.1f, "
                      "\"copy_start_us\": %.1f, \"copy_return_us\": %.1f}",
                      med(tail, 0), med(tail, 1), med(tail, 2), med(tail, 3), med(tail, 4), med(tail, 5), med(tail, -1),
                      med(tail, 6), med(tail, 7));
        return std::string(b);
    };
    std::printf("{\"mode\": \"proposal-phases\", \"requests\": %d, \"calls\": %d, \"registered\": %d, "
                "\"p50_ms\": %.4f, \"p95_ms\": %.4f, \"p99_ms\": %.4f, \"kernel_us_p50\": %.1f, "
                "\"kernel_us_p99\": %.1f, \"traced_calls\": %zu, \"all_p50\": %s, \"tail_above_p95\": %s, "
                "\"wrong_verdicts\": %d}\n",
                requests, calls, registered, pct(tot, 50) / 1e3, p95 / 1e3, pct(tot, 99) / 1e3, pct(kern, 50),
                pct(kern, 99), ph.size(), group(false).c_str(), group(true).c_str(), wrong);
    sbft_verifier_free(v);
    sbft_gv_destroy(ctx);
    return wrong ? 2 : 0;
}

static int proposal_gpu(int requests, int decisions) {
    sbft_gv_ctx* ctx = nullptr;
    if (sbft_gv_init(nullptr, &ctx)) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    sbft_verifier* gen = sbft_verifier_new(ctx, 0);
    sbft_verifier* reg = sbft_verifier_new(ctx, 0);
    std::vector<uint8_t> payload(4), keys;
    std::vector<size_t> sig_at;  // offset of each request's signature inside payload
    uint32_t cnt = (uint32_t)requests;
    std::memcpy(payload.data(), &cnt, 4);
    for (int i = 0; i < requests; ++i) {
        uint8_t d[32], pub[65], buf[1024];
        priv_of(50'000 + i, d);
        sbft_signer* c = sbft_signer_new(ctx, 1, d);
        sbft_signer_public_key(c, pub);
        keys.insert(keys.end(), pub, pub + 65);
        std::string body(64 + i % 193, (char)('a' + i % 26));
        const std::string cid = "client" + std::to_string(i), rid = "tx" + std::to_string(i);
        const int64_t len = sbft_make_request(c, cid.c_str(), rid.c_str(), (const uint8_t*)body.data(), body.size(), buf,
                                              sizeof buf);
        sbft_signer_free(c);
        if (len <= 0) return 3;
        const uint32_t l = (uint32_t)len;
        payload.insert(payload.end(), (const uint8_t*)&l, (const uint8_t*)&l + 4);
        payload.insert(payload.end(), buf, buf + len);
        sig_at.push_back(payload.size() - 64);
    }
    sbft_verifier_add_clients(reg, keys.data(), (size_t)requests);
    std::vector<char> infos((size_t)requests * 40);
    std::vector<double> t;
    int wrong = 0;
    char err[256];
    auto call = [&](sbft_verifier* v, const std::vector<uint8_t>& pl, size_t& count, int64_t& bad) {
        sbft_proposal p{pl.data(), pl.size(), (const uint8_t*)"h", 1, (const uint8_t*)"m", 1, 0};
        return sbft_verifier_verify_proposal(v, &p, infos.data(), infos.size(), &count, &bad, err, sizeof err);
    };
    for (int g = -3; g < decisions; ++g) {
        size_t count = 0;
        int64_t bad = -1;
        const auto t0 = Clock::now();
        int rc = call(gen, payload, count, bad);
        const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        if (g >= 0) t.push_back(us);
        wrong += rc != 0 || count != (size_t)requests;
        const int k = (g + 3) * 7919 % requests;
        std::vector<uint8_t> pb = payload;
        pb[sig_at[k] + 5] ^= 0x40;
        rc = call(gen, pb, count, bad);
        wrong += rc != SBFT_V_EVERIFY || bad != k;
        pb.assign(payload.begin(), payload.end() - 1 - (g + 3) % 50);
        rc = call(gen, pb, count, bad);
        wrong += rc != SBFT_V_EFORMAT;
        rc = call(reg, payload, count, bad);
        wrong += rc != 0 || count != (size_t)requests;
    }
    std::printf("{\"mode\": \"proposal-gpu\", \"requests\": %d, \"decisions\": %d, \"p50_ms\": %.4f, "
                "\"p99_ms\": %.4f, \"wrong_verdicts\": %d}\n",
                requests, decisions, pct(t, 50) / 1e3, pct(t, 99) / 1e3, wrong);
    sbft_verifier_free(reg);
    sbft_verifier_free(gen);
    sbft_gv_destroy(ctx);
    return wrong ? 2 : 0;
}

// parse-cpu REQUESTS ITERS: RequestsFromProposal on a parse-only verifier (no GPU): a proposal of
// REQUESTS format-only requests (garbage keys and signatures), parsed ITERS times -- the
// 3-thread parse (verifier.cpp parse_payload_par and its helper pool) from several caller threads
// at once, plus truncated copies. A race detector's workload, not a measurement.
static int parse_cpu(int requests, int iters) {
    std::vector<uint8_t> pl(4);
    const uint32_t cnt = (uint32_t)requests;
    std::memcpy(pl.data(), &cnt, 4);
    for (int i = 0; i < requests; ++i) {
        const std::string cid = "client" + std::to_string(i), rid = "tx" + std::to_string(i);
        std::vector<uint8_t> r = {'S', 'B', 'R', '1'};
        auto u = [&](uint64_t v, int n) {
            for (int k = 0; k < n; ++k) r.push_back((uint8_t)(v >> (8 * k)));
        };
        u(cid.size(), 2);
        r.insert(r.end(), cid.begin(), cid.end());
        u(rid.size(), 2);
        r.insert(r.end(), rid.begin(), rid.end());
        const size_t body = 64 + i % 193;
        u(body, 4);
        r.insert(r.end(), body, (uint8_t)i);
        r.push_back(0x04);
        r.insert(r.end(), 64 + 64, 0x5a);
        const uint32_t l = (uint32_t)r.size();
        pl.insert(pl.end(), (const uint8_t*)&l, (const uint8_t*)&l + 4);
        pl.insert(pl.end(), r.begin(), r.end());
    }
    sbft_verifier* v = sbft_verifier_new(nullptr, 0);
    std::atomic<int> wrong{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 3; ++t)
        th.emplace_back([&, t] {
            std::vector<char> infos((size_t)requests * 24);
            for (int it = 0; it < iters; ++it) {
                const bool cut = (it + t) % 4 == 3;
                sbft_proposal p{pl.data(), pl.size() - (cut ? 1 + it % 7 : 0), (const uint8_t*)"h", 1,
                                (const uint8_t*)"m", 1, 0};
                size_t count = 0;
                const int rc = sbft_verifier_requests_from_proposal(v, &p, infos.data(), infos.size(), &count);
                if (cut ? rc != SBFT_V_EFORMAT : (rc != 0 || count != (size_t)requests)) wrong++;
            }
        });
    for (auto& x : th) x.join();
    sbft_verifier_free(v);
    std::printf("{\"mode\": \"parse-cpu\", \"requests\": %d, \"iters\": %d, \"wrong\": %d}\n", requests, iters,
                wrong.load());
    return wrong.load() ? 2 : 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s quorum-gpu|quorum-batch|quorum-hook|quorum-pipe|sign|quorum-cpu|quorum-vote-cpu|proposal-cpu|proposal-gpu|parse-cpu ...\n", argv[0]);
        return 1;
    }
    const std::string mode = argv[1];
    auto arg = [&](int i, int def) { return argc > i ? std::atoi(argv[i]) : def; };
    if (mode == "quorum-gpu") return quorum_gpu(arg(2, 66), arg(3, 200), arg(4, 0), arg(5, 0));
    if (mode == "quorum-batch") return quorum_batch(arg(2, 67), arg(3, 200));
    if (mode == "quorum-hook") return quorum_hook(arg(2, 67), arg(3, 66), arg(4, 200), arg(5, 2));
    if (mode == "sign") return sign_both(arg(2, 200));
    if (mode == "quorum-pipe") {
        const std::string b = argc > 4 ? argv[4] : "gpu";
        return quorum_pipe(arg(2, 2), arg(3, 200), b != "cpu" && b != "cpu-batched", b == "cpu-batched");
    }
    if (mode == "quorum-cpu") return quorum_cpu(arg(2, 66), arg(3, 200), arg(4, 66));
    if (mode == "quorum-vote-cpu") return quorum_vote_cpu(arg(2, 67), arg(3, 66), arg(4, 200), arg(5, 67));
    if (mode == "proposal-cpu") return proposal_cpu(arg(2, 10000), arg(3, 20), arg(4, 16));
    if (mode == "proposal-gpu") return proposal_gpu(arg(2, 3000), arg(3, 20));
    if (mode == "proposal-phases") return proposal_phases(arg(2, 10000), arg(3, 200), arg(4, 0));
    if (mode == "parse-cpu") return parse_cpu(arg(2, 6000), arg(3, 50));
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 1;
}
