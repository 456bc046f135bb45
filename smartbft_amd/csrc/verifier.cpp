// verifier.cpp — plugin-level mirror of SmartBFT's api.Verifier and api.Signer
// (pkg/api/dependencies.go:46-71) on top of the GPU engine (include/sbft_verifier.h).
//
// Every signature check goes through the engine: a proposal is ONE fused launch (SHA-256 of
// every request body + P-256 verify, view.go:555), a batch of consenter signatures is ONE
// launch (view.go:631, :834). The host side only parses formats, checks bindings and builds
// the structure-of-arrays batches; there is no CPU verification path.
#include "../../include/sbft_verifier.h"
#include "engine_internal.h"
#include "modn_host.hpp"

#include <pthread.h>
#include <cpuid.h>
#include <immintrin.h>

#include <array>
#include <atomic>
#include <thread>
#include <functional>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include <climits>
#include <linux/futex.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/random.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace {

// ------------------------------------------------------------------ SHA-256 (host)
const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// SHA-256 compression with the x86 SHA extensions (Proposal.Digest hashes whole proposals on
// the host: 3.2 MB at 10k requests; Go's crypto/sha256 uses the same instructions). Two rounds
// per sha256rnds2; state kept as ABEF / CDGH; message schedule by sha256msg1/msg2:
//   X_g = msg2(msg1(X_{g-4}, X_{g-3}) + alignr(X_{g-1}, X_{g-2}, 4), X_{g-1}), X_g = W[4g..4g+3].
__attribute__((target("sha,sse4.1"))) void sha256_blocks_ni(uint32_t h[8], const uint8_t* p, size_t nblk) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[0]), 0xB1);  // C D A B
    __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&h[4]), 0x1B); // E F G H
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                         // A B E F
    s1 = _mm_blend_epi16(s1, t, 0xF0);                                              // C D G H
    for (; nblk; --nblk, p += 64) {
        const __m128i save0 = s0, save1 = s1;
        __m128i x[4];
        for (int g = 0; g < 16; ++g) {
            __m128i m;
            if (g < 4) {
                m = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * g)), bswap);
            } else {
                m = _mm_sha256msg1_epu32(x[g & 3], x[(g + 1) & 3]);                    // X_{g-4}, X_{g-3}
                m = _mm_add_epi32(m, _mm_alignr_epi8(x[(g + 3) & 3], x[(g + 2) & 3], 4)); // X_{g-1}, X_{g-2}
                m = _mm_sha256msg2_epu32(m, x[(g + 3) & 3]);
            }
            x[g & 3] = m;
            __m128i k = _mm_add_epi32(m, _mm_loadu_si128((const __m128i*)&K256[4 * g]));
            s1 = _mm_sha256rnds2_epu32(s1, s0, k);
            k = _mm_shuffle_epi32(k, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, k);
        }
        s0 = _mm_add_epi32(s0, save0);
        s1 = _mm_add_epi32(s1, save1);
    }
    t = _mm_shuffle_epi32(s0, 0x1B);    // F E B A
    s1 = _mm_shuffle_epi32(s1, 0xB1);   // D C H G
    s0 = _mm_blend_epi16(t, s1, 0xF0);  // D C B A
    s1 = _mm_alignr_epi8(s1, t, 8);     // H G F E
    _mm_storeu_si128((__m128i*)&h[0], s0);
    _mm_storeu_si128((__m128i*)&h[4], s1);
}

bool cpu_has_sha() {
    static const bool has = [] {
        if (std::getenv("SBFT_NO_SHANI")) return false;  // tests exercise the portable path too
        unsigned a, b, c, d;
        if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
        const bool sha = (b >> 29) & 1;
        if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
        return sha && ((c >> 19) & 1);  // SSE4.1
    }();
    return has;
}

struct Sha256 {
    uint32_t h[8];
    uint8_t buf[64];
    uint64_t total = 0;
    size_t fill = 0;
    Sha256() {
        static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        std::memcpy(h, iv, sizeof h);
    }
    void block(const uint8_t* p) { blocks(p, 1); }
    void blocks(const uint8_t* p, size_t nblk) {
        if (cpu_has_sha()) {
            sha256_blocks_ni(h, p, nblk);
            return;
        }
        for (; nblk; --nblk, p += 64) block_portable(p);
    }
    void block_portable(const uint8_t* p) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i)
            w[i] = w[i - 16] + (rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
                   (rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10));
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t t1 = k + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
    }
    void update(const uint8_t* p, size_t n) {
        total += n;
        while (n) {
            if (fill == 0 && n >= 64) {
                const size_t nb = n / 64;
                blocks(p, nb);
                p += 64 * nb;
                n -= 64 * nb;
                continue;
            }
            const size_t take = std::min(n, 64 - fill);
            std::memcpy(buf + fill, p, take);
            fill += take;
            p += take;
            n -= take;
            if (fill == 64) {
                block(buf);
                fill = 0;
            }
        }
    }
    void final(uint8_t out[32]) {
        const uint64_t bits = total * 8;
        const uint8_t pad = 0x80;
        update(&pad, 1);
        const uint8_t zero = 0;
        while (fill != 56) update(&zero, 1);
        uint8_t lenb[8];
        for (int i = 0; i < 8; ++i) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(lenb, 8);
        for (int i = 0; i < 8; ++i) {
            out[4 * i] = (uint8_t)(h[i] >> 24);
            out[4 * i + 1] = (uint8_t)(h[i] >> 16);
            out[4 * i + 2] = (uint8_t)(h[i] >> 8);
            out[4 * i + 3] = (uint8_t)h[i];
        }
    }
};

void sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
    Sha256 s;
    s.update(p, n);
    s.final(out);
}

// HMAC-SHA-256 over the concatenation of up to four parts (RFC 2104).
void hmac_sha256(const uint8_t key[32], std::initializer_list<std::pair<const uint8_t*, size_t>> parts,
                 uint8_t out[32]) {
    uint8_t ipad[64], opad[64];
    for (int i = 0; i < 64; ++i) {
        const uint8_t k = i < 32 ? key[i] : 0;
        ipad[i] = k ^ 0x36;
        opad[i] = k ^ 0x5c;
    }
    uint8_t inner[32];
    Sha256 a;
    a.update(ipad, 64);
    for (auto& pr : parts) a.update(pr.first, pr.second);
    a.final(inner);
    Sha256 b;
    b.update(opad, 64);
    b.update(inner, 32);
    b.final(out);
}

const uint8_t N_BE[32] = {0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x00, 0xff, 0xff, 0xff,
                          0xff, 0xff, 0xff, 0xff, 0xff, 0xbc, 0xe6, 0xfa, 0xad, 0xa7, 0x17,
                          0x9e, 0x84, 0xf3, 0xb9, 0xca, 0xc2, 0xfc, 0x63, 0x25, 0x51};

int cmp_be32(const uint8_t* a, const uint8_t* b) { return std::memcmp(a, b, 32); }
bool is_zero32(const uint8_t* a) {
    for (int i = 0; i < 32; ++i)
        if (a[i]) return false;
    return true;
}
void sub_be32(uint8_t* a, const uint8_t* b) {  // a -= b (mod 2^256)
    int borrow = 0;
    for (int i = 31; i >= 0; --i) {
        const int d = (int)a[i] - b[i] - borrow;
        a[i] = (uint8_t)d;
        borrow = d < 0;
    }
}

// RFC 6979 3.2 deterministic nonce for P-256 with HMAC-SHA-256 (qlen = hlen = 256).
// `attempt` > 0 continues the generator (step h.3) past nonces that produced r or s = 0.
void rfc6979_nonce(const uint8_t x[32], const uint8_t h1[32], int attempt, uint8_t k_out[32]) {
    uint8_t h[32];
    std::memcpy(h, h1, 32);
    if (cmp_be32(h, N_BE) >= 0) sub_be32(h, N_BE);  // bits2octets: bits2int(h1) mod q
    uint8_t V[32], K[32];
    std::memset(V, 0x01, 32);
    std::memset(K, 0x00, 32);
    const uint8_t z0 = 0x00, z1 = 0x01;
    hmac_sha256(K, {{V, 32}, {&z0, 1}, {x, 32}, {h, 32}}, K);
    hmac_sha256(K, {{V, 32}}, V);
    hmac_sha256(K, {{V, 32}, {&z1, 1}, {x, 32}, {h, 32}}, K);
    hmac_sha256(K, {{V, 32}}, V);
    for (int found = 0;;) {
        hmac_sha256(K, {{V, 32}}, V);
        if (!is_zero32(V) && cmp_be32(V, N_BE) < 0 && found++ == attempt) {
            std::memcpy(k_out, V, 32);
            return;
        }
        hmac_sha256(K, {{V, 32}, {&z0, 1}}, K);
        hmac_sha256(K, {{V, 32}}, V);
    }
}

// ------------------------------------------------------------------ ASN.1 DER (Digest)
void der_len(std::vector<uint8_t>& o, size_t n) {
    if (n < 0x80) {
        o.push_back((uint8_t)n);
        return;
    }
    uint8_t tmp[8];
    int k = 0;
    while (n) {
        tmp[k++] = (uint8_t)(n & 0xff);
        n >>= 8;
    }
    o.push_back((uint8_t)(0x80 | k));
    while (k) o.push_back(tmp[--k]);
}
void der_int64(std::vector<uint8_t>& o, int64_t v) {
    // minimal two's complement, as Go encoding/asn1 marshals int64
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)((uint64_t)v >> (56 - 8 * i));
    int start = 0;
    while (start < 7 && ((b[start] == 0x00 && !(b[start + 1] & 0x80)) || (b[start] == 0xff && (b[start + 1] & 0x80))))
        ++start;
    o.push_back(0x02);
    der_len(o, 8 - start);
    o.insert(o.end(), b + start, b + 8);
}

// ------------------------------------------------------------------ formats
struct Reader {
    const uint8_t* p;
    size_t n, pos = 0;
    bool take(size_t k, const uint8_t*& out) {
        if (n - pos < k) return false;
        out = p + pos;
        pos += k;
        return true;
    }
    bool u16(uint32_t& v) {
        const uint8_t* q;
        if (!take(2, q)) return false;
        v = (uint32_t)q[0] | (uint32_t)q[1] << 8;
        return true;
    }
    bool u32(uint32_t& v) {
        const uint8_t* q;
        if (!take(4, q)) return false;
        v = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
        return true;
    }
};

struct Req {
    // views into the request bytes (borrowed for the call; no per-request allocation)
    struct Str {
        const char* p = "";
        int n = 0;
    } client_id, req_id;
    size_t body_off = 0, body_len = 0;  // relative to the buffer handed to parse_request
    const uint8_t* pub = nullptr;       // 65 bytes SEC1
    const uint8_t* sig = nullptr;       // 64 bytes r||s
};

// Per-thread scratch for the proposal paths: a 10k-request proposal needs ~0.8 MB of
// request views and offsets, and fresh vectors of that size are mmap'd and page-faulted on
// every call (~0.1-0.25 ms); reused ones keep their pages.
struct ProposalScratch {
    std::vector<Req> reqs;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<uint32_t> kid;  // registered client key ids (VerifyProposal with clients registered)
    std::vector<uint8_t> ok;
};
ProposalScratch& proposal_scratch() {
    thread_local ProposalScratch s;
    return s;
}

// A one-shot "results are published" flag for the followers of a coalesced batch. They spin
// briefly, then sleep on a futex; the leader's wake-up does not make them re-acquire a mutex
// one after another (a condition variable's notify_all does: ~3-4 us per follower, 0.25 ms
// for a 66-vote quorum).
// The wake-up is a tree: set() wakes two sleepers and every sleeper that wakes wakes two more.
// One FUTEX_WAKE of all 65 followers of a commit quorum runs their 65 wake-ups one after
// another inside the leader's system call (~80 us); the tree spreads them over the cores.
struct DoneFlag {
    std::atomic<int> v{0};
    void wake2() { syscall(SYS_futex, reinterpret_cast<int*>(&v), FUTEX_WAKE_PRIVATE, 2, nullptr, nullptr, 0); }
    void set() {
        v.store(1, std::memory_order_release);
        wake2();
    }
    // spin: pause iterations before sleeping (0 when the wait is known to be long: a follower
    // spinning on a busy host only delays the callers that still have to arrive)
    void wait(int spin = 256) {
        for (int i = 0; i < spin; ++i) {
            if (v.load(std::memory_order_acquire)) return;
            __builtin_ia32_pause();
        }
        bool slept = false;
        while (!v.load(std::memory_order_acquire)) {
            syscall(SYS_futex, reinterpret_cast<int*>(&v), FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
            slept = true;
        }
        if (slept) wake2();
    }
};

const char* REQ_MAGIC = "SBR1";
const char* MSG_MAGIC = "SBC1";

// true if any of the n bytes at q is 0. SWAR over 8-byte words; the caller guarantees 8
// readable bytes past q + n (an id is followed by at least the 65-byte key and 64-byte
// signature), so the last word is loaded whole and its excess bytes masked off. A memchr
// call per id cost ~4 ns x 20k ids on the proposal-parse critical path.
inline bool has_nul(const uint8_t* q, size_t n) {
    for (size_t k = 0; k < n; k += 8) {
        uint64_t w;
        std::memcpy(&w, q + k, 8);
        const size_t left = n - k;
        if (left < 8) w |= ~0ull << (8 * left);  // bytes past the id count as non-zero
        if ((w - 0x0101010101010101ull) & ~w & 0x8080808080808080ull) return true;
    }
    return false;
}

bool parse_request(const uint8_t* d, size_t len, size_t base, Req& out) {
    Reader r{d, len};
    const uint8_t* q;
    uint32_t a, b, c;
    if (!r.take(4, q) || std::memcmp(q, REQ_MAGIC, 4)) return false;
    // ids are returned as NUL-terminated "client_id\0id\0" records (write_info): an id holding
    // a NUL would shift every later record, so such a request is malformed
    if (!r.u16(a) || !r.take(a, q)) return false;
    out.client_id = {(const char*)q, (int)a};
    if (!r.u16(b) || !r.take(b, q)) return false;
    out.req_id = {(const char*)q, (int)b};
    if (!r.u32(c) || !r.take(c, q)) return false;
    if (!r.take(65, out.pub)) return false;
    // the ids are followed by >= 4 + 65 readable bytes here: the whole-word reads stay inside
    if (has_nul((const uint8_t*)out.client_id.p, a) || has_nul((const uint8_t*)out.req_id.p, b)) return false;
    out.body_off = base;
    out.body_len = r.pos;
    if (!r.take(64, out.sig) || r.pos != len) return false;
    return true;
}

// on_req(i) runs as soon as request i is parsed (its memory accesses then overlap the walk's
// dependent loads)
template <class F>
bool parse_payload(const uint8_t* p, size_t len, std::vector<Req>& out, F&& on_req) {
    Reader r{p, len};
    uint32_t count;
    if (!r.u32(count)) return false;
    if (count > len / 4) return false;
    out.resize(count);
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t l;
        const uint8_t* q;
        __builtin_prefetch(p + r.pos + 2048);  // keep the chain of length prefixes in L1
        if (!r.u32(l)) return false;
        const size_t at = r.pos;
        if (!r.take(l, q)) return false;
        if (!parse_request(q, l, at, out[i])) return false;
        on_req(i);
    }
    return r.pos == len;
}
bool parse_payload(const uint8_t* p, size_t len, std::vector<Req>& out) {
    return parse_payload(p, len, out, [](uint32_t) {});
}

// The chain of length prefixes alone, VerifyProposal's part of the parse before its launch:
// each request's body offset and length (the request without its 64-byte signature). Every
// request must be at least as long as the smallest well-formed one (magic, two empty ids, an
// empty payload, key, signature), so the kernel's reads of the body's last 64 bytes (Q) and of
// the signature stay inside it. A payload this rejects, parse_payload rejects too; one it
// accepts can still be malformed inside a request (the full parse decides, during the verify).
constexpr uint32_t kMinRequest = 4 + 2 + 2 + 4 + 65 + 64;
bool walk_payload(const uint8_t* p, size_t len, std::vector<uint64_t>& off, std::vector<uint32_t>& blen) {
    Reader r{p, len};
    uint32_t count;
    if (!r.u32(count) || count > len / 4) return false;
    off.resize(count);
    blen.resize(count);
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t l;
        const uint8_t* q;
        __builtin_prefetch(p + r.pos + 2048);
        if (!r.u32(l) || l < kMinRequest) return false;
        const size_t at = r.pos;
        if (!r.take(l, q)) return false;
        off[i] = at;
        blen[i] = l - 64;
    }
    return r.pos == len;
}

// A process-wide pool of warm helper threads for the proposal parse. run(T, f) runs f(0) on the
// caller and f(1..T-1) on helpers, and returns when all are done. A helper spins (yielding) for
// ~0.5 ms after a job, so back-to-back proposals find it awake; then it sleeps. If another
// caller holds the pool, run() returns false and the caller parses alone.
struct ParsePool {
    static constexpr int kMax = 4;  // threads per parse, the caller included
    std::mutex busy;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> gen{0};
    std::atomic<int> left{0};
    std::function<void(int)> job;
    std::thread th[kMax - 1];
    bool started = false;

    void worker(int t) {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            const auto t0 = std::chrono::steady_clock::now();
            while ((g = gen.load(std::memory_order_acquire)) == seen &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(500))
                std::this_thread::yield();
            if (g == seen) {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return gen.load(std::memory_order_acquire) != seen; });
                g = gen.load(std::memory_order_acquire);
            }
            seen = g;
            if (t < (int)(g & 0xff)) {  // the job's thread count rides in the generation's low byte
                job(t);
                left.fetch_sub(1, std::memory_order_acq_rel);
            }
        }
    }
    bool run(int T, const std::function<void(int)>& f) {
        if (T <= 1) {
            f(0);
            return true;
        }
        std::unique_lock<std::mutex> b(busy, std::try_to_lock);
        if (!b.owns_lock()) return false;
        T = std::min(T, kMax);
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!started) {
                for (int t = 1; t < kMax; ++t) {
                    th[t - 1] = std::thread([this, t] {
                        pthread_setname_np(pthread_self(), "sbft-parse");
                        worker(t);
                    });
                    th[t - 1].detach();  // process-lifetime helpers
                }
                started = true;
            }
            job = f;
            left.store(T - 1, std::memory_order_release);
            gen.store(((gen.load() >> 8) + 1) << 8 | (uint64_t)T, std::memory_order_release);
        }
        cv.notify_all();
        f(0);
        while (left.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
        return true;
    }
};
ParsePool& parse_pool() {
    static ParsePool* pool = new ParsePool();  // never destroyed: its threads live with the process
    return *pool;
}

// The first position q >= from (q < to) that can start a request of a payload p[0, len): a u32
// length l at q with q + 4 + l <= len and a request that parses at q + 4. A candidate only: the
// walk that reaches it decides whether it is a real boundary.
// The search gives up after kCandidateWindow bytes: the split only pays for many small requests,
// and a bounded scan keeps a payload crafted full of false "SBR1" headers cheap.
constexpr size_t kCandidateWindow = 4096;
size_t payload_candidate(const uint8_t* p, size_t len, size_t from, size_t to) {
    to = std::min(to, from + kCandidateWindow);
    for (size_t q = from; q + 8 <= len && q < to; ++q) {
        if (p[q + 4] != 'S' || std::memcmp(p + q + 4, REQ_MAGIC, 4) != 0) continue;
        const uint32_t l = (uint32_t)p[q] | (uint32_t)p[q + 1] << 8 | (uint32_t)p[q + 2] << 16 | (uint32_t)p[q + 3] << 24;
        Req tmp;
        if (l <= len - q - 4 && parse_request(p + q + 4, l, q + 4, tmp)) return q;
    }
    return SIZE_MAX;
}

// parse_payload over T threads, in two phases. sized(n) runs on the caller once the request count
// is known (before any range call).
//   walk : thread t follows the chain of length prefixes from its start (the payload's first
//          request for t = 0; for t > 0 the first candidate boundary at or after t/T of the
//          payload) up to the next thread's candidate, recording request positions. This chain of
//          dependent loads is most of a sequential parse (a cache miss per request).
//   join : thread t's walk is the payload's own chain iff thread t-1's ended exactly on its
//          start. A false candidate (bytes that look like a request inside some payload) breaks
//          the joint: the caller walks on from thread t-1's end alone. The walk must end at len
//          with exactly `count` requests, as the sequential parse requires.
//   parse: each thread parses its requests into their final slots, then calls range(b, e) on
//          them (the caller's per-request work: offsets, key checks, registry lookups).
// Returns false for a malformed payload (the same payloads parse_payload rejects). Falls back to
// the sequential parse for small payloads or when the pool is busy.
template <class Sized, class Range>
bool parse_payload_par(const uint8_t* p, size_t len, std::vector<Req>& out, int T, Sized&& sized, Range&& range) {
    if (len < 4) return false;
    const uint32_t count = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
    if (count > len / 4) return false;
    if (T > 1 && (count < 2048 || len < ((size_t)256 << 10) || len > 0xffffffffu)) T = 1;
    T = std::min(T, ParsePool::kMax);
    if (T <= 1) {
        if (!parse_payload(p, len, out)) return false;
        sized(out.size());
        range((uint32_t)0, (uint32_t)out.size());
        return true;
    }
    struct Part {
        size_t start = SIZE_MAX, limit = 0, end = 0;
        std::vector<uint32_t> pos;
        bool bad = false;
        uint32_t base = 0;
        bool used = false;
    };
    thread_local std::vector<Part> parts_tl;
    std::vector<Part>& parts = parts_tl;
    parts.resize(T);
    for (auto& x : parts) {
        x.pos.clear();
        x.start = SIZE_MAX;
        x.end = 0;
        x.bad = false;
        x.used = false;
    }
    std::vector<size_t> cut(T + 1);
    for (int t = 0; t <= T; ++t) cut[t] = t == 0 ? 4 : t == T ? len : 4 + (len - 4) * (size_t)t / (size_t)T;
    std::atomic<bool> bad_parse{false};
    auto walk = [&](int t) {
        Part& x = parts[t];
        x.start = t == 0 ? 4 : payload_candidate(p, len, cut[t], cut[t + 1]);
        size_t nxt = len;  // the next thread's start (or the payload's end)
        for (int u = t + 1; u < T; ++u) {
            const size_t c = payload_candidate(p, len, cut[u], cut[u + 1]);
            if (c != SIZE_MAX) {
                nxt = c;
                break;
            }
        }
        x.limit = nxt;
        if (x.start == SIZE_MAX) return;
        x.pos.reserve(count / T + 64);
        size_t pos = x.start;
        while (pos < nxt) {
            if (len - pos < 4) {
                x.bad = true;
                break;
            }
            __builtin_prefetch(p + pos + 2048);
            const uint32_t l = (uint32_t)p[pos] | (uint32_t)p[pos + 1] << 8 | (uint32_t)p[pos + 2] << 16 |
                               (uint32_t)p[pos + 3] << 24;
            if (l > len - pos - 4) {
                x.bad = true;
                break;
            }
            x.pos.push_back((uint32_t)pos);
            pos += 4 + (size_t)l;
        }
        x.end = pos;
    };
    auto parse = [&](int t) {
        Part& x = parts[t];
        if (!x.used) return;
        for (size_t k = 0; k < x.pos.size(); ++k) {
            const size_t q = x.pos[k];
            const uint32_t l = (uint32_t)p[q] | (uint32_t)p[q + 1] << 8 | (uint32_t)p[q + 2] << 16 |
                               (uint32_t)p[q + 3] << 24;
            if (!parse_request(p + q + 4, l, q + 4, out[x.base + k])) {
                bad_parse.store(true, std::memory_order_relaxed);
                return;
            }
        }
        range(x.base, x.base + (uint32_t)x.pos.size());
    };
    auto& pool = parse_pool();
    if (!pool.run(T, walk)) {
        if (!parse_payload(p, len, out)) return false;
        sized(out.size());
        range((uint32_t)0, (uint32_t)out.size());
        return true;
    }
    // join: accept thread t's walk while the chain reaches its start exactly
    size_t at = parts[0].end;
    bool chain_bad = parts[0].bad;
    parts[0].used = true;
    int last = 0;
    for (int t = 1; t < T && !chain_bad; ++t) {
        if (parts[t].start == SIZE_MAX) continue;  // no candidate in this range: t-1 walked over it
        if (parts[t].start != at) break;          // a false candidate: walk on alone from `at`
        parts[t].used = true;
        chain_bad = parts[t].bad;
        at = parts[t].end;
        last = t;
    }
    if (chain_bad) return false;
    if (at != len) {  // the rest of the chain, on this thread
        Part& x = parts[last];
        size_t pos = at;
        while (pos < len) {
            if (len - pos < 4) return false;
            const uint32_t l = (uint32_t)p[pos] | (uint32_t)p[pos + 1] << 8 | (uint32_t)p[pos + 2] << 16 |
                               (uint32_t)p[pos + 3] << 24;
            if (l > len - pos - 4) return false;
            x.pos.push_back((uint32_t)pos);
            pos += 4 + (size_t)l;
        }
        for (int t = last + 1; t < T; ++t) parts[t].used = false;
    }
    uint32_t total = 0;
    for (auto& x : parts)
        if (x.used) {
            x.base = total;
            total += (uint32_t)x.pos.size();
        }
    static const bool trace = getenv("SBFT_PARSE_TRACE") != nullptr;  // diagnostics
    if (trace) {
        fprintf(stderr, "parse T=%d", T);
        for (auto& x : parts) fprintf(stderr, " [%s %zu]", x.used ? "used" : "dropped", x.pos.size());
        fprintf(stderr, " total=%u count=%u\n", total, count);
    }
    if (total != count) return false;
    out.resize(count);
    sized((size_t)count);
    if (!pool.run(T, parse)) {  // another caller took the pool meanwhile: parse alone
        for (int t = 0; t < T; ++t) parse(t);
    }
    return !bad_parse.load();
}

struct Msg {
    const uint8_t* digest = nullptr;
    size_t digest_len = 0;
    const uint8_t* aux = nullptr;
    size_t aux_len = 0;
};

bool parse_msg(const uint8_t* m, size_t len, Msg& out) {
    Reader r{m, len};
    const uint8_t* q;
    uint32_t a, b;
    if (!m || !r.take(4, q) || std::memcmp(q, MSG_MAGIC, 4)) return false;
    if (!r.u16(a) || !r.take(a, out.digest)) return false;
    out.digest_len = a;
    if (!r.u32(b) || !r.take(b, out.aux)) return false;
    out.aux_len = b;
    return r.pos == len;
}

void put_err(char* err, size_t cap, const char* fmt, ...) {
    if (!err || !cap) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err, cap, fmt, ap);
    va_end(ap);
}

bool write_info(char*& w, char* end, const Req::Str& cid, const Req::Str& id) {
    if ((size_t)(end - w) < (size_t)cid.n + (size_t)id.n + 2) return false;
    std::memcpy(w, cid.p, cid.n);
    w += cid.n;
    *w++ = 0;
    std::memcpy(w, id.p, id.n);
    w += id.n;
    *w++ = 0;
    return true;
}

// VerifyProposal's result: the first request with a 0 verdict fails the whole proposal (with
// its index and ids in the message), else the RequestInfos in payload order.
// infos == nullptr: the records were already written (info_rc is how that went)
int finish_proposal(const std::vector<Req>& reqs, const std::vector<uint8_t>& ok, char* infos, size_t infos_cap,
                    size_t* count, int64_t* bad_index, char* err, size_t err_cap, int info_rc = 0) {
    const size_t n = reqs.size();
    if (ok.size() != n) return SBFT_GV_EINVAL;
    for (size_t i = 0; i < n; ++i)
        if (!ok[i]) {
            if (bad_index) *bad_index = (int64_t)i;
            put_err(err, err_cap, "request %zu (%.*s:%.*s) has an invalid signature", i, reqs[i].client_id.n,
                    reqs[i].client_id.p, reqs[i].req_id.n, reqs[i].req_id.p);
            return SBFT_V_EVERIFY;
        }
    if (infos) {
        char* w = infos;
        char* end = infos + infos_cap;
        for (auto& q : reqs)
            if (!write_info(w, end, q.client_id, q.req_id)) return SBFT_V_ESPACE;
    } else if (info_rc) {
        return info_rc;
    }
    *count = n;
    return 0;
}

// Open-addressing map from a 64-byte public key (x || y) to its engine key id: the
// VerifyProposal lookup runs once per request (10k per proposal), so no per-lookup allocation.
struct KeyMap {
    std::vector<std::array<uint8_t, 64>> keys;
    std::vector<uint32_t> ids;  // 0 = empty slot
    size_t count = 0;
    static size_t hash(const uint8_t* k) {
        uint64_t a, b;
        std::memcpy(&a, k + 24, 8);  // low words of x and y: uniformly distributed
        std::memcpy(&b, k + 56, 8);
        return (size_t)((a * 0x9E3779B97F4A7C15ull) ^ b);
    }
    uint32_t find(const uint8_t* k) const {
        if (ids.empty()) return 0;
        const size_t mask = ids.size() - 1;
        for (size_t i = hash(k) & mask;; i = (i + 1) & mask) {
            if (!ids[i]) return 0;
            if (std::memcmp(keys[i].data(), k, 64) == 0) return ids[i];
        }
    }
    // the slot find(k) probes first: fetched ahead while earlier lookups run (a 10k-key table
    // is ~2 MB, mostly outside L2, and the lookups are otherwise serial misses)
    void prefetch(const uint8_t* k) const {
        if (ids.empty()) return;
        const size_t i = hash(k) & (ids.size() - 1);
        __builtin_prefetch(&ids[i]);
        __builtin_prefetch(keys[i].data());
        __builtin_prefetch(keys[i].data() + 63);
    }
    void put(const uint8_t* k, uint32_t id) {
        if (2 * (count + 1) > ids.size()) {
            KeyMap bigger;
            const size_t cap = std::max<size_t>(64, 2 * ids.size());
            bigger.keys.resize(cap);
            bigger.ids.assign(cap, 0);
            for (size_t i = 0; i < ids.size(); ++i)
                if (ids[i]) bigger.put(keys[i].data(), ids[i]);
            *this = std::move(bigger);
        }
        const size_t mask = ids.size() - 1;
        for (size_t i = hash(k) & mask;; i = (i + 1) & mask) {
            if (!ids[i]) {
                std::memcpy(keys[i].data(), k, 64);
                ids[i] = id;
                ++count;
                return;
            }
            if (std::memcmp(keys[i].data(), k, 64) == 0) {
                ids[i] = id;
                return;
            }
        }
    }
};

}  // namespace

// ---------------------------------------------------------------------- verifier
struct sbft_verifier {
    sbft_gv_ctx* ctx;
    std::atomic<uint64_t> vseq;
    std::shared_mutex keys_mu;
    // consenter id -> x || y (big-endian) and its engine key id (comb tables, 0 = none)
    struct KeyEnt {
        std::array<uint8_t, 64> xy;
        uint32_t kid = 0;
    };
    std::unordered_map<uint64_t, KeyEnt> keys;
    // client-key registry (sbft_verifier_add_clients): request key -> engine key id
    mutable std::shared_mutex clients_mu;
    KeyMap clients;
    // Proposal.Digest memo (view.go:435,443,524 recompute it per proposal): exact-content key
    std::mutex memo_mu;
    struct Memo {
        std::vector<uint8_t> payload, header, metadata;
        int64_t vseq = 0;
        char digest[65] = {0};
        bool valid = false;
    } memo[4];
    int memo_next = 0;

    // VerifyConsenterSig coalescer (sbft_verifier_coalesce_consenter_sigs). The library verifies
    // a decision's q-1 commit votes from q-1 goroutines at once (view.go:537-541 -> :834), each
    // with a single VerifyConsenterSig call; concurrent calls join one batch and share one
    // launch. A batch closes when it holds cs_max calls or cs_wait after its first call.
    struct CsEntry {
        const sbft_signature* sig;
        const sbft_proposal* p;
        int32_t status = 0;
        std::string why;
    };
    struct CsBatch {
        std::vector<CsEntry*> entries;
        bool closed = false;  // no more entries (full, or the leader's window ended)
        int rc = 0;
        std::chrono::steady_clock::time_point t_open;  // the leader's arrival
        std::condition_variable cv;                    // wakes the leader when the batch fills
        DoneFlag done;                                 // wakes the followers when the results are published
        DoneFlag ready;  // the batch is closed and its launch under way (pre-wake, see consenter_coalesced)
    };
    std::mutex cs_mu;
    std::shared_ptr<CsBatch> cs_open;
    size_t cs_max = 0;  // 0 = off: every call is its own launch
    std::chrono::microseconds cs_wait{0};
    // a batch that opens within 2 cs_wait of the previous one's close holds the stragglers of
    // the same burst (callers the OS scheduled late): it waits only cs_follow for more
    std::chrono::steady_clock::time_point cs_last_close{};
    std::chrono::microseconds cs_follow{-1};  // < 0: cs_wait / 4 (SBFT_CS_FOLLOW_US overrides)
    std::atomic<uint64_t> cs_launches{0}, cs_calls{0};

    void digest_of(const sbft_proposal* p, char out[65]) {
        auto same = [](const std::vector<uint8_t>& v, const uint8_t* q, size_t n) {
            return v.size() == n && (n == 0 || std::memcmp(v.data(), q, n) == 0);
        };
        {
            std::lock_guard<std::mutex> g(memo_mu);
            for (auto& m : memo)
                if (m.valid && m.vseq == p->verification_sequence && same(m.payload, p->payload, p->payload_len) &&
                    same(m.header, p->header, p->header_len) && same(m.metadata, p->metadata, p->metadata_len)) {
                    std::memcpy(out, m.digest, 65);
                    return;
                }
        }
        sbft_proposal_digest(p, out);
        std::lock_guard<std::mutex> g(memo_mu);
        Memo& m = memo[memo_next];
        memo_next = (memo_next + 1) % 4;
        m.payload.assign(p->payload, p->payload + p->payload_len);
        m.header.assign(p->header, p->header + p->header_len);
        m.metadata.assign(p->metadata, p->metadata + p->metadata_len);
        m.vseq = p->verification_sequence;
        std::memcpy(m.digest, out, 65);
        m.valid = true;
    }

    bool key_of(uint64_t id, std::array<uint8_t, 64>& k, uint32_t* kid = nullptr) {
        std::shared_lock<std::shared_mutex> g(keys_mu);
        auto it = keys.find(id);
        if (it == keys.end()) return false;
        k = it->second.xy;
        if (kid) *kid = it->second.kid;
        return true;
    }

    // Verify n (message, r||s, registered key id) triples with one keyed launch
    // (p256_keyed.hip: comb tables, no doublings; the messages are hashed in the launch).
    int gpu_verify_keyed(const std::vector<const uint8_t*>& msgs, const std::vector<size_t>& lens,
                         const std::vector<const uint8_t*>& sigs, const std::vector<uint32_t>& kids, uint8_t* ok) {
        const size_t n = msgs.size();
        if (!n) return 0;
        if (!ctx) return SBFT_GV_ENODEV;
        size_t total = 0;
        for (size_t l : lens) total += l;
        std::vector<uint8_t> blob(total ? total : 1);
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n);
        std::vector<uint8_t> r(32 * n), s(32 * n);
        size_t at = 0;
        for (size_t i = 0; i < n; ++i) {
            off[i] = at;
            len[i] = (uint32_t)lens[i];
            if (lens[i]) std::memcpy(&blob[at], msgs[i], lens[i]);
            at += lens[i];
            std::memcpy(&r[32 * i], sigs[i], 32);
            std::memcpy(&s[32 * i], sigs[i] + 32, 32);
        }
        return sbft_gv_sha256_verify_p256_keyed(ctx, blob.data(), total, off.data(), len.data(), r.data(), s.data(),
                                                kids.data(), n, ok);
    }

    // Verify n (message, r||s, key) triples with one fused launch. ok must hold n bytes.
    int gpu_verify_messages(const std::vector<const uint8_t*>& msgs, const std::vector<size_t>& lens,
                            const std::vector<const uint8_t*>& sigs, const std::vector<const uint8_t*>& keys64,
                            uint8_t* ok) {
        const size_t n = msgs.size();
        if (!n) return 0;
        if (!ctx) return SBFT_GV_ENODEV;
        std::vector<uint8_t> blob;
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n);
        std::vector<uint8_t> r(32 * n), s(32 * n), qx(32 * n), qy(32 * n);
        for (size_t i = 0; i < n; ++i) {
            off[i] = blob.size();
            len[i] = (uint32_t)lens[i];
            blob.insert(blob.end(), msgs[i], msgs[i] + lens[i]);
            std::memcpy(&r[32 * i], sigs[i], 32);
            std::memcpy(&s[32 * i], sigs[i] + 32, 32);
            std::memcpy(&qx[32 * i], keys64[i], 32);
            std::memcpy(&qy[32 * i], keys64[i] + 32, 32);
        }
        if (blob.empty()) blob.push_back(0);
        return sbft_gv_sha256_verify_p256(ctx, blob.data(), blob.size(), off.data(), len.data(), r.data(),
                                          s.data(), qx.data(), qy.data(), n, ok, nullptr);
    }

    // Verify n standalone signed requests with one fused launch (VerifyRequest's batch form).
    // status[i]: 0 ok, SBFT_V_EFORMAT, SBFT_V_EVERIFY; parsed[i] holds the request's ids.
    int requests_batch(const uint8_t* const* reqs, const size_t* lens, size_t n, int32_t* status,
                       std::vector<Req>& parsed) {
        parsed.assign(n, Req());
        std::vector<const uint8_t*> msgs, sv, kv;
        std::vector<size_t> mlens, which;
        for (size_t i = 0; i < n; ++i) {
            status[i] = 0;
            if (!reqs[i] || !parse_request(reqs[i], lens[i], 0, parsed[i]) || parsed[i].pub[0] != 0x04) {
                status[i] = SBFT_V_EFORMAT;
                continue;
            }
            msgs.push_back(reqs[i]);
            mlens.push_back(parsed[i].body_len);
            sv.push_back(parsed[i].sig);
            kv.push_back(parsed[i].pub + 1);
            which.push_back(i);
        }
        std::vector<uint8_t> ok(which.size());
        const int rc = gpu_verify_messages(msgs, mlens, sv, kv, ok.data());
        if (rc) return rc;
        for (size_t k = 0; k < which.size(); ++k)
            if (!ok[k]) status[which[k]] = SBFT_V_EVERIFY;
        return 0;
    }

    // VerifySignature's batch form: n (id, r||s, msg) under registered keys; keys with comb
    // tables take the keyed launch, the rest the generic fused launch. reasons[i] = error text.
    int signatures_batch(const sbft_signature* sigs, size_t n, int32_t* status, std::vector<std::string>* reasons) {
        std::vector<const uint8_t*> msgs, sv, kv, kmsgs, ksv;
        std::vector<size_t> lens, which, klens, kwhich;
        std::vector<uint32_t> kids;
        std::vector<std::array<uint8_t, 64>> keybuf(n);
        if (reasons) reasons->assign(n, std::string());
        static const uint8_t empty = 0;
        for (size_t i = 0; i < n; ++i) {
            status[i] = 0;
            uint32_t kid = 0;
            if (!key_of(sigs[i].id, keybuf[i], &kid)) {
                status[i] = SBFT_V_EKEY;
                if (reasons) (*reasons)[i] = "unknown signer " + std::to_string(sigs[i].id);
                continue;
            }
            if (sigs[i].value_len != 64 || !sigs[i].value) {
                status[i] = SBFT_V_EFORMAT;
                if (reasons) (*reasons)[i] = "signature value must be 64 bytes r||s";
                continue;
            }
            const uint8_t* m = sigs[i].msg ? sigs[i].msg : &empty;
            if (kid) {
                kmsgs.push_back(m);
                klens.push_back(sigs[i].msg_len);
                ksv.push_back(sigs[i].value);
                kids.push_back(kid);
                kwhich.push_back(i);
            } else {
                msgs.push_back(m);
                lens.push_back(sigs[i].msg_len);
                sv.push_back(sigs[i].value);
                kv.push_back(keybuf[i].data());
                which.push_back(i);
            }
        }
        std::vector<uint8_t> ok(which.size()), kok(kwhich.size());
        int rc = gpu_verify_keyed(kmsgs, klens, ksv, kids, kok.data());
        if (rc) return rc;
        rc = gpu_verify_messages(msgs, lens, sv, kv, ok.data());
        if (rc) return rc;
        auto mark = [&](const std::vector<size_t>& w, const std::vector<uint8_t>& o) {
            for (size_t k = 0; k < w.size(); ++k)
                if (!o[k]) {
                    status[w[k]] = SBFT_V_EVERIFY;
                    if (reasons) (*reasons)[w[k]] = "invalid signature from " + std::to_string(sigs[w[k]].id);
                }
        };
        mark(kwhich, kok);
        mark(which, ok);
        return 0;
    }

    // Check + verify consenter signatures over one proposal. status[i]: 0 ok, <0 error;
    // reasons[i] gets the error text.
    int consenter_batch(const sbft_signature* sigs, size_t n, const sbft_proposal* p, int32_t* status,
                        std::vector<std::string>* reasons) {
        std::vector<const sbft_proposal*> props(n, p);
        return consenter_batch(sigs, n, props.data(), status, reasons);
    }
    // The same with a proposal per signature (the consenter-signature coalescer batches calls
    // from concurrent callers, which may check different proposals): one launch for all.
    int consenter_batch(const sbft_signature* sigs, size_t n, const sbft_proposal* const* props, int32_t* status,
                        std::vector<std::string>* reasons) {
        char digest[65];
        const sbft_proposal* last = nullptr;
        std::vector<const uint8_t*> msgs, sv, kv, kmsgs, ksv;
        std::vector<size_t> lens, which, klens, kwhich;
        std::vector<uint32_t> kids;
        std::vector<std::array<uint8_t, 64>> keybuf(n);
        if (reasons) reasons->assign(n, std::string());
        for (size_t i = 0; i < n; ++i) {
            Msg m;
            status[i] = 0;
            if (props[i] != last) {  // digest_of is memoised; consecutive equal proposals skip it
                digest_of(props[i], digest);
                last = props[i];
            }
            if (!parse_msg(sigs[i].msg, sigs[i].msg_len, m)) {
                status[i] = SBFT_V_EFORMAT;
                if (reasons) (*reasons)[i] = "malformed signature message";
                continue;
            }
            if (m.digest_len != 64 || std::memcmp(m.digest, digest, 64) != 0) {
                status[i] = SBFT_V_EVERIFY;
                if (reasons) (*reasons)[i] = "signature message does not bind the proposal digest";
                continue;
            }
            uint32_t kid = 0;
            if (!key_of(sigs[i].id, keybuf[i], &kid)) {
                status[i] = SBFT_V_EKEY;
                if (reasons) (*reasons)[i] = "unknown consenter " + std::to_string(sigs[i].id);
                continue;
            }
            if (sigs[i].value_len != 64 || !sigs[i].value) {
                status[i] = SBFT_V_EFORMAT;
                if (reasons) (*reasons)[i] = "signature value must be 64 bytes r||s";
                continue;
            }
            if (kid) {  // registered consenter key: comb-table launch
                kmsgs.push_back(sigs[i].msg);
                klens.push_back(sigs[i].msg_len);
                ksv.push_back(sigs[i].value);
                kids.push_back(kid);
                kwhich.push_back(i);
                continue;
            }
            msgs.push_back(sigs[i].msg);
            lens.push_back(sigs[i].msg_len);
            sv.push_back(sigs[i].value);
            kv.push_back(keybuf[i].data());
            which.push_back(i);
        }
        std::vector<uint8_t> ok(which.size()), kok(kwhich.size());
        int rc = gpu_verify_keyed(kmsgs, klens, ksv, kids, kok.data());
        if (rc) return rc;
        rc = gpu_verify_messages(msgs, lens, sv, kv, ok.data());
        if (rc) return rc;
        auto mark = [&](const std::vector<size_t>& w, const std::vector<uint8_t>& o) {
            for (size_t k = 0; k < w.size(); ++k)
                if (!o[k]) {
                    status[w[k]] = SBFT_V_EVERIFY;
                    if (reasons) (*reasons)[w[k]] = "invalid signature";
                }
        };
        mark(kwhich, kok);
        mark(which, ok);
        return 0;
    }
};

extern "C" {

void sbft_sha256_host(const uint8_t* msg, size_t len, uint8_t out[32]) { sha256(msg, len, out); }

void sbft_proposal_digest(const sbft_proposal* p, char out65[65]) {
    // SHA-256 over the DER encoding, streamed: SEQUENCE { OCTET STRING payload, header,
    // metadata; INTEGER verification_sequence }. Only the tag/length prefixes are built here;
    // the (MB-sized) payload is hashed where it lies.
    std::vector<uint8_t> pre[3], seq, tail;
    const uint8_t* data[3] = {p->payload, p->header, p->metadata};
    const size_t lens[3] = {p->payload_len, p->header_len, p->metadata_len};
    size_t body = 0;
    for (int i = 0; i < 3; ++i) {
        pre[i].push_back(0x04);
        der_len(pre[i], lens[i]);
        body += pre[i].size() + lens[i];
    }
    der_int64(tail, p->verification_sequence);
    body += tail.size();
    seq.push_back(0x30);
    der_len(seq, body);
    Sha256 h;
    h.update(seq.data(), seq.size());
    for (int i = 0; i < 3; ++i) {
        h.update(pre[i].data(), pre[i].size());
        if (lens[i]) h.update(data[i], lens[i]);
    }
    h.update(tail.data(), tail.size());
    uint8_t d[32];
    h.final(d);
    static const char* hx = "0123456789abcdef";
    for (int i = 0; i < 32; ++i) {
        out65[2 * i] = hx[d[i] >> 4];
        out65[2 * i + 1] = hx[d[i] & 15];
    }
    out65[64] = 0;
}

int sbft_commit_signatures_digest(const sbft_signature* sigs, size_t n, uint8_t out32[32]) {
    // CommitSignaturesDigest (internal/bft/util.go:557-579): SHA-256 over Go asn1.Marshal of
    // IntDoubleBytes{A: [{A: int64(Signer), B: Value, C: Msg}, ...]}, i.e.
    //   SEQUENCE { SEQUENCE { SEQUENCE { INTEGER signer, OCTET STRING value, OCTET STRING msg } ... } }
    // No signatures: nil (returns 0, out32 untouched). Values and messages are hashed in place;
    // only the tag/length prefixes are built.
    if (n == 0) return 0;
    if (!sigs || !out32) return SBFT_GV_EINVAL;
    std::vector<uint8_t> ints;  // the n INTEGER encodings, back to back
    std::vector<uint32_t> int_end(n);
    std::vector<size_t> elem(n);
    size_t inner = 0;
    for (size_t i = 0; i < n; ++i) {
        der_int64(ints, (int64_t)sigs[i].id);
        int_end[i] = (uint32_t)ints.size();
        std::vector<uint8_t> l;
        der_len(l, sigs[i].value_len);
        size_t body = (int_end[i] - (i ? int_end[i - 1] : 0)) + 1 + l.size() + sigs[i].value_len;
        l.clear();
        der_len(l, sigs[i].msg_len);
        body += 1 + l.size() + sigs[i].msg_len;
        elem[i] = body;
        l.clear();
        der_len(l, body);
        inner += 1 + l.size() + body;
    }
    std::vector<uint8_t> hdr;
    std::vector<uint8_t> mid;
    mid.push_back(0x30);
    der_len(mid, inner);
    hdr.push_back(0x30);
    der_len(hdr, mid.size() + inner);
    Sha256 h;
    h.update(hdr.data(), hdr.size());
    h.update(mid.data(), mid.size());
    for (size_t i = 0; i < n; ++i) {
        std::vector<uint8_t> t;
        t.push_back(0x30);
        der_len(t, elem[i]);
        const size_t i0 = i ? int_end[i - 1] : 0;
        t.insert(t.end(), ints.begin() + i0, ints.begin() + int_end[i]);
        t.push_back(0x04);
        der_len(t, sigs[i].value_len);
        h.update(t.data(), t.size());
        if (sigs[i].value_len) h.update(sigs[i].value, sigs[i].value_len);
        t.clear();
        t.push_back(0x04);
        der_len(t, sigs[i].msg_len);
        h.update(t.data(), t.size());
        if (sigs[i].msg_len) h.update(sigs[i].msg, sigs[i].msg_len);
    }
    h.final(out32);
    return 32;
}

sbft_verifier* sbft_verifier_new(sbft_gv_ctx* ctx, uint64_t verification_sequence) {
    // ctx may be NULL for a parse-only verifier (RequestsFromProposal, AuxiliaryData);
    // verification calls on it fail with SBFT_GV_ENODEV.
    auto* v = new sbft_verifier();
    v->ctx = ctx;
    v->vseq = verification_sequence;
    return v;
}
void sbft_verifier_free(sbft_verifier* v) { delete v; }

int sbft_verifier_add_consenter(sbft_verifier* v, uint64_t id, const uint8_t pubkey65[65]) {
    if (!v || !pubkey65 || pubkey65[0] != 0x04) return SBFT_GV_EINVAL;
    sbft_verifier::KeyEnt k;
    std::memcpy(k.xy.data(), pubkey65 + 1, 64);
    if (v->ctx) {
        // precompute the key's comb tables on every device; an invalid point keeps kid = 0
        // (its signatures then take the generic path, which rejects them like Go does)
        const int rc = sbft_gv_register_key(v->ctx, pubkey65 + 1, pubkey65 + 33, &k.kid);
        if (rc && rc != SBFT_GV_EINVAL) return rc;
        if (rc) k.kid = 0;
    }
    std::unique_lock<std::shared_mutex> g(v->keys_mu);
    v->keys[id] = k;
    return 0;
}

int sbft_verifier_add_clients(sbft_verifier* v, const uint8_t* pubkeys65, size_t n) {
    if (!v || (n && !pubkeys65)) return SBFT_GV_EINVAL;
    if (!v->ctx) return SBFT_GV_ENODEV;
    std::vector<uint8_t> qx(32 * n), qy(32 * n);
    std::vector<uint32_t> ids(n);
    size_t m = 0;
    std::vector<size_t> which;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* k = pubkeys65 + 65 * i;
        if (k[0] != 0x04) continue;  // not SEC1 uncompressed: its requests stay on the generic path
        std::memcpy(&qx[32 * m], k + 1, 32);
        std::memcpy(&qy[32 * m], k + 33, 32);
        which.push_back(i);
        ++m;
    }
    // under the engine's client-table budget: keys past it get id 0 and stay on the generic path
    const int rc = sbft_gv_register_client_keys(v->ctx, qx.data(), qy.data(), m, ids.data(), nullptr);
    if (rc) return rc;
    std::unique_lock<std::shared_mutex> g(v->clients_mu);
    for (size_t j = 0; j < m; ++j)
        if (ids[j]) v->clients.put(pubkeys65 + 65 * which[j] + 1, ids[j]);
    return 0;
}

size_t sbft_verifier_client_count(const sbft_verifier* v) {
    if (!v) return 0;
    std::shared_lock<std::shared_mutex> g(v->clients_mu);
    return v->clients.count;
}

uint64_t sbft_verifier_verification_sequence(const sbft_verifier* v) { return v ? v->vseq.load() : 0; }
void sbft_verifier_set_verification_sequence(sbft_verifier* v, uint64_t seq) {
    if (v) v->vseq = seq;
}

// Threads per proposal parse (parse_payload_par), SBFT_PARSE_THREADS overriding the default.
// VerifyProposal parses on one: there the payload's DMA staging runs on another core at the same
// time, and on the GPU box (16-core share of a 256-thread host) three parse threads took the
// parse from ~92 to ~155 us and the call's p50 from 0.92 to 0.98 ms
// (profiles/r03h_parse_threads_ab.txt). RequestsFromProposal parses on one as well: that A/B
// is the only measurement on the box, and the helpers yield-spin for 0.5 ms after every job,
// which costs the job's CPU quota (the throttling behind r03w's coalescer tail). A deployment
// with cores to spare sets SBFT_PARSE_THREADS.
static int parse_threads_for(int dflt) {
    const char* e = getenv("SBFT_PARSE_THREADS");
    return e ? std::max(1, std::atoi(e)) : dflt;
}

int sbft_verifier_requests_from_proposal(sbft_verifier* v, const sbft_proposal* p, char* infos,
                                         size_t infos_cap, size_t* count) {
    if (!v || !p || !count) return SBFT_GV_EINVAL;
    std::vector<Req>& reqs = proposal_scratch().reqs;
    *count = 0;
    static const int parse_threads = parse_threads_for(1);
    if (!parse_payload_par(p->payload, p->payload_len, reqs, parse_threads, [](size_t) {}, [](uint32_t, uint32_t) {}))
        return SBFT_V_EFORMAT;
    char* w = infos;
    char* end = infos + infos_cap;
    for (auto& r : reqs)
        if (!write_info(w, end, r.client_id, r.req_id)) return SBFT_V_ESPACE;
    *count = reqs.size();
    return 0;
}

int sbft_verifier_verify_proposal(sbft_verifier* v, const sbft_proposal* p, char* infos, size_t infos_cap,
                                  size_t* count, int64_t* bad_index, char* err, size_t err_cap) {
    if (!v || !p || !count) return SBFT_GV_EINVAL;
    *count = 0;
    if (bad_index) *bad_index = -1;
    ProposalScratch& scr = proposal_scratch();  // this thread's, also when prepare runs elsewhere
    std::vector<Req>& reqs = scr.reqs;
    std::vector<uint8_t>& ok = scr.ok;
    // The format verdict: the full parse (magic, ids, lengths) and the key prefix of every
    // request, the first bad one in order reported. It runs while the GPU verifies (`during`):
    // the launch needs only the chain of length prefixes (walk_payload), and the call returns
    // its verdict, not the GPU's, whenever it finds a malformed request.
    static const int parse_threads = parse_threads_for(1);
    bool checked = false;
    int fmt_rc = 0;
    auto check = [&]() -> int {
        checked = true;
        std::atomic<uint32_t> first_bad_key{UINT32_MAX};
        const bool ok_parse = parse_payload_par(
            p->payload, p->payload_len, reqs, parse_threads, [](size_t) {}, [&](uint32_t b, uint32_t e) {
                for (uint32_t i = b; i < e; ++i)
                    if (reqs[i].pub[0] != 0x04) {  // the first one in order is reported below
                        uint32_t cur = first_bad_key.load(std::memory_order_relaxed);
                        while (i < cur && !first_bad_key.compare_exchange_weak(cur, i)) {
                        }
                        break;
                    }
            });
        if (!ok_parse) {
            reqs.clear();
            put_err(err, err_cap, "malformed proposal payload");
            return SBFT_V_EFORMAT;
        }
        const uint32_t i = first_bad_key.load();
        if (i != UINT32_MAX) {
            if (bad_index) *bad_index = (int64_t)i;
            put_err(err, err_cap, "request %u (%.*s:%.*s): public key is not SEC1 uncompressed", i,
                    reqs[i].client_id.n, reqs[i].client_id.p, reqs[i].req_id.n, reqs[i].req_id.p);
            return SBFT_V_EFORMAT;
        }
        return 0;
    };
    if (!v->ctx) {
        if (int prc = check()) return prc;
        ok.clear();
        if (reqs.empty()) return finish_proposal(reqs, ok, infos, infos_cap, count, bad_index, err, err_cap);
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(SBFT_GV_ENODEV));
        return SBFT_GV_ENODEV;
    }
    bool registered;
    {
        std::shared_lock<std::shared_mutex> g(v->clients_mu);
        registered = v->clients.count != 0;
    }
    // One framed launch, the walk overlapped with the payload copy; the format check and the
    // RequestInfo records run while the GPU verifies (they are returned only if every request
    // passes). With client keys registered, every request's key (the 64 bytes before its
    // signature) is looked up after the walk: if all are registered, the batch takes the keyed
    // launch over their comb tables (no doublings); otherwise the generic launch verifies every
    // request (the same verdicts).
    std::vector<uint32_t>& kid = scr.kid;
    kid.clear();
    auto prepare = [&](std::vector<uint64_t>& off, std::vector<uint32_t>& len) -> int {
        if (!walk_payload(p->payload, p->payload_len, off, len)) {
            checked = true;  // the full parse would reject it too: no launch
            reqs.clear();
            put_err(err, err_cap, "malformed proposal payload");
            return fmt_rc = SBFT_V_EFORMAT;
        }
        return 0;
    };
    auto prepare_keyed = [&](std::vector<uint64_t>& off, std::vector<uint32_t>& len) -> int {
        if (int prc = prepare(off, len)) return prc;
        // each key's map slot prefetched kAhead lookups before it is read
        constexpr size_t kAhead = 8;
        const size_t n = off.size();
        auto key = [&](size_t i) { return p->payload + off[i] + len[i] - 64; };
        std::shared_lock<std::shared_mutex> g(v->clients_mu);
        kid.resize(n);
        for (size_t i = 0; i < n && i < kAhead; ++i) v->clients.prefetch(key(i));
        for (size_t i = 0; i < n; ++i) {
            if (i + kAhead < n) v->clients.prefetch(key(i + kAhead));
            if (!(kid[i] = v->clients.find(key(i)))) {
                kid.clear();
                break;
            }
        }
        return 0;
    };
    int info_rc = 0;
    auto during = [&] {
        if ((fmt_rc = check())) return;
        char* w = infos;
        char* end = infos + infos_cap;
        for (auto& q : reqs)
            if (!write_info(w, end, q.client_id, q.req_id)) {
                info_rc = SBFT_V_ESPACE;
                return;
            }
    };
    const int rc = registered ? sbft_gv_framed_overlapped(v->ctx, p->payload, p->payload_len, 0, -64, prepare_keyed,
                                                          ok, during, &kid)
                              : sbft_gv_framed_overlapped(v->ctx, p->payload, p->payload_len, 0, -64, prepare, ok,
                                                          during);
    if (!checked) fmt_rc = check();  // the engine returned before `during` (or failed)
    if (fmt_rc) return fmt_rc;       // the format verdict first, as before any launch
    if (rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(rc));
        return rc;
    }
    if (reqs.size() != ok.size()) return SBFT_GV_EINVAL;
    return finish_proposal(reqs, ok, nullptr, 0, count, bad_index, err, err_cap, info_rc);
}

int sbft_verifier_verify_request(sbft_verifier* v, const uint8_t* req, size_t len, char* info, size_t info_cap,
                                 char* err, size_t err_cap) {
    if (!v || (!req && len)) return SBFT_GV_EINVAL;
    Req q;
    // an empty request (a Go nil or zero-length slice arrives as NULL, 0) is a malformed request
    // from the network, never an engine error: Controller.HandleRequest passes whatever a client
    // or a forwarding replica sent (controller.go:233-246)
    if (!req || !parse_request(req, len, 0, q) || q.pub[0] != 0x04) {
        put_err(err, err_cap, "malformed request");
        return SBFT_V_EFORMAT;
    }
    std::vector<const uint8_t*> msgs{req}, sigs{q.sig}, keys{q.pub + 1};
    std::vector<size_t> lens{q.body_len};
    uint8_t ok = 0;
    const int rc = v->gpu_verify_messages(msgs, lens, sigs, keys, &ok);
    if (rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(rc));
        return rc;
    }
    if (!ok) {
        put_err(err, err_cap, "request %.*s:%.*s has an invalid signature", q.client_id.n, q.client_id.p,
                q.req_id.n, q.req_id.p);
        return SBFT_V_EVERIFY;
    }
    char* w = info;
    if (info && !write_info(w, info + info_cap, q.client_id, q.req_id)) return SBFT_V_ESPACE;
    return 0;
}

// One VerifyConsenterSig through the coalescer: join the open batch (or open one and lead
// it), and return this call's own status and reason. The leader waits until the batch is full
// or its deadline passes, closes it, runs ONE consenter_batch over every joined call (their
// proposals may differ) and wakes the others. No background thread.
static int consenter_coalesced(sbft_verifier* v, const sbft_signature* s, const sbft_proposal* p, int32_t& st,
                               std::string& why) {
    using Batch = sbft_verifier::CsBatch;
    sbft_verifier::CsEntry me{s, p};
    std::shared_ptr<Batch> batch;
    bool leader = false;
    {
        std::unique_lock<std::mutex> g(v->cs_mu);
        std::chrono::microseconds window = v->cs_wait;
        if (!v->cs_open) {
            v->cs_open = std::make_shared<Batch>();
            const auto now = std::chrono::steady_clock::now();
            v->cs_open->t_open = now;
            leader = true;
            // stragglers of a burst whose first batch has just closed: the rest of the burst is
            // already in that batch, so a full window would only delay these callers
            if (now - v->cs_last_close < 2 * v->cs_wait) {
                static const long follow_env = [] {
                    const char* e = getenv("SBFT_CS_FOLLOW_US");
                    return e ? std::atol(e) : -1L;
                }();
                window = follow_env >= 0 ? std::chrono::microseconds(follow_env)
                         : v->cs_follow.count() >= 0 ? v->cs_follow
                                                     : v->cs_wait / 4;
            }
        }
        batch = v->cs_open;
        batch->entries.push_back(&me);
        if (batch->entries.size() >= v->cs_max) {
            batch->closed = true;
            v->cs_open.reset();
            v->cs_last_close = std::chrono::steady_clock::now();
            batch->cv.notify_all();  // wakes the leader early
        }
        if (leader) {
            // a sleep, not a spin: with more callers than cores a spinning leader delays the
            // arrivals it waits for. The timed wait would oversleep a window of tens of us by
            // the thread's timer slack (50 us by default): 1 us for the wait, then restored.
            const int slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
            if (slack > 1000) (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
            batch->cv.wait_until(g, batch->t_open + window, [&] { return batch->closed; });
            if (slack > 1000) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)slack, 0, 0, 0);
            if (!batch->closed) {
                batch->closed = true;
                v->cs_open.reset();
                v->cs_last_close = std::chrono::steady_clock::now();
            }
        }
    }
    // Pre-wake (followers yield-spin through the launch) is off by default: it doubles the
    // fan-out's CPU time (7.2-7.5 against 3.0-3.7 ms per 66-caller decision) and a job under a
    // CPU quota (the GPU box: cpu.max 16 CPUs, 256 in the affinity mask) is then throttled for
    // the rest of a quota period, a 2.7-48 ms outlier every few hundred decisions; without it
    // p99 0.30 ms, max 0.35-0.78 ms, p50 the same (profiles/r03w_cs_tail.txt).
    static const bool prewake = [] {
        const char* e = getenv("SBFT_CS_PREWAKE");
        return e && std::strcmp(e, "1") == 0;
    }();
    if (!leader) {
        if (prewake) {
            // Sleep until the leader closes the batch (the arrivals still to come need the
            // cores), then wait out the launch awake: the leader wakes the followers (a tree)
            // right before it stages and launches, so their wake-ups overlap the ~50 us the GPU
            // takes instead of following it. Bounded: a long batch sleeps again.
            batch->ready.wait(0);
            const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(400);
            while (!batch->done.v.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < until)
                sched_yield();
        }
        batch->done.wait(0);  // the batch is one launch away: sleep at once
    }
    if (leader) {
        if (prewake) batch->ready.set();
        static const bool trace = getenv("SBFT_CS_TRACE") != nullptr;  // diagnostics
        const auto tc = std::chrono::steady_clock::now();
        // closed: nobody else touches the entries until done is published
        const size_t n = batch->entries.size();
        std::vector<sbft_signature> sigs(n);
        std::vector<const sbft_proposal*> props(n);
        for (size_t i = 0; i < n; ++i) {
            sigs[i] = *batch->entries[i]->sig;
            props[i] = batch->entries[i]->p;
        }
        std::vector<int32_t> sts(n);
        std::vector<std::string> whys;
        const int rc = v->consenter_batch(sigs.data(), n, props.data(), sts.data(), &whys);
        v->cs_launches++;
        v->cs_calls += n;
        for (size_t i = 0; i < n; ++i) {
            batch->entries[i]->status = rc ? 0 : sts[i];
            if (!rc) batch->entries[i]->why = std::move(whys[i]);
        }
        batch->rc = rc;
        batch->done.set();
        if (trace)
            fprintf(stderr, "cs n=%zu gather=%.1f batch=%.1f us\n", n,
                    std::chrono::duration<double, std::micro>(tc - batch->t_open).count(),
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tc).count());
    }
    st = me.status;
    why = std::move(me.why);
    return batch->rc;
}

int sbft_verifier_coalesce_consenter_sigs(sbft_verifier* v, size_t max_batch, uint32_t max_wait_us) {
    if (!v) return SBFT_GV_EINVAL;
    std::lock_guard<std::mutex> g(v->cs_mu);
    v->cs_max = max_batch;
    v->cs_wait = std::chrono::microseconds(max_wait_us);
    return 0;
}

void sbft_verifier_consenter_stats(const sbft_verifier* v, uint64_t* launches, uint64_t* calls) {
    if (!v) return;
    if (launches) *launches = v->cs_launches.load();
    if (calls) *calls = v->cs_calls.load();
}

int sbft_verifier_verify_consenter_sig(sbft_verifier* v, const sbft_signature* s, const sbft_proposal* p,
                                       uint8_t* aux, size_t aux_cap, size_t* aux_len, char* err, size_t err_cap) {
    if (!v || !s || !p) return SBFT_GV_EINVAL;
    int32_t st = 0;
    int rc;
    std::string reason;
    size_t coalesce;
    {
        std::lock_guard<std::mutex> g(v->cs_mu);
        coalesce = v->cs_max;
    }
    if (coalesce > 1) {
        rc = consenter_coalesced(v, s, p, st, reason);
    } else {
        std::vector<std::string> why;
        rc = v->consenter_batch(s, 1, p, &st, &why);
        v->cs_launches++;
        v->cs_calls++;
        if (!rc) reason = why[0];
    }
    if (rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(rc));
        return rc;
    }
    if (st) {
        put_err(err, err_cap, "%s", reason.c_str());
        return st;
    }
    Msg m;
    parse_msg(s->msg, s->msg_len, m);
    if (aux_len) *aux_len = m.aux_len;
    if (aux) {
        if (aux_cap < m.aux_len) return SBFT_V_ESPACE;
        if (m.aux_len) std::memcpy(aux, m.aux, m.aux_len);
    }
    return 0;
}

int sbft_verifier_verify_consenter_sigs(sbft_verifier* v, const sbft_signature* sigs, size_t n,
                                        const sbft_proposal* p, int32_t* status) {
    if (!v || (n && (!sigs || !status)) || !p) return SBFT_GV_EINVAL;
    return v->consenter_batch(sigs, n, p, status, nullptr);
}

int sbft_verifier_verify_signature(sbft_verifier* v, const sbft_signature* s, char* err, size_t err_cap) {
    if (!v || !s) return SBFT_GV_EINVAL;
    int32_t st = 0;
    std::vector<std::string> why;
    const int rc = v->signatures_batch(s, 1, &st, &why);
    if (rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(rc));
        return rc;
    }
    if (st) put_err(err, err_cap, "%s", why[0].c_str());
    return st;
}

int sbft_verifier_verify_signatures(sbft_verifier* v, const sbft_signature* sigs, size_t n, int32_t* status) {
    if (!v || (n && (!sigs || !status))) return SBFT_GV_EINVAL;
    return v->signatures_batch(sigs, n, status, nullptr);
}

int sbft_verifier_verify_requests(sbft_verifier* v, const uint8_t* const* reqs, const size_t* lens, size_t n,
                                  int32_t* status) {
    if (!v || (n && (!reqs || !lens || !status))) return SBFT_GV_EINVAL;
    std::vector<Req> parsed;
    return v->requests_batch(reqs, lens, n, status, parsed);
}

int64_t sbft_verifier_auxiliary_data(const uint8_t* msg, size_t msg_len, uint8_t* aux, size_t aux_cap) {
    Msg m;
    if (!parse_msg(msg, msg_len, m)) return -1;
    if (aux && m.aux_len) std::memcpy(aux, m.aux, std::min(aux_cap, m.aux_len));
    return (int64_t)m.aux_len;
}

// ---------------------------------------------------------------------- batching hook
void sbft_compute_quorum(uint64_t n, int* q, int* f) {
    const int ff = ((int)n - 1) / 3;
    const int num = (int)n + ff + 1;
    if (f) *f = ff;
    if (q) *q = (num + 1) / 2;  // ceil(num / 2)
}

int sbft_verify_prev_commit_signatures(sbft_verifier* v, const sbft_signature* sigs, size_t n,
                                       const sbft_proposal* prev, uint64_t curr_vseq, int* skipped, char* err,
                                       size_t err_cap) {
    if (!v || !prev || (n && !sigs)) return SBFT_GV_EINVAL;
    if (skipped) *skipped = 0;
    if ((uint64_t)prev->verification_sequence != curr_vseq) {
        if (skipped) *skipped = 1;
        return 0;
    }
    std::vector<int32_t> st(n);
    std::vector<std::string> why;
    const int rc = v->consenter_batch(sigs, n, prev, st.data(), &why);
    if (rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(rc));
        return rc;
    }
    for (size_t i = 0; i < n; ++i)
        if (st[i]) {
            put_err(err, err_cap, "failed verifying consenter signature of %llu: %s", (unsigned long long)sigs[i].id,
                    why[i].c_str());
            return SBFT_V_EVERIFY;
        }
    return 0;
}

int sbft_collect_commits(sbft_verifier* v, const sbft_signature* votes, const char* const* vote_digests, size_t n,
                         const sbft_proposal* p, size_t need, size_t* valid_idx, size_t* n_valid, char* log,
                         size_t log_cap) {
    if (!v || !p || !n_valid || (n && (!votes || !vote_digests || !valid_idx))) return SBFT_GV_EINVAL;
    *n_valid = 0;
    char expected[65];
    v->digest_of(p, expected);
    std::string lg;
    std::vector<size_t> pend;  // arrived, pre-checked votes not verified yet (in arrival order)
    std::unordered_map<uint64_t, bool> seen;
    // one batch call over the pending votes, as go/patches/internal_bft_commits.patch does
    auto run = [&]() -> int {
        std::vector<sbft_signature> batch;
        batch.reserve(pend.size());
        for (size_t i : pend) batch.push_back(votes[i]);
        std::vector<int32_t> st(batch.size());
        std::vector<std::string> why;
        const int rc = v->consenter_batch(batch.data(), batch.size(), p, st.data(), &why);
        if (rc) return rc;
        for (size_t k = 0; k < batch.size(); ++k) {
            if (st[k]) {
                lg += "Couldn't verify " + std::to_string(batch[k].id) + "'s signature: " + why[k] + "\n";
                continue;
            }
            if (*n_valid < need) valid_idx[(*n_valid)++] = pend[k];
        }
        pend.clear();
        return 0;
    };
    for (size_t i = 0; i < n && *n_valid < need; ++i) {  // the quorum complete: the loop returns
        if (seen.count(votes[i].id)) continue;             // voteSet.registerVote: one vote per signer
        seen[votes[i].id] = true;
        if (!vote_digests[i] || std::strcmp(vote_digests[i], expected) != 0) {
            lg += "Got wrong digest at processCommits\n";
            continue;
        }
        pend.push_back(i);
        // enough arrived to complete the quorum if all are valid: verify them as one batch
        if (*n_valid + pend.size() >= need)
            if (const int rc = run()) return rc;
    }
    // arrivals ended with the quorum still short (the library would keep waiting): verify what
    // arrived, so every rejected vote is logged
    if (!pend.empty())
        if (const int rc = run()) return rc;
    if (log && log_cap) {
        const size_t m = std::min(log_cap - 1, lg.size());
        std::memcpy(log, lg.data(), m);
        log[m] = 0;
    }
    return 0;
}

// ---------------------------------------------------------------------- view change (N1)
int sbft_validate_last_decision(sbft_verifier* v, const sbft_proposal* last_decision,
                                const sbft_view_metadata* md, uint64_t next_view, const sbft_signature* sigs,
                                size_t n_sigs, int quorum, uint64_t* last_sequence, char* err, size_t err_cap) {
    if (!v || (n_sigs && !sigs)) return SBFT_GV_EINVAL;
    if (last_sequence) *last_sequence = 0;
    if (!last_decision) {
        put_err(err, err_cap, "the last decision is not set");
        return SBFT_V_EVERIFY;
    }
    if (!md) return 0;  // genesis proposal: no signatures to validate
    if (md->view_id >= next_view) {
        put_err(err, err_cap, "last decision view %llu is greater or equal to requested next view %llu",
                (unsigned long long)md->view_id, (unsigned long long)next_view);
        return SBFT_V_EVERIFY;
    }
    if ((long long)n_sigs < (long long)quorum) {
        put_err(err, err_cap, "there are only %zu last decision signatures", n_sigs);
        return SBFT_V_EVERIFY;
    }
    // dedupe by signer in arrival order (viewchanger.go:700-706), then one launch for all
    std::vector<sbft_signature> batch;
    std::unordered_map<uint64_t, bool> seen;
    for (size_t i = 0; i < n_sigs; ++i) {
        if (seen.count(sigs[i].id)) continue;
        seen[sigs[i].id] = true;
        batch.push_back(sigs[i]);
    }
    std::vector<int32_t> st(batch.size());
    std::vector<std::string> why;
    const int rc = v->consenter_batch(batch.data(), batch.size(), last_decision, st.data(), &why);
    if (rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(rc));
        return rc;
    }
    for (size_t k = 0; k < batch.size(); ++k)
        if (st[k]) {  // the first invalid one in order, as the serial loop reports it
            put_err(err, err_cap, "last decision signature is invalid, error: %s", why[k].c_str());
            return SBFT_V_EVERIFY;
        }
    if ((long long)batch.size() < (long long)quorum) {
        put_err(err, err_cap, "there are only %zu valid last decision signatures", batch.size());
        return SBFT_V_EVERIFY;
    }
    if (last_sequence) *last_sequence = md->latest_sequence;
    return 0;
}

// ---------------------------------------------------------------------- pool prune (N2)
int sbft_pool_prune(sbft_verifier* v, const uint8_t* const* reqs, const size_t* lens, size_t n, size_t* pruned_idx,
                    size_t* n_pruned) {
    if (!v || !n_pruned || (n && (!reqs || !lens || !pruned_idx))) return SBFT_GV_EINVAL;
    *n_pruned = 0;
    std::vector<int32_t> st(n);
    std::vector<Req> parsed;
    const int rc = v->requests_batch(reqs, lens, n, st.data(), parsed);
    if (rc) return rc;
    for (size_t i = 0; i < n; ++i)
        if (st[i]) pruned_idx[(*n_pruned)++] = i;
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------- request batcher (N3)
// Concurrent VerifyRequest callers (Controller.HandleRequest from transport goroutines,
// controller.go:233-246) are coalesced into one launch. No background thread: the first
// caller of an open batch leads it - it waits until the batch is full or its deadline
// passes, closes it, runs one requests_batch launch and wakes the followers. Batches that
// close while another is in flight launch concurrently (the engine is thread-safe).
struct sbft_request_batcher {
    sbft_verifier* v;
    size_t max_batch;
    std::chrono::microseconds max_wait;
    struct Entry {
        const uint8_t* req;
        size_t len;
        int32_t status = 0;
        Req parsed;
    };
    struct Batch {
        std::vector<Entry*> entries;
        bool closed = false;
        int rc = 0;
        std::condition_variable cv;  // wakes the leader when the batch fills
        DoneFlag done;               // wakes the followers when the results are published
    };
    std::mutex mu;
    std::shared_ptr<Batch> open;
    std::atomic<uint64_t> launches{0}, requests{0};
};

extern "C" {

sbft_request_batcher* sbft_request_batcher_new(sbft_verifier* v, size_t max_batch, uint32_t max_wait_us) {
    if (!v || max_batch == 0) return nullptr;
    auto* b = new sbft_request_batcher();
    b->v = v;
    b->max_batch = max_batch;
    b->max_wait = std::chrono::microseconds(max_wait_us);
    return b;
}

void sbft_request_batcher_free(sbft_request_batcher* b) { delete b; }

void sbft_request_batcher_stats(const sbft_request_batcher* b, uint64_t* launches, uint64_t* requests) {
    if (!b) return;
    if (launches) *launches = b->launches.load();
    if (requests) *requests = b->requests.load();
}

int sbft_request_batcher_verify(sbft_request_batcher* b, const uint8_t* req, size_t len, char* info, size_t info_cap,
                                char* err, size_t err_cap) {
    if (!b || (!req && len)) return SBFT_GV_EINVAL;
    if (!req) {  // empty request: malformed (as sbft_verifier_verify_request), no batch taken
        put_err(err, err_cap, "malformed request");
        return SBFT_V_EFORMAT;
    }
    using Batch = sbft_request_batcher::Batch;
    sbft_request_batcher::Entry me;
    me.req = req;
    me.len = len;
    std::shared_ptr<Batch> batch;
    bool leader = false;
    {
        std::unique_lock<std::mutex> g(b->mu);
        if (!b->open) {
            b->open = std::make_shared<Batch>();
            leader = true;
        }
        batch = b->open;
        batch->entries.push_back(&me);
        if (batch->entries.size() >= b->max_batch) {
            batch->closed = true;
            b->open.reset();
            batch->cv.notify_all();  // wakes the leader early
        }
        if (leader) {
            const auto deadline = std::chrono::steady_clock::now() + b->max_wait;
            batch->cv.wait_until(g, deadline, [&] { return batch->closed; });
            if (!batch->closed) {
                batch->closed = true;
                b->open.reset();
            }
        }
    }
    if (!leader) batch->done.wait();
    if (leader) {
        // the batch is closed: nobody else touches its entries until done is published
        const size_t n = batch->entries.size();
        std::vector<const uint8_t*> reqs(n);
        std::vector<size_t> lens(n);
        for (size_t i = 0; i < n; ++i) {
            reqs[i] = batch->entries[i]->req;
            lens[i] = batch->entries[i]->len;
        }
        std::vector<int32_t> st(n);
        std::vector<Req> parsed;
        const int rc = b->v->requests_batch(reqs.data(), lens.data(), n, st.data(), parsed);
        b->launches++;
        b->requests += n;
        for (size_t i = 0; i < n; ++i) {
            batch->entries[i]->status = st[i];
            batch->entries[i]->parsed = std::move(parsed[i]);
        }
        batch->rc = rc;
        batch->done.set();
    }
    if (batch->rc) {
        put_err(err, err_cap, "gpu engine: %s", sbft_gv_strerror(batch->rc));
        return batch->rc;
    }
    if (me.status == SBFT_V_EFORMAT) {
        put_err(err, err_cap, "malformed request");
        return SBFT_V_EFORMAT;
    }
    if (me.status) {
        put_err(err, err_cap, "request %.*s:%.*s has an invalid signature", me.parsed.client_id.n,
                me.parsed.client_id.p, me.parsed.req_id.n, me.parsed.req_id.p);
        return me.status;
    }
    char* w = info;
    if (info && !write_info(w, info + info_cap, me.parsed.client_id, me.parsed.req_id)) return SBFT_V_ESPACE;
    return 0;
}

// ---------------------------------------------------------------------- signer
struct sbft_signer {
    sbft_gv_ctx* ctx;
    uint64_t id;
    uint8_t d[32];
    uint8_t qx[32], qy[32];
    // pre-signature pool (sbft_signer_presign): r and the mod-n factors A = k^-1, B = k^-1 r d
    struct Presig {
        uint8_t r[32];
        sbft::modn::u64 a[4], b[4];
    };
    std::mutex pool_mu;
    std::vector<Presig> pool;
    size_t pool_size = 0;
    ~sbft_signer() {
        std::memset(d, 0, sizeof d);
        for (Presig& p : pool) std::memset(&p, 0, sizeof p);
    }
};

// One launch of 2m signatures over m fresh random nonces: tuple 2i signs e = 0 (s = k^-1 r d
// = B), tuple 2i+1 signs e = 1 (s = k^-1 (1 + r d) = A + B), so A = s(2i+1) - s(2i). Caller
// holds pool_mu.
static int presign_refill(sbft_signer* s, size_t m) {
    std::vector<uint8_t> dd(64 * m), kk(64 * m), ee(64 * m, 0), r(64 * m), sv(64 * m), st(2 * m);
    for (size_t i = 0; i < m; ++i) {
        uint8_t k[32];
        do {  // rejection sampling: 0 < k < n
            size_t got = 0;
            while (got < 32) {
                const ssize_t g = getrandom(k + got, 32 - got, 0);
                if (g <= 0) return SBFT_GV_EDEVICE;
                got += (size_t)g;
            }
        } while (is_zero32(k) || cmp_be32(k, N_BE) >= 0);
        for (int t = 0; t < 2; ++t) {
            std::memcpy(&dd[32 * (2 * i + t)], s->d, 32);
            std::memcpy(&kk[32 * (2 * i + t)], k, 32);
        }
        ee[32 * (2 * i + 1) + 31] = 1;
        std::memset(k, 0, sizeof k);
    }
    const int rc = sbft_gv_sign_p256(s->ctx, dd.data(), kk.data(), ee.data(), 2 * m, nullptr, nullptr, r.data(),
                                     sv.data(), st.data());
    std::memset(kk.data(), 0, kk.size());
    std::memset(dd.data(), 0, dd.size());
    if (rc) return rc;
    // no growth inside the loop: a reallocation would free a buffer still holding
    // pre-signatures (any one reveals d = B / (A r))
    s->pool.reserve(s->pool.size() + m);
    for (size_t i = 0; i < m; ++i) {
        if (!st[2 * i] || !st[2 * i + 1]) continue;  // s came out 0 for this nonce: skip it
        sbft_signer::Presig p;
        std::memcpy(p.r, &r[32 * 2 * i], 32);
        sbft::modn::u64 s0[4], s1[4], neg[4] = {0, 0, 0, 0};
        sbft::modn::from_be32(s0, &sv[32 * 2 * i]);
        sbft::modn::from_be32(s1, &sv[32 * (2 * i + 1)]);
        // A = s1 - s0 = s1 + (n - s0)
        if (!sbft::modn::is_zero(s0)) {
            std::memcpy(neg, sbft::modn::N, sizeof neg);
            sbft::modn::u64 bw = 0;
            for (int j = 0; j < 4; ++j) {
                const unsigned __int128 dlt = (unsigned __int128)neg[j] - s0[j] - bw;
                neg[j] = (sbft::modn::u64)dlt;
                bw = (sbft::modn::u64)(dlt >> 64) & 1u;
            }
        }
        sbft::modn::add_mod(p.a, s1, neg);
        std::memcpy(p.b, s0, sizeof s0);
        s->pool.push_back(p);
        explicit_bzero(&p, sizeof p);
        explicit_bzero(s0, sizeof s0);
        explicit_bzero(s1, sizeof s1);
        explicit_bzero(neg, sizeof neg);
    }
    explicit_bzero(sv.data(), sv.size());
    return 0;
}

sbft_signer* sbft_signer_new(sbft_gv_ctx* ctx, uint64_t id, const uint8_t priv32[32]) {
    if (!ctx || !priv32 || is_zero32(priv32) || cmp_be32(priv32, N_BE) >= 0) return nullptr;
    auto* s = new sbft_signer();
    s->ctx = ctx;
    s->id = id;
    std::memcpy(s->d, priv32, 32);
    uint8_t k[32] = {0}, e[32] = {0}, r[32], sg[32], st = 0;
    k[31] = 1;
    if (sbft_gv_sign_p256(ctx, s->d, k, e, 1, s->qx, s->qy, r, sg, &st) || !st) {
        delete s;
        return nullptr;
    }
    return s;
}
void sbft_signer_free(sbft_signer* s) { delete s; }

int sbft_signer_public_key(const sbft_signer* s, uint8_t pubkey65[65]) {
    if (!s || !pubkey65) return SBFT_GV_EINVAL;
    pubkey65[0] = 0x04;
    std::memcpy(pubkey65 + 1, s->qx, 32);
    std::memcpy(pubkey65 + 33, s->qy, 32);
    return 0;
}

int sbft_signer_presign(sbft_signer* s, size_t pool) {
    if (!s || pool > (1u << 20)) return SBFT_GV_EINVAL;
    std::lock_guard<std::mutex> g(s->pool_mu);
    s->pool_size = pool;
    for (auto& p : s->pool) std::memset(&p, 0, sizeof p);
    s->pool.clear();
    return pool ? presign_refill(s, pool) : 0;
}

int sbft_signer_sign(sbft_signer* s, const uint8_t* data, size_t len, uint8_t sig64[64]) {
    if (!s || (!data && len) || !sig64) return SBFT_GV_EINVAL;
    uint8_t e[32];
    sha256(data ? data : (const uint8_t*)"", len, e);
    {
        std::lock_guard<std::mutex> g(s->pool_mu);
        while (s->pool_size) {  // pooled: s = A e + B (mod n), no launch
            if (s->pool.empty()) {
                const int rc = presign_refill(s, s->pool_size);
                if (rc) return rc;
                if (s->pool.empty()) return SBFT_V_EVERIFY;
            }
            sbft_signer::Presig p = s->pool.back();
            std::memset(&s->pool.back(), 0, sizeof p);
            s->pool.pop_back();
            sbft::modn::u64 ev[4], t[4], sg[4];
            sbft::modn::from_be32(ev, e);
            sbft::modn::mul_mod(t, p.a, ev);
            sbft::modn::add_mod(sg, t, p.b);
            const bool zero = sbft::modn::is_zero(sg);
            if (!zero) {
                std::memcpy(sig64, p.r, 32);
                sbft::modn::to_be32(sig64 + 32, sg);
            }
            explicit_bzero(&p, sizeof p);
            explicit_bzero(t, sizeof t);
            explicit_bzero(sg, sizeof sg);
            if (zero) continue;  // s = 0: take the next nonce
            return 0;
        }
    }
    for (int attempt = 0; attempt < 8; ++attempt) {
        uint8_t k[32], st = 0;
        rfc6979_nonce(s->d, e, attempt, k);
        const int rc = sbft_gv_sign_p256(s->ctx, s->d, k, e, 1, nullptr, nullptr, sig64, sig64 + 32, &st);
        if (rc) return rc;
        if (st) return 0;
    }
    return SBFT_V_EVERIFY;
}

int sbft_signer_sign_proposal(sbft_signer* s, const sbft_proposal* p, const uint8_t* aux, size_t aux_len,
                              uint8_t* msg, size_t msg_cap, size_t* msg_len, uint8_t sig64[64]) {
    if (!s || !p || !msg || !msg_len || (aux_len && !aux)) return SBFT_GV_EINVAL;
    const size_t need = 4 + 2 + 64 + 4 + aux_len;
    if (msg_cap < need) return SBFT_V_ESPACE;
    char digest[65];
    sbft_proposal_digest(p, digest);
    uint8_t* w = msg;
    std::memcpy(w, MSG_MAGIC, 4);
    w += 4;
    *w++ = 64;
    *w++ = 0;
    std::memcpy(w, digest, 64);
    w += 64;
    for (int i = 0; i < 4; ++i) *w++ = (uint8_t)(aux_len >> (8 * i));
    if (aux_len) std::memcpy(w, aux, aux_len);
    *msg_len = need;
    return sbft_signer_sign(s, msg, need, sig64);
}

int64_t sbft_make_request(sbft_signer* client, const char* client_id, const char* req_id, const uint8_t* payload,
                          size_t payload_len, uint8_t* out, size_t out_cap) {
    if (!client || !client_id || !req_id || (payload_len && !payload) || !out) return SBFT_GV_EINVAL;
    const size_t a = std::strlen(client_id), b = std::strlen(req_id);
    if (a > 0xffff || b > 0xffff || payload_len > 0xffffffffu) return SBFT_GV_EINVAL;
    const size_t body = 4 + 2 + a + 2 + b + 4 + payload_len + 65;
    if (out_cap < body + 64) return SBFT_V_ESPACE;
    uint8_t* w = out;
    std::memcpy(w, REQ_MAGIC, 4);
    w += 4;
    *w++ = (uint8_t)a;
    *w++ = (uint8_t)(a >> 8);
    std::memcpy(w, client_id, a);
    w += a;
    *w++ = (uint8_t)b;
    *w++ = (uint8_t)(b >> 8);
    std::memcpy(w, req_id, b);
    w += b;
    for (int i = 0; i < 4; ++i) *w++ = (uint8_t)(payload_len >> (8 * i));
    if (payload_len) std::memcpy(w, payload, payload_len);
    w += payload_len;
    sbft_signer_public_key(client, w);
    w += 65;
    const int rc = sbft_signer_sign(client, out, body, w);
    if (rc) return rc;
    return (int64_t)(body + 64);
}

}  // extern "C"
