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
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/sbft_gpuverify.h"
#include "sbft_kernels.h"

namespace {

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

    int reserve(size_t bytes) {
        if (bytes <= dcap) return SBFT_GV_OK;
        if (dbuf) (void)hipFree(dbuf);
        dbuf = nullptr;
        dcap = 0;
        size_t want = std::max(bytes, (size_t)1 << 20);
        want = (want + 4095) & ~(size_t)4095;
        if (hipMalloc(&dbuf, want) != hipSuccess) return SBFT_GV_ENOMEM;
        dcap = want;
        return SBFT_GV_OK;
    }
};

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct sbft_gv_ctx {
    std::vector<Slot*> slots;
    uint32_t min_split = 65536;
    std::atomic<uint32_t> rr{0};
};

extern "C" {

const char* sbft_gv_strerror(int code) {
    switch (code) {
    case SBFT_GV_OK: return "ok";
    case SBFT_GV_EINVAL: return "invalid argument";
    case SBFT_GV_ENODEV: return "no usable GPU";
    case SBFT_GV_ENOMEM: return "allocation failed";
    case SBFT_GV_ELAUNCH: return "kernel launch failed";
    case SBFT_GV_EDEVICE: return "HIP runtime error";
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
    if (opts && opts->min_split) ctx->min_split = opts->min_split;
    for (int d = 0; d < ndev && d < 32; ++d) {
        if (!(mask & (1u << d))) continue;
        auto* s = new Slot();
        s->device = d;
        if (hipSetDevice(d) != hipSuccess ||
            hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
            delete s;
            continue;
        }
        ctx->slots.push_back(s);
    }
    if (ctx->slots.empty()) {
        delete ctx;
        return SBFT_GV_ENODEV;
    }
    *out = ctx;
    return SBFT_GV_OK;
}

void sbft_gv_destroy(sbft_gv_ctx* ctx) {
    if (!ctx) return;
    for (Slot* s : ctx->slots) {
        (void)hipSetDevice(s->device);
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (s->dbuf) (void)hipFree(s->dbuf);
        for (auto& kv : s->ws) {
            (void)hipStreamSynchronize(kv.first);
            if (kv.second.ptr) (void)hipFree(kv.second.ptr);
        }
        if (s->stream) (void)hipStreamDestroy(s->stream);
        delete s;
    }
    delete ctx;
}

size_t sbft_gv_verify_workspace_bytes(size_t n) { return sbft_verify_work_bytes(n); }

int sbft_gv_device_count(const sbft_gv_ctx* ctx) { return ctx ? (int)ctx->slots.size() : 0; }

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
    uint32_t* work = sl->stream_workspace((hipStream_t)stream, sbft_verify_work_bytes(n));
    if (!work) return SBFT_GV_ENOMEM;
    return sbft_launch_p256_verify((const uint8_t*)d_digest, (const uint8_t*)d_r, (const uint8_t*)d_s,
                                   (const uint8_t*)d_qx, (const uint8_t*)d_qy, (uint8_t*)d_ok,
                                   (uint32_t)n, work, (hipStream_t)stream)
               ? SBFT_GV_ELAUNCH
               : SBFT_GV_OK;
}

int sbft_gv_sha256_dev(sbft_gv_ctx* ctx, int device, const void* d_blob, const void* d_off,
                       const void* d_len, const void* d_order, size_t n, void* d_dig, void* stream) {
    if (!ctx || (n && (!d_blob || !d_off || !d_len || !d_dig))) return SBFT_GV_EINVAL;
    if (n > 0xffffffffu) return SBFT_GV_EINVAL;
    if (!slot_for(ctx, device)) return SBFT_GV_ENODEV;
    if (hipSetDevice(device) != hipSuccess) return SBFT_GV_EDEVICE;
    return sbft_launch_sha256((const uint8_t*)d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len,
                              (const uint32_t*)d_order, (uint8_t*)d_dig, (uint32_t)n, (hipStream_t)stream)
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
};

std::vector<Chunk> plan(sbft_gv_ctx* ctx, size_t n) {
    std::vector<Chunk> out;
    const size_t nd = ctx->slots.size();
    if (n < ctx->min_split || nd == 1) {
        const uint32_t k = ctx->rr.fetch_add(1) % nd;
        out.push_back({ctx->slots[k], 0, n});
        return out;
    }
    for (size_t d = 0; d < nd; ++d) {
        const size_t b = n * d / nd, e = n * (d + 1) / nd;
        if (e > b) out.push_back({ctx->slots[d], b, e - b});
    }
    return out;
}

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return SBFT_GV_EDEVICE; \
    } while (0)

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
    uint8_t* base = sl->dbuf;
    uint32_t* work = (uint32_t*)(base + 5 * f + fo);
    const uint8_t* src[5] = {digest, r, s, qx, qy};
    for (int k = 0; k < 5; ++k)
        HIPCHK(hipMemcpyAsync(base + k * f, src[k] + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice,
                              sl->stream));
    if (sbft_launch_p256_verify(base, base + f, base + 2 * f, base + 3 * f, base + 4 * f, base + 5 * f,
                                (uint32_t)c.count, work, sl->stream))
        return SBFT_GV_ELAUNCH;
    HIPCHK(hipMemcpyAsync(ok_out + c.begin, base + 5 * f, c.count, hipMemcpyDeviceToHost, sl->stream));
    return SBFT_GV_OK;
}

// Hash (and optionally verify) messages [c.begin, +c.count). Offsets are rebased to the
// chunk's first message so each device receives only its slice of the blob.
int enqueue_hash(const Chunk& c, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                 const uint32_t* len, const uint8_t* r, const uint8_t* s, const uint8_t* qx,
                 const uint8_t* qy, uint8_t* ok_out, uint8_t* dig_out, std::vector<uint64_t>& rebased) {
    Slot* sl = c.slot;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t k = c.begin; k < c.begin + c.count; ++k) {
        if (off[k] + len[k] > blob_len) return SBFT_GV_EINVAL;
        lo = std::min(lo, off[k]);
        hi = std::max(hi, off[k] + len[k]);
    }
    if (c.count == 0) return SBFT_GV_OK;
    rebased.resize(c.count);
    for (size_t k = 0; k < c.count; ++k) rebased[k] = off[c.begin + k] - lo;
    // lanes take messages in length order (descending) so each wavefront's lanes finish together
    std::vector<uint32_t> order(c.count);
    for (size_t k = 0; k < c.count; ++k) order[k] = (uint32_t)k;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return len[c.begin + a] > len[c.begin + b]; });
    const size_t span = hi - lo;
    const size_t fb = align_up(span + 128, 256);  // funnel over-read padding
    const size_t fo = align_up(8 * c.count, 256), fl = align_up(4 * c.count, 256);
    const size_t fd = align_up(32 * c.count, 256);
    const bool verify = ok_out != nullptr;
    const size_t need = fb + fo + 2 * fl + fd +
                        (verify ? 4 * fd + align_up(c.count, 256) + sbft_verify_work_bytes(c.count) : 0);
    HIPCHK(hipSetDevice(sl->device));
    int rc = sl->reserve(need);
    if (rc) return rc;
    uint8_t* b = sl->dbuf;
    uint8_t *d_blob = b, *d_off = b + fb, *d_len = d_off + fo, *d_order = d_len + fl, *d_dig = d_order + fl;
    HIPCHK(hipMemcpyAsync(d_blob, blob + lo, span, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(d_off, rebased.data(), 8 * c.count, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(d_len, len + c.begin, 4 * c.count, hipMemcpyHostToDevice, sl->stream));
    HIPCHK(hipMemcpyAsync(d_order, order.data(), 4 * c.count, hipMemcpyHostToDevice, sl->stream));
    // pageable-source copies are staged before hipMemcpyAsync returns, so `order` may go out
    // of scope; `rebased` is owned by the caller until the stream is synchronised anyway.
    if (sbft_launch_sha256(d_blob, (const uint64_t*)d_off, (const uint32_t*)d_len,
                           (const uint32_t*)d_order, d_dig, (uint32_t)c.count, sl->stream))
        return SBFT_GV_ELAUNCH;
    if (verify) {
        uint8_t* v = d_dig + fd;
        const uint8_t* src[4] = {r, s, qx, qy};
        for (int k = 0; k < 4; ++k)
            HIPCHK(hipMemcpyAsync(v + k * fd, src[k] + 32 * c.begin, 32 * c.count, hipMemcpyHostToDevice,
                                  sl->stream));
        uint8_t* d_ok = v + 4 * fd;
        uint32_t* work = (uint32_t*)(d_ok + align_up(c.count, 256));
        if (sbft_launch_p256_verify(d_dig, v, v + fd, v + 2 * fd, v + 3 * fd, d_ok, (uint32_t)c.count,
                                    work, sl->stream))
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

template <class F>
int run_chunks(sbft_gv_ctx* ctx, size_t n, F&& enqueue) {
    std::vector<Chunk> chunks = plan(ctx, n);
    std::vector<std::unique_lock<std::mutex>> locks;
    locks.reserve(chunks.size());
    for (auto& c : chunks) locks.emplace_back(c.slot->mu);
    int rc = SBFT_GV_OK;
    for (size_t i = 0; i < chunks.size() && rc == SBFT_GV_OK; ++i) rc = enqueue(chunks[i], i);
    for (auto& c : chunks) {
        (void)hipSetDevice(c.slot->device);
        if (hipStreamSynchronize(c.slot->stream) != hipSuccess && rc == SBFT_GV_OK) rc = SBFT_GV_EDEVICE;
    }
    return rc;
}

}  // namespace

extern "C" {

int sbft_gv_verify_p256(sbft_gv_ctx* ctx, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                        const uint8_t* qx, const uint8_t* qy, size_t n, uint8_t* ok_out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!digest || !r || !s || !qx || !qy || !ok_out || n > 0xffffffffu) return SBFT_GV_EINVAL;
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) {
        return enqueue_verify(c, digest, r, s, qx, qy, ok_out);
    });
}

int sbft_gv_sign_p256(sbft_gv_ctx* ctx, const uint8_t* d, const uint8_t* k, const uint8_t* digest,
                      size_t n, uint8_t* qx, uint8_t* qy, uint8_t* r, uint8_t* s, uint8_t* status) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!d || !k || !digest || !qx || !qy || !r || !s || !status || n > 0xffffffffu) return SBFT_GV_EINVAL;
    return run_chunks(ctx, n, [&](const Chunk& c, size_t) {
        return enqueue_sign(c, d, k, digest, qx, qy, r, s, status);
    });
}

int sbft_gv_selftest_field(sbft_gv_ctx* ctx, int op, const uint8_t* a, const uint8_t* b, size_t n,
                           uint8_t* out) {
    if (!ctx) return SBFT_GV_EINVAL;
    if (n == 0) return SBFT_GV_OK;
    if (!a || !b || !out || op < 0 || op > 9 || n > 0xffffffffu) return SBFT_GV_EINVAL;
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

}  // extern "C"
