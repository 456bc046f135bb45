/*
 * sbft_gpuverify.h — C ABI of libsbft_gpuverify.so, the MI355X signature-verification
 * engine behind SmartBFT's api.Verifier plugin.
 *
 * Drop-in boundary. The reference's plugin interface is Go:
 *   pkg/api/dependencies.go:54-71   type Verifier interface { VerifyProposal, VerifyRequest,
 *                                   VerifyConsenterSig, VerifySignature, VerificationSequence,
 *                                   RequestsFromProposal, AuxiliaryData }
 * and the library calls it at internal/bft/view.go:555 (VerifyProposal), view.go:631 and
 * view.go:834 (VerifyConsenterSig), viewchanger.go:718 and controller.go:239. Every in-tree
 * implementation is an accept-all stub (test/test_app.go:206-253,
 * examples/naive_chain/node.go:64-100); the arithmetic a real plugin runs is Go 1.24.1
 * crypto/ecdsa.Verify (P-256) + crypto/sha256. This header is what a cgo shim binds to
 * replace that arithmetic with one GPU launch per proposal / per quorum (binding in
 * INTEGRATION.md; the plugin-level mirror is include/sbft_verifier.h).
 *
 * Conventions
 *  - Every 256-bit field is 32 bytes big-endian (Go big.Int.FillBytes(make([]byte,32))).
 *  - Batches are structure-of-arrays: field i of tuple k is at ptr + 32*k.
 *  - digest is the hash already normalised as Go's hashToNat consumes it: the first 32
 *    bytes of a hash of >= 32 bytes, a shorter hash left-padded with zeros
 *    (sbft_gv_normalize_hash). r/s/x/y wider than 32 bytes or negative are rejected by
 *    the caller before the call (sbft_gv_normalize_scalar returns 0 for them).
 *  - Verdicts: ok_out[k] = 1 accept, 0 reject — bit-exact with crypto/ecdsa.Verify,
 *    including r/s out of [1, n-1], Q off-curve or non-canonical, R = infinity.
 *  - Return value: 0 on success, negative SBFT_GV_E* on an infrastructure failure
 *    (distinct from a 0 verdict). Host-pointer calls are synchronous; the caller owns all
 *    buffers. A context is thread-safe (calls are serialised per device).
 *  - *_dev entry points take device pointers already resident in HBM on `device` and a
 *    hipStream_t (as void*); they enqueue and return without synchronising.
 */
#ifndef SBFT_GPUVERIFY_H
#define SBFT_GPUVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBFT_GV_OK 0
#define SBFT_GV_EINVAL (-1)     /* bad argument */
#define SBFT_GV_ENODEV (-2)     /* no usable GPU / device mask selects none */
#define SBFT_GV_ENOMEM (-3)     /* device or pinned allocation failed */
#define SBFT_GV_ELAUNCH (-4)    /* kernel launch failed */
#define SBFT_GV_EDEVICE (-5)    /* HIP runtime error during copy/sync */
#define SBFT_GV_ESELFTEST (-6)  /* sbft_gv_init: a device failed the engine's known-answer self-test */

typedef struct sbft_gv_ctx sbft_gv_ctx;

typedef struct sbft_gv_opts {
    uint32_t device_mask;   /* bit d selects HIP device d; 0 = all visible devices */
    uint32_t min_split;     /* batches smaller than this stay on one device (0 = default: 65536, or
                               halfq_max + 1 when the wide half kernel is on) */
    int32_t pair_max;       /* per-device batches of at most this many tuples run the latency kernel
                               (two lanes per tuple); 0 = default SBFT_GV_PAIR_MAX_DEFAULT, < 0 = never
                               (and then no latency kernel at all unless half_max is set explicitly:
                               pair_max < 0 with half_max 0 forces the one-lane throughput kernel) */
    int32_t reserved0;      /* must be 0 */
    uint32_t slots_per_device; /* engine slots per selected device (0 = 1). Each slot owns a stream,
                                  staging, G's comb table and the registered-key tables, and takes
                                  one share of a split batch, exactly as a separate GPU would: with
                                  k > 1 the multi-device split (shares, offset rebasing, verdict
                                  placement, per-device host workers) runs on a single GPU. For
                                  testing the split; a deployment leaves it 0. The environment
                                  variable SBFT_GV_SLOTS_PER_DEVICE overrides it. */
    int32_t half_max;       /* per-device batches of at most this many tuples run the
                               half-size-scalar latency kernel (checked before pair_max): four lanes per tuple, w Q and
                               v R0 as two 128-bit ladders (p256_verify_half_kernel); 0 = default
                               SBFT_GV_HALF_MAX_DEFAULT, < 0 = never. The environment variable
                               SBFT_GV_HALF_MAX overrides it. */
    uint64_t client_table_bytes; /* per-device budget for client-key comb tables
                                    (sbft_gv_register_client_keys; 512 KiB per key and slot):
                                    0 = default, 1/8 of the device's memory (36 GB of the
                                    MI355X's 288 GB, ~70,000 clients); the environment variable
                                    SBFT_GV_CLIENT_TABLE_BYTES overrides it. Keys past the
                                    budget stay unregistered (their requests take the generic
                                    launch, same verdicts), so client registration can never
                                    use the memory the verify paths stage in. */
    int32_t halfq_max;      /* per-device batches of at most this many tuples run the wide form of the
                               half-size-scalar kernel (eight lanes per tuple: each 128-bit ladder on a
                               quad, 15 steps per 4-bit digit instead of 21; checked before half_max),
                               sized so that its workgroups fit one per CU; 0 = default, 24 x the
                               device's CUs (6,144 on an MI355X), < 0 = never. The environment variable
                               SBFT_GV_HALFQ_MAX overrides it. With more than one slot and the default
                               min_split, a batch larger than this is split, so that each share runs
                               the wide kernel (a 10k proposal over 2-8 GPUs). */
    int32_t reserved1;      /* must be 0 */
} sbft_gv_opts;

#define SBFT_GV_PAIR_MAX_DEFAULT 32768u
/* The device-resident hash entry points (sbft_gv_sha256_dev, sbft_gv_sha256_verify_p256_dev)
 * read no byte outside the 16-byte-aligned granules that hold message bytes (the hash kernel
 * moves whole 16-B pieces into LDS and clamps every piece past a message's last granule onto
 * it), so a blob sized exactly to its messages is safe. The host-buffer entry points stage the
 * blob with this much slack, which the hash-measurement variants selected by SBFT_SHA_VARIANT
 * (per-lane 68-byte block loads) need. */
#define SBFT_GV_SHA_BLOB_PAD 256u
#define SBFT_GV_HALF_MAX_DEFAULT 12288u

/* Create a context (per-device stream + device/pinned staging grown on demand).
 * opts may be NULL. Replaces: the plugin construction a Go app does before handing its
 * Verifier to consensus.Consensus.Verifier (pkg/consensus/consensus.go:36). */
int sbft_gv_init(const sbft_gv_opts* opts, sbft_gv_ctx** out);
void sbft_gv_destroy(sbft_gv_ctx* ctx);
/* Number of engine slots: the selected devices times slots_per_device. A host-buffer batch is
 * split over this many shares. */
int sbft_gv_device_count(const sbft_gv_ctx* ctx);
/* The host-side batch split every host-buffer call uses (no GPU; pure arithmetic, exported so
 * the split is testable without devices): a batch of n >= min_split (0 = 65536) tuples on
 * n_devices devices is cut into contiguous shares [begin[i], begin[i] + count[i]) that differ
 * by at most one tuple, one per device in device order; a smaller batch stays whole on one
 * device. begin / count hold n_devices entries; returns the number of shares. There is no
 * collective: every tuple is independent. */
size_t sbft_gv_plan_split(size_t n, size_t n_devices, size_t min_split, size_t* begin, size_t* count);
const char* sbft_gv_strerror(int code);

/* Batched P-256 ECDSA verify, host buffers, synchronous. Split over the context's devices
 * for n >= min_split. Replaces n calls of crypto/ecdsa.Verify made by a Verifier inside
 * VerifyProposal (view.go:555) / VerifyConsenterSig (view.go:631, :834). */
int sbft_gv_verify_p256(sbft_gv_ctx* ctx, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                        const uint8_t* qx, const uint8_t* qy, size_t n, uint8_t* ok_out);
/* sbft_gv_verify_p256 on a named kernel instead of the one the batch size selects (tests and
 * diagnostics; same verdicts whichever kernel runs): SBFT_GV_KERNEL_THROUGHPUT (one lane per
 * tuple), _PAIR (two lanes), _HALF (half-size scalars, four lanes), _HALF_WIDE (half-size
 * scalars, eight lanes: a quad per ladder), or _EXACT: every tuple
 * through the exact case-split kernel alone -- the net the others hand flagged tuples to
 * (Booth digits, explicit infinity and doubling branches; slow, one lane per tuple). */
#define SBFT_GV_KERNEL_EXACT 0
#define SBFT_GV_KERNEL_THROUGHPUT 1
#define SBFT_GV_KERNEL_PAIR 2
#define SBFT_GV_KERNEL_HALF 3
#define SBFT_GV_KERNEL_HALF_WIDE 4
int sbft_gv_verify_p256_kernel(sbft_gv_ctx* ctx, int kernel, const uint8_t* digest, const uint8_t* r,
                               const uint8_t* s, const uint8_t* qx, const uint8_t* qy, size_t n, uint8_t* ok_out);

/* Page-locked host memory, visible to every device of the process (hipHostMalloc, portable).
 * When all five input arrays of sbft_gv_verify_p256 live in such memory and a device's share
 * is large, the call overlaps the H2D copies of later sub-batches with the verify kernels of
 * earlier ones (a cgo caller allocates its batch buffers here instead of on the Go heap).
 * No reference counterpart: Go's heap memory is pageable. */
int sbft_gv_host_alloc(size_t bytes, void** out);
void sbft_gv_host_free(void* p);

/* Batched SHA-256 over variable-length messages: message k = blob[off[k] .. off[k]+len[k]).
 * Replaces crypto/sha256.Sum256 per request payload. */
int sbft_gv_sha256(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                   const uint32_t* len, size_t n, uint8_t* dig_out);

/* Fused: digest_k = SHA-256(message k) stays on the GPU and feeds the verify of tuple k.
 * dig_out may be NULL. */
int sbft_gv_sha256_verify_p256(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len,
                               const uint64_t* off, const uint32_t* len, const uint8_t* r,
                               const uint8_t* s, const uint8_t* qx, const uint8_t* qy, size_t n,
                               uint8_t* ok_out, uint8_t* dig_out);

/* Fused hash + verify of framed messages, whose tuples live inside the blob: message k is
 * blob[off[k], off[k] + len[k]), its signature r || s the 64 bytes at off[k] + len[k] + sig_rel
 * and its public key x || y the 64 bytes at off[k] + len[k] + pub_rel (both inside the blob,
 * else SBFT_GV_EINVAL). The device gathers the verify inputs itself, so only the blob and the
 * offsets cross PCIe. For the signed-request format of sbft_verifier.h (public key at the end
 * of the signed body, signature right after it): sig_rel = 0, pub_rel = -64.
 * Replaces: the per-request loop of an api.Verifier's VerifyProposal (pkg/api/dependencies.go:56). */
int sbft_gv_sha256_verify_p256_framed(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len,
                                      const uint64_t* off, const uint32_t* len, size_t n, int32_t sig_rel,
                                      int32_t pub_rel, uint8_t* ok_out);

/* Streamed hash + verify of a batch far larger than one launch (BASELINE config 5: requests
 * with 1-64 KiB payloads, hashed on the GPU, then verified). Same inputs and outputs as
 * sbft_gv_sha256_verify_p256 (dig_out may be NULL). Each device takes a contiguous share of the
 * messages (sbft_gv_plan_split) on a host thread of its own and streams it in windows of about
 * window_bytes of payload (0 = 256 MiB) through six staging buffers: up to six windows hash
 * and verify concurrently (each on a stream of its own: hashing is serial within a message, so
 * one window alone leaves most CUs idle) while the host thread stages and copies the next.
 * Windows whose messages
 * lie densely in the blob are DMA'd in place (at the full PCIe rate when the blob is in
 * page-locked memory, sbft_gv_host_alloc); scattered ones are gathered on the host first.
 * Digests never leave the device unless dig_out is given.
 * Replaces: per-request crypto/sha256 + crypto/ecdsa.Verify in an api.Verifier's
 * VerifyRequest for requests of up to RequestMaxBytes (pkg/types/config.go:111) arriving
 * through Controller.HandleRequest (internal/bft/controller.go:233-246). */
int sbft_gv_sha256_verify_p256_stream(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len,
                                      const uint64_t* off, const uint32_t* len, const uint8_t* r,
                                      const uint8_t* s, const uint8_t* qx, const uint8_t* qy, size_t n,
                                      size_t window_bytes, uint8_t* ok_out, uint8_t* dig_out);

/* Bytes of device workspace the verify pipeline uses for a batch of n tuples (fixup list +
 * batched-inversion arrays, ~65 B per tuple). The device-resident entry points keep one such
 * workspace per caller stream inside the context. */
size_t sbft_gv_verify_workspace_bytes(size_t n);

/* Device-resident variants (inputs already in HBM on `device`; stream = hipStream_t). */
int sbft_gv_verify_p256_dev(sbft_gv_ctx* ctx, int device, const void* d_digest, const void* d_r,
                            const void* d_s, const void* d_qx, const void* d_qy, size_t n,
                            void* d_ok, void* stream);
/* d_order (may be NULL): u32 permutation of [0, n): the messages are taken in that sequence.
 * NULL (index order) is the fast choice: the kernel load-balances messages of any lengths over
 * its lanes and index order keeps each wavefront's streams adjacent in memory. Digests land at
 * their message's index either way. */
int sbft_gv_sha256_dev(sbft_gv_ctx* ctx, int device, const void* d_blob, const void* d_off,
                       const void* d_len, const void* d_order, size_t n, void* d_dig, void* stream);
int sbft_gv_sha256_verify_p256_dev(sbft_gv_ctx* ctx, int device, const void* d_blob,
                                   const void* d_off, const void* d_len, const void* d_order,
                                   const void* d_r, const void* d_s, const void* d_qx,
                                   const void* d_qy, size_t n, void* d_ok, void* d_dig,
                                   void* stream);

/* Batched key derivation + ECDSA signing with caller-supplied nonces (the api.Signer side,
 * pkg/api/dependencies.go:46-52; also the synthetic-workload generator). For each k:
 * Q = d*G (qx, qy), r = x(k*G) mod n, s = k^-1 (digest + r d) mod n; status[k] = 1 on
 * success, 0 if d or k is outside [1, n-1] or r or s came out 0. qx = qy = NULL skips the key
 * derivation (a signer that knows its public key; the latency path then runs one scalar
 * multiplication instead of two). Nonces must be secret and unique per key (RFC 6979 or a
 * CSPRNG) — the engine does not generate them. */
int sbft_gv_sign_p256(sbft_gv_ctx* ctx, const uint8_t* d, const uint8_t* k, const uint8_t* digest,
                      size_t n, uint8_t* qx, uint8_t* qy, uint8_t* r, uint8_t* s, uint8_t* status);
int sbft_gv_sign_p256_dev(sbft_gv_ctx* ctx, int device, const void* d_d, const void* d_k,
                          const void* d_digest, size_t n, void* d_qx, void* d_qy, void* d_r,
                          void* d_s, void* d_status, void* stream);

/* Registered keys (fixed-base comb tables; smartbft_amd/csrc/p256_keyed.hip).
 * Precomputes table[w][j] = j 2^(8w) Q (32 x 256 affine points, 512 KiB of HBM per key and
 * device) so a signature under this key verifies with 64 table lookups and no doublings.
 * Meant for the consenter keys of the configuration, which every VerifyConsenterSig /
 * VerifySignature call checks against (view.go:631, :834; viewchanger.go:598, :718): the
 * plugin registers them when it learns the membership (sbft_verifier_add_consenter).
 * Returns SBFT_GV_EINVAL for a key that is not a valid P-256 point (such a key can only
 * fail verification: use the unkeyed calls, which reject it). Registering the same key
 * twice returns the same id. Ids start at 1. */
int sbft_gv_register_key(sbft_gv_ctx* ctx, const uint8_t qx[32], const uint8_t qy[32], uint32_t* key_id);
/* Batch form: n keys (qx, qy: n x 32 bytes big-endian), their comb tables built in one launch
 * per device (a client-key registry: 10,000 keys = 5 GB of tables). key_ids[i] receives the
 * key's id, or 0 if it is not a point on the curve. Keys registered before keep their id.
 * Returns a negative SBFT_GV_E* only on an engine failure (nothing is registered then). */
int sbft_gv_register_keys(sbft_gv_ctx* ctx, const uint8_t* qx, const uint8_t* qy, size_t n, uint32_t* key_ids);
/* Client-key registry form of sbft_gv_register_keys, under a memory budget: new keys are
 * registered in order while their tables fit both sbft_gv_opts.client_table_bytes and the
 * headroom every device keeps free for staging (SBFT_GV_HBM_RESERVE bytes, or 1/32 of the
 * device's memory if larger); the rest get key_ids[i] = 0 (unregistered: the generic verify
 * paths take their requests, with the same verdicts). *registered (may be NULL) receives the
 * number of keys of this call that hold an id. A budget that is spent is not an error: this
 * returns a negative SBFT_GV_E* only on an engine failure (nothing is registered then). */
#define SBFT_GV_HBM_RESERVE (8ull << 30)
int sbft_gv_register_client_keys(sbft_gv_ctx* ctx, const uint8_t* qx, const uint8_t* qy, size_t n,
                                 uint32_t* key_ids, size_t* registered);

/* Verify n tuples (digest, r, s) against registered keys key_id[k]. Same verdict semantics
 * as sbft_gv_verify_p256 (an unknown key id verifies false). Small batches run one
 * wavefront per signature (latency path: one H2D, one launch, one D2H). */
int sbft_gv_verify_p256_keyed(sbft_gv_ctx* ctx, const uint8_t* digest, const uint8_t* r, const uint8_t* s,
                              const uint32_t* key_id, size_t n, uint8_t* ok_out);
/* Same with digest_k = SHA-256(blob[off[k] .. off[k]+len[k])) computed inside the launch
 * (consenter Signature.Msg hashing, A5 in SURVEY.md 8(a)). */
int sbft_gv_sha256_verify_p256_keyed(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len, const uint64_t* off,
                                     const uint32_t* len, const uint8_t* r, const uint8_t* s, const uint32_t* key_id,
                                     size_t n, uint8_t* ok_out);

/* Kernel timing (measurement): while enabled, every device-resident verify records HIP
 * events on the caller's stream around its main p256_verify_kernel launch (not the s^-1
 * batching or fixup kernels), and so do the latency paths around their one launch: the fused
 * hash + verify kernel of a one-slot VerifyProposal (sbft_verifier_verify_proposal), its
 * registered-client keyed launch, and the keyed launches of VerifyConsenterSig(s) (with a hash
 * kernel in front where the batch carries messages). sbft_gv_kernel_time waits for the recorded
 * events and returns (then forgets) the number of timed launches and their summed duration in
 * milliseconds. */
int sbft_gv_kernel_timing(sbft_gv_ctx* ctx, int enable);
int sbft_gv_kernel_time(sbft_gv_ctx* ctx, uint64_t* launches, double* ms);

/* Element-wise self-test of the device primitives (diagnostics; op codes in
 * smartbft_amd/csrc/p256_selftest.hip). a, b, out: n x 32 bytes big-endian. */
int sbft_gv_selftest_field(sbft_gv_ctx* ctx, int op, const uint8_t* a, const uint8_t* b, size_t n,
                           uint8_t* out);

/* Fault injection (tests of the error paths; not for production use). Arms a process-wide fault
 * of `kind`: its next `count` fault points fail (count < 0: every one until disarmed with
 * SBFT_GV_FAULT_OFF) as the runtime would fail there -- the staging allocations return
 * SBFT_GV_ENOMEM, the kernel launchers fail before launching (SBFT_GV_ELAUNCH), the checked
 * stream synchronisations report SBFT_GV_EDEVICE once the work has drained. Every entry point
 * must then return the negative SBFT_GV_E* code (never a verdict) and the context stays usable:
 * the next call after disarming succeeds. Contexts created while a fault is armed fail their
 * self-test, so arm after sbft_gv_init. Arming prints a warning on stderr. In a library built
 * with -DSBFT_FAULT_INJECTION (test builds only) the environment variable
 * SBFT_GV_FAULT=nomem|launch|sync[:count] arms one at the end of sbft_gv_init. Returns 0, or
 * SBFT_GV_EINVAL for an unknown kind. */
#define SBFT_GV_FAULT_OFF 0
#define SBFT_GV_FAULT_NOMEM 1
#define SBFT_GV_FAULT_LAUNCH 2
#define SBFT_GV_FAULT_SYNC 3
int sbft_gv_inject_fault(int kind, int count);

/* Go-semantics host helpers (no GPU). */
void sbft_gv_normalize_hash(const uint8_t* hash, size_t len, uint8_t out32[32]);
/* Big-endian magnitude of arbitrary length -> 32 bytes; returns 0 if it needs > 256 bits. */
int sbft_gv_normalize_scalar(const uint8_t* be, size_t len, uint8_t out32[32]);

#ifdef __cplusplus
}
#endif
#endif
