// sbft_kernels.h — internal launcher declarations shared by the HIP kernels and the
// host runtime (gpuverify.cpp). Not part of the public C ABI (include/sbft_gpuverify.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// Device workspace the verify pipeline needs for n tuples (see sbft_launch_p256_verify):
// fixup counter + list (4(n+1) B, rounded to 256), then the batched-inversion arrays
// pre | suf (32 B per tuple) and tot | kb (32 B per 1,024-tuple s^-1 group). tot | kb are
// sized per 256 tuples (an over-allocation of 48 B per 1,024 tuples, kept so the workspace
// formula, and so sbft_gv_verify_workspace_bytes, did not change with the group size). Then,
// 256-aligned, the throughput kernel's per-lane Q tables: 2^(w-1) affine entries x 80 B per
// tuple (SBFT_VERIFY_QTAB_BYTES; w = SBFT_TQWIN, p256_verify.hip kTWin: 640 B at w = 4). The size is computed by the object that
// holds the kernel (sbft_verify_work_bytes below), so a -DSBFT_TQWIN build of p256_verify.hip
// alone sizes its own workspace.
#ifndef SBFT_TQWIN
#define SBFT_TQWIN 4
#endif
#define SBFT_VERIFY_QTAB_BYTES (80 << (SBFT_TQWIN - 1))

// Test-only fault injection (gpuverify.cpp, sbft_gv_inject_fault): nonzero when the armed fault
// of this kind fires at this pass. The launchers below return failure then, before launching.
extern "C" int sbft_fault_hit(int kind);

extern "C" {
// bytes of device workspace one sbft_launch_p256_verify call of n tuples needs
size_t sbft_verify_work_bytes(size_t n);
// P-256 verify of n SoA tuples (32-byte big-endian fields) -> n verdict bytes.
// d_work: device workspace of sbft_verify_work_bytes(n) bytes, private to the stream.
// d_gcomb: the device's fixed-base comb table for u1*G (sbft_gcomb_table_bytes() bytes, built
// once by sbft_launch_gcomb_build; unused when that size is 0).
// ev0/ev1 (may be NULL): events recorded on the stream right before / after the main
// verify kernel (kernel timing, sbft_gv_kernel_time). lanes: 1 = the one-lane throughput
// kernel, 2 = the pair latency kernel (p256_verify_small_kernel<2>), 3 = the half-size-scalar
// kernel (p256_verify_half_kernel), 0 = every tuple through the exact case-split fixup kernel
// alone (the net the others hand flagged tuples to; the self-test and tests exercise it this way).
int sbft_launch_p256_verify(const uint8_t* d_digest, const uint8_t* d_r, const uint8_t* d_s,
                            const uint8_t* d_qx, const uint8_t* d_qy, uint8_t* d_ok, uint32_t n,
                            uint32_t* d_work, const void* d_gcomb, hipStream_t stream,
                            hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, int lanes = 1,
                            int work_zeroed = 0);  // 1: the caller has zeroed d_work's first word
// Framed tuples (message k = blob[off[k], off[k]+len[k]), r||s at its end + sig_rel, Qx||Qy at
// its end + pub_rel; the blob readable SBFT_GV_SHA_BLOB_PAD bytes past its end) on the
// small-batch kernel, lanes 2 or 4: SHA-256 and verify in one launch, then the fixup. d_dig ..
// d_qy: 32n-byte rows each (written only for tuples the fixup recomputes). d_work's first word
// must be zero (sbft_launch_gather_framed's zero0 can clear it).
int sbft_launch_p256_verify_framed(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len, uint32_t n,
                                   int32_t sig_rel, int32_t pub_rel, uint8_t* d_dig, uint8_t* d_r, uint8_t* d_s,
                                   uint8_t* d_qx, uint8_t* d_qy, uint8_t* d_ok, uint32_t* d_work,
                                   const void* d_gcomb, hipStream_t stream, int lanes,
                                   uint32_t* h_flagged = nullptr);
// h_flagged (mapped host memory, zeroed by the caller): when given, the fixup kernel is not
// launched; the verify kernel sets *h_flagged = 1 if it flagged a tuple, and the caller then
// runs sbft_launch_p256_verify_fixup (same arguments) after its synchronisation.
int sbft_launch_p256_verify_fixup(const uint8_t* d_dig, const uint8_t* d_r, const uint8_t* d_s, const uint8_t* d_qx,
                                  const uint8_t* d_qy, uint8_t* d_ok, const uint32_t* d_work, uint32_t n,
                                  hipStream_t stream);
size_t sbft_gcomb_table_bytes(void);
int sbft_launch_gcomb_build(void* d_table, hipStream_t stream);
// SHA-256 of n messages blob[off[k] .. off[k]+len[k]); the blob must be readable
// SBFT_GV_SHA_BLOB_PAD (256) bytes past its last message (whole-step LDS-DMA over-read). Digests are 32-byte big-endian. d_order (may be
// NULL): the messages are taken in the order d_order[0], d_order[1], ... (load-balanced;
// NULL = index order, which keeps each wavefront's streams adjacent in memory). d_ctr: one
// device u32 of scratch private to the stream (zeroed by the launch).
int sbft_launch_sha256(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                       const uint32_t* d_order, uint8_t* d_dig, uint32_t n, uint32_t* d_ctr, hipStream_t stream,
                       int ctr_zeroed = 0);  // 1: the caller has zeroed *d_ctr (no memset launch)
// Longest-first message order for sbft_launch_sha256 (d_order): a counting sort of the lengths
// over 128 length classes. d_ws: sbft_sha256_lpt_ws_bytes() of device scratch private to the
// stream; d_order: n u32 indices. Worth it for large batches of unequal lengths (config 5).
size_t sbft_sha256_lpt_ws_bytes(void);
int sbft_launch_sha256_lpt_order(const uint32_t* d_len, uint32_t n, uint32_t* d_ws, uint32_t* d_order,
                                 hipStream_t stream);
// SoA verify inputs (32-byte fields, 16-B aligned outputs) gathered from framed messages in
// the blob: r || s at off[k] + len[k] + sig_rel, x || y at off[k] + len[k] + pub_rel (the
// caller has bounds-checked both against the blob).
// zero0 / zero1 (may be NULL): device u32s the launch sets to 0 (the counters of the hash and
// verify launches that follow on the stream, so they need no memset launches of their own).
int sbft_launch_gather_framed(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len, uint32_t n,
                              int32_t sig_rel, int32_t pub_rel, uint8_t* d_r, uint8_t* d_s, uint8_t* d_qx,
                              uint8_t* d_qy, hipStream_t stream, uint32_t* zero0 = nullptr,
                              uint32_t* zero1 = nullptr);
// Key derivation + ECDSA sign with caller nonces: Q = d*G, (r, s); status 1 = ok.
int sbft_launch_p256_sign(const uint8_t* d_d, const uint8_t* d_k, const uint8_t* d_e, uint8_t* d_qx,
                          uint8_t* d_qy, uint8_t* d_r, uint8_t* d_s, uint8_t* d_status, uint32_t n,
                          hipStream_t stream);
// Element-wise primitive self-test (see p256_selftest.hip for op codes).
int sbft_launch_selftest(int op, const uint8_t* d_a, const uint8_t* d_b, uint8_t* d_out, uint32_t n,
                         hipStream_t stream);
}

extern "C" {
// Registered-key (comb table) path, p256_keyed.hip.
size_t sbft_comb_table_bytes(void);
// table[w][j] = j 2^(8w) Q for the key (qx, qy) (32-byte big-endian, device memory);
// d_status[0] = 1 iff the key is valid.
// Latency-path signing, one wavefront per signature over G's comb table (keytab[0]); same
// outputs as sbft_launch_p256_sign.
int sbft_launch_p256_sign_wave(const uint8_t* d_d, const uint8_t* d_k, const uint8_t* d_e,
                               const void* const* d_keytab, uint8_t* d_qx, uint8_t* d_qy, uint8_t* d_r,
                               uint8_t* d_s, uint8_t* d_status, uint32_t n, hipStream_t stream);
int sbft_launch_comb_build(const uint8_t* d_qx, const uint8_t* d_qy, void* d_tables, uint32_t* d_status,
                           uint32_t nk, hipStream_t stream);
// Verify n tuples against registered keys: d_key[t] in [1, nkeys) indexes d_keytab (slot 0 = G).
// Either d_digest (n x 32 B) or the messages (d_blob, d_off, d_len) hashed in the launch.
// d_ok[t] = verdict (0/1) | mark: a nonzero mark lets a host polling d_ok in mapped memory see
// each verdict land (the zero-copy latency path).
// Large batches against registered keys (p256_verify.hip): four lanes per signature, each
// lane inverting s itself; digests precomputed.
int sbft_launch_p256_verify_keyed_lanes(const uint8_t* d_digest, const uint8_t* d_r, const uint8_t* d_s,
                                        const uint32_t* d_key, const void* const* d_keytab, uint32_t nkeys,
                                        uint8_t* d_ok, uint32_t n, hipStream_t stream);
// The same over framed signatures (r || s at body end + sig_rel in d_blob; the blob readable
// SBFT_GV_SHA_BLOB_PAD bytes past its end): the bodies are hashed inside the launch.
int sbft_launch_p256_verify_keyed_framed(const uint8_t* d_blob, const uint64_t* d_off, const uint32_t* d_len,
                                         int32_t sig_rel, const uint32_t* d_key, const void* const* d_keytab,
                                         uint32_t nkeys, uint8_t* d_ok, uint32_t n, hipStream_t stream);
int sbft_launch_p256_verify_keyed(const uint8_t* d_digest, const uint8_t* d_blob, const uint64_t* d_off,
                                  const uint32_t* d_len, const uint8_t* d_r, const uint8_t* d_s,
                                  const uint32_t* d_key, const void* const* d_keytab, uint32_t nkeys,
                                  uint8_t* d_ok, uint32_t n, uint8_t mark, const uint32_t* d_winv,
                                  hipStream_t stream);
}
