// engine_internal.h — C++ entry points of the engine (gpuverify.cpp) used by the plugin
// mirror (verifier.cpp) inside the same library. Not part of the public C ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <vector>

struct sbft_gv_ctx;

// Framed hash + verify of one payload (sbft_gv_sha256_verify_p256_framed) with the host-side
// parse overlapped with the payload's H2D copy: the copy does not need the offsets, so
// The engine's helper thread copies the payload to the device while `prepare` runs on the
// caller's thread. prepare fills off / len (one entry per framed message) and returns 0, or a
// nonzero code that is returned unchanged (nothing is launched). `during` (optional) runs on
// the caller's thread once the hash and verify launches are queued, before the call waits for
// them. ok receives one verdict per message. Batches of min_split or more messages on a multi-device context fall back to the
// split path after the parse.
// kid (optional): registered key ids (sbft_gv_register_keys), read after prepare returns. If
// prepare left one nonzero id per message there (and the batch is large enough for the
// four-lane keyed kernel), the batch is verified against those keys' comb tables instead.
int sbft_gv_framed_overlapped(sbft_gv_ctx* ctx, const uint8_t* blob, size_t blob_len, int32_t sig_rel,
                              int32_t pub_rel,
                              const std::function<int(std::vector<uint64_t>&, std::vector<uint32_t>&)>& prepare,
                              std::vector<uint8_t>& ok, const std::function<void()>& during = nullptr,
                              const std::vector<uint32_t>* kid = nullptr);
