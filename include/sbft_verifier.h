/*
 * sbft_verifier.h — C ABI of the plugin-level mirror of SmartBFT's api.Verifier / api.Signer
 * (pkg/api/dependencies.go:46-71), implemented in C++ (smartbft_amd/csrc/verifier.cpp) on top
 * of the GPU engine (sbft_gpuverify.h). Go is absent from this image and from the GPU box,
 * so the host side is C++ with the same method set, argument meaning and error behaviour; the
 * cgo plugin a Go maintainer would add binds these symbols.
 *
 * Formats (the reference defines none):
 *  signed request  "SBR1" | u16 len | client_id | u16 len | req_id | u32 len | payload |
 *                  65-byte SEC1 uncompressed public key | 64-byte r||s
 *                  signature over SHA-256(every byte before r||s); integers little-endian;
 *                  client_id and req_id hold no NUL byte (else the request is malformed,
 *                  SBFT_V_EFORMAT: RequestInfos are returned as NUL-terminated records)
 *  proposal payload u32 count | count x (u32 len | signed request)
 *  consenter Msg   "SBC1" | u16 len | proposal digest (hex, Proposal.Digest()) | u32 len | aux
 *                  Signature.Value = r||s over SHA-256(Msg) by consenter ID's registered key
 *
 * Error convention (as the library uses the Go interface, view.go:388,637,840): a call returns
 * 0 on success, SBFT_V_EVERIFY (-10) when verification rejects, other negative codes on bad
 * arguments / infrastructure; err (if not NULL) receives a NUL-terminated message whose text
 * follows the reference's log lines where one exists. Thread-safe: every entry point may be
 * called concurrently (view.go:539-541 verifies q-1 votes from q-1 goroutines).
 */
#ifndef SBFT_VERIFIER_H
#define SBFT_VERIFIER_H

#include <stddef.h>
#include <stdint.h>

#include "sbft_gpuverify.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SBFT_V_EVERIFY (-10) /* a signature or binding check failed */
#define SBFT_V_EFORMAT (-11) /* malformed request / payload / message */
#define SBFT_V_EKEY (-12)    /* unknown consenter id */
#define SBFT_V_ESPACE (-13)  /* caller's output buffer too small */

typedef struct sbft_verifier sbft_verifier;

/* Wire structs mirroring pkg/types/types.go:18-48. Byte slices are borrowed for the call. */
typedef struct sbft_proposal {
    const uint8_t* payload;
    size_t payload_len;
    const uint8_t* header;
    size_t header_len;
    const uint8_t* metadata;
    size_t metadata_len;
    int64_t verification_sequence;
} sbft_proposal;

typedef struct sbft_signature {
    uint64_t id;
    const uint8_t* value;
    size_t value_len;
    const uint8_t* msg;
    size_t msg_len;
} sbft_signature;

/* A verifier bound to an engine context (not owned) and a verification sequence. */
sbft_verifier* sbft_verifier_new(sbft_gv_ctx* ctx, uint64_t verification_sequence);
void sbft_verifier_free(sbft_verifier* v);
/* Consenter key registry (SEC1 uncompressed, 65 bytes). With an engine context the key's
 * fixed-base comb tables are precomputed here (sbft_gv_register_key), so VerifyConsenterSig /
 * VerifySignature under it take the keyed launch (no doublings, one wavefront per signature).
 * Returns a negative SBFT_GV_E* only on an engine failure; an invalid point is stored and
 * every signature under it is rejected. */
int sbft_verifier_add_consenter(sbft_verifier* v, uint64_t id, const uint8_t pubkey65[65]);
/* Client-key registry (optional): a proposal whose requests are all signed by registered keys
 * (and that holds at least 1,025 of them) is verified by VerifyProposal against those keys'
 * precomputed comb tables (the keyed launch: no doublings, four lanes per signature); any
 * other proposal by the generic launch. Verdicts are the same either way.
 * pubkeys65: n x 65 bytes SEC1 uncompressed; keys that are not valid points are ignored.
 * Registration builds 512 KiB of tables per key per device (10,000 clients = 5 GB), up to the
 * engine's client-table budget (sbft_gv_register_client_keys): keys past it are left
 * unregistered, not an error. */
int sbft_verifier_add_clients(sbft_verifier* v, const uint8_t* pubkeys65, size_t n);
/* Client keys registered so far (sbft_verifier_add_clients stops at the engine's client-table
 * budget, sbft_gv_opts.client_table_bytes; the others stay on the generic path). */
size_t sbft_verifier_client_count(const sbft_verifier* v);
/* api.Verifier.VerificationSequence (dependencies.go:65-66). */
uint64_t sbft_verifier_verification_sequence(const sbft_verifier* v);
void sbft_verifier_set_verification_sequence(sbft_verifier* v, uint64_t seq);

/* api.Verifier.VerifyProposal (dependencies.go:56-57; called view.go:555): one fused GPU
 * launch (SHA-256 of every request body + P-256 verify). On success writes *count RequestInfo
 * pairs into infos as "client_id\0id\0" records (infos_cap bytes); bad_index (may be NULL)
 * receives the first failing request index on SBFT_V_EVERIFY. On failure *count is 0 and the
 * contents of infos are unspecified (the records are written while the GPU verifies). */
int sbft_verifier_verify_proposal(sbft_verifier* v, const sbft_proposal* p, char* infos,
                                  size_t infos_cap, size_t* count, int64_t* bad_index, char* err,
                                  size_t err_cap);
/* api.Verifier.RequestsFromProposal (dependencies.go:67-68): parse only, same output layout. */
int sbft_verifier_requests_from_proposal(sbft_verifier* v, const sbft_proposal* p, char* infos,
                                         size_t infos_cap, size_t* count);
/* api.Verifier.VerifyRequest (dependencies.go:58-59): "client_id\0id\0" into info. */
int sbft_verifier_verify_request(sbft_verifier* v, const uint8_t* req, size_t len, char* info,
                                 size_t info_cap, char* err, size_t err_cap);
/* api.Verifier.VerifyConsenterSig (dependencies.go:60-62): on success copies the auxiliary
 * data into aux (aux_cap bytes) and sets *aux_len. */
int sbft_verifier_verify_consenter_sig(sbft_verifier* v, const sbft_signature* s, const sbft_proposal* p,
                                       uint8_t* aux, size_t aux_cap, size_t* aux_len, char* err,
                                       size_t err_cap);
/* Coalescing of concurrent VerifyConsenterSig calls, for the unmodified library: view.go
 * verifies a decision's q-1 commit votes from q-1 goroutines at once (view.go:537-541 ->
 * voteVerifier.verifyVote :834), each with a single call. With coalescing on (max_batch > 1),
 * concurrent calls join one batch that launches when it holds max_batch calls or max_wait_us
 * after its first call, so a quorum costs one or two launches instead of q-1 serialised ones.
 * Every caller still gets exactly its own result (status, error text, aux). max_batch <= 1
 * turns it off (the default). The calls may check different proposals. */
int sbft_verifier_coalesce_consenter_sigs(sbft_verifier* v, size_t max_batch, uint32_t max_wait_us);
/* VerifyConsenterSig launches and calls served so far (observability). */
void sbft_verifier_consenter_stats(const sbft_verifier* v, uint64_t* launches, uint64_t* calls);
/* Batching hook (new): n consenter signatures over one proposal in one GPU
 * launch. status[i] = 0 ok, else the per-signature error code; auxes are not returned (use
 * sbft_verifier_auxiliary_data on the accepted messages). Returns 0 if the call ran. */
int sbft_verifier_verify_consenter_sigs(sbft_verifier* v, const sbft_signature* sigs, size_t n,
                                        const sbft_proposal* p, int32_t* status);
/* api.Verifier.VerifySignature (dependencies.go:63-64). */
int sbft_verifier_verify_signature(sbft_verifier* v, const sbft_signature* s, char* err, size_t err_cap);
/* Batch form of VerifySignature for the SignedViewData signatures a NewView carries
 * (viewchanger.go:982,1021,1075): n signatures in one launch. status[i] = 0
 * ok, SBFT_V_EKEY unknown signer, SBFT_V_EFORMAT bad value, SBFT_V_EVERIFY invalid. Returns 0 if
 * the call ran. */
int sbft_verifier_verify_signatures(sbft_verifier* v, const sbft_signature* sigs, size_t n, int32_t* status);
/* Batch form of VerifyRequest (N2): n standalone signed requests in one fused launch. status[i]
 * = 0 ok, SBFT_V_EFORMAT malformed, SBFT_V_EVERIFY invalid signature. */
int sbft_verifier_verify_requests(sbft_verifier* v, const uint8_t* const* reqs, const size_t* lens, size_t n,
                                  int32_t* status);
/* api.Verifier.AuxiliaryData (dependencies.go:69-70): returns the aux length, or -1 if msg
 * is malformed; copies min(len, aux_cap) bytes. */
int64_t sbft_verifier_auxiliary_data(const uint8_t* msg, size_t msg_len, uint8_t* aux, size_t aux_cap);

/* types.Proposal.Digest (pkg/types/types.go:50-69): hex(SHA-256(ASN.1 DER of the proposal)),
 * 64 characters + NUL into out65. */
void sbft_proposal_digest(const sbft_proposal* p, char out65[65]);
/* CommitSignaturesDigest (internal/bft/util.go:557-579; callers view.go:598 checks the leader's
 * PrevCommitSignatureDigest, view.go:984 fills it): SHA-256 of the ASN.1 DER of the signatures
 * as Go's encoding/asn1 marshals IntDoubleBytes. Returns 32 with the digest in out32, 0 for no
 * signatures (Go returns nil), SBFT_GV_EINVAL on NULL pointers. Host only (no GPU). */
int sbft_commit_signatures_digest(const sbft_signature* sigs, size_t n, uint8_t out32[32]);
/* Host SHA-256 (no GPU), used for Proposal.Digest and small messages. */
void sbft_sha256_host(const uint8_t* msg, size_t len, uint8_t out[32]);

/* api.Signer mirror (dependencies.go:46-52) for one node key. The nonce is RFC 6979
 * (HMAC-SHA-256), so signatures are deterministic. */
typedef struct sbft_signer sbft_signer;
sbft_signer* sbft_signer_new(sbft_gv_ctx* ctx, uint64_t id, const uint8_t priv32[32]);
void sbft_signer_free(sbft_signer* s);
int sbft_signer_public_key(const sbft_signer* s, uint8_t pubkey65[65]);
/* Signer.Sign: 64-byte r||s over SHA-256(data). */
int sbft_signer_sign(sbft_signer* s, const uint8_t* data, size_t len, uint8_t sig64[64]);
/* Pre-signature pool (off by default). With pool > 0 the signer draws random nonces k from
 * the kernel's CSPRNG (getrandom) and has the GPU compute, for `pool` nonces per launch,
 * r = x(kG) mod n, A = k^-1 and B = k^-1 r d (mod n); a signature then costs the host
 * s = A e + B (mod n) and no launch, and the pool refills (one launch) when it runs out.
 * Signatures become randomized instead of RFC 6979-deterministic; each nonce is used once and
 * then erased. pool = 0 returns to RFC 6979 nonces, one launch per signature. */
int sbft_signer_presign(sbft_signer* s, size_t pool);
/* Signer.SignProposal: builds Msg = "SBC1"|digest|aux into msg (msg_cap) and signs it. */
int sbft_signer_sign_proposal(sbft_signer* s, const sbft_proposal* p, const uint8_t* aux, size_t aux_len,
                              uint8_t* msg, size_t msg_cap, size_t* msg_len, uint8_t sig64[64]);
/* Build a signed request (format above) for the given client key: returns its length or a
 * negative code (test/bench helper; a client library's job). */
int64_t sbft_make_request(sbft_signer* client, const char* client_id, const char* req_id,
                          const uint8_t* payload, size_t payload_len, uint8_t* out, size_t out_cap);

/* ---- batching hook: mirrors of the library's call sites (internal/bft/view.go) ----
 * computeQuorum (util.go:176-180): f = (n-1)/3, q = ceil((n+f+1)/2). */
void sbft_compute_quorum(uint64_t n, int* q, int* f);
/* View.verifyPrevCommitSignatures (view.go:606-647) with one GPU launch for all signatures.
 * Skips (returns 0, *skipped = 1) when prev->verification_sequence != curr_vseq
 * (view.go:614-618). On failure returns SBFT_V_EVERIFY with err =
 * "failed verifying consenter signature of <id>: <reason>" for the first failing signer. */
int sbft_verify_prev_commit_signatures(sbft_verifier* v, const sbft_signature* sigs, size_t n,
                                       const sbft_proposal* prev, uint64_t curr_vseq, int* skipped,
                                       char* err, size_t err_cap);
/* View.processCommits + voteVerifier.verifyVote (view.go:519-551, 820-849) with the batch hook
 * of go/patches/internal_bft_commits.patch: votes are taken in arrival order; votes whose digest
 * differs from the proposal's are dropped ("Got wrong digest at processCommits"), duplicates by
 * signer are ignored (voteSet.registerVote, util.go:123-136); once the valid votes so far plus
 * the pending ones can complete the quorum, the pending ones are verified in one GPU launch,
 * and after an invalid vote the next arrivals form the next batch. Collection stops at `need`
 * (= quorum - 1) valid votes: later votes are not verified. valid_idx receives the indices of
 * the collected votes, log one line per rejected vote ("Couldn't verify <id>'s signature:
 * <reason>", view.go:840). If the votes run out first, the pending ones are verified anyway. */
int sbft_collect_commits(sbft_verifier* v, const sbft_signature* votes, const char* const* vote_digests,
                         size_t n, const sbft_proposal* p, size_t need, size_t* valid_idx,
                         size_t* n_valid, char* log, size_t log_cap);

/* ---- view change ----
 * The decoded protos.ViewMetadata of a last decision (messages.proto; the Go side unmarshals it
 * before the call, as ValidateLastDecision does at viewchanger.go:689-692). */
typedef struct sbft_view_metadata {
    uint64_t view_id;
    uint64_t latest_sequence;
} sbft_view_metadata;
/* ValidateLastDecision (viewchanger.go:681-727) with ONE launch for all signatures.
 * last_decision NULL = "the last decision is not set"; md NULL = genesis (Metadata == nil:
 * returns 0, *last_sequence = 0). Signatures are deduplicated by signer in order, verified as
 * VerifyConsenterSig against last_decision, and the first invalid one fails the call with the
 * reference's error text ("last decision signature is invalid, error: ..."); fewer than quorum
 * signatures (before or after dedupe) fail as the reference does. On success *last_sequence =
 * md->latest_sequence. */
int sbft_validate_last_decision(sbft_verifier* v, const sbft_proposal* last_decision,
                                const sbft_view_metadata* md, uint64_t next_view, const sbft_signature* sigs,
                                size_t n_sigs, int quorum, uint64_t* last_sequence, char* err, size_t err_cap);

/* ---- pool re-verification (N2) ----
 * Pool.Prune's predicate (requestpool.go:335-354) as called by MaybePruneRevokedRequests
 * (controller.go:733-746) when the verification sequence changes: VerifyRequest over every
 * pooled request in ONE launch. pruned_idx receives the indices (ascending) whose predicate
 * fails, i.e. the requests the pool removes; *n_pruned their count. */
int sbft_pool_prune(sbft_verifier* v, const uint8_t* const* reqs, const size_t* lens, size_t n, size_t* pruned_idx,
                    size_t* n_pruned);

/* ---- forwarded-request micro-batching (N3) ----
 * Controller.HandleRequest (controller.go:233-246) calls VerifyRequest from concurrent
 * transport goroutines, one request each. A batcher coalesces concurrent calls: a call joins
 * the open batch, which launches when it holds max_batch requests or max_wait_us after its
 * first request arrived. sbft_request_batcher_verify blocks and returns exactly what
 * sbft_verifier_verify_request would for that request. Thread-safe. */
typedef struct sbft_request_batcher sbft_request_batcher;
sbft_request_batcher* sbft_request_batcher_new(sbft_verifier* v, size_t max_batch, uint32_t max_wait_us);
void sbft_request_batcher_free(sbft_request_batcher* b);
int sbft_request_batcher_verify(sbft_request_batcher* b, const uint8_t* req, size_t len, char* info,
                                size_t info_cap, char* err, size_t err_cap);
/* launches and requests served so far (observability; the tests check coalescing with it) */
void sbft_request_batcher_stats(const sbft_request_batcher* b, uint64_t* launches, uint64_t* requests);

#ifdef __cplusplus
}
#endif
#endif
