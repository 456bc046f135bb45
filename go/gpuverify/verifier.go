// Package gpuverify implements SmartBFT's api.Verifier (pkg/api/dependencies.go:54-71) and
// api.Signer (:46-52) on the MI355X signature-verification engine (libsbft_gpuverify.so,
// C ABI in include/sbft_verifier.h and include/sbft_gpuverify.h).
//
// It is meant to live in the SmartBFT module as pkg/gpuverify. Go is not installed in the
// image this engine is built and tested in, so this package is uncompiled here; every C entry
// point it binds is exercised through ctypes by tests/test_gpu_plugin.py and
// tests/test_gpu_configs.py on the GPU.
//
// Memory: the library keeps using the byte slices of the proposals and signatures it hands
// over (SURVEY.md 8(b) "Ownership"), so nothing is copied: each call pins the slices it passes
// with a runtime.Pinner (Go >= 1.21; the reference builds with 1.24.1, go.mod:3), which lets C
// read them through the Go-allocated sbft_proposal / sbft_signature structs for the duration
// of the call, and unpins them before returning. C never retains a pointer past a call.
package gpuverify

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/sbft_gpuverify/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/sbft_gpuverify/lib -lsbft_gpuverify -Wl,-rpath,${SRCDIR}/../../third_party/sbft_gpuverify/lib
#include <stdlib.h>
#include "sbft_verifier.h"
*/
import "C"

import (
	"bytes"
	"errors"
	"fmt"
	"log"
	"runtime"
	"unsafe"

	"github.com/hyperledger-labs/SmartBFT/pkg/api"
	"github.com/hyperledger-labs/SmartBFT/pkg/types"
	protos "github.com/hyperledger-labs/SmartBFT/smartbftprotos"
)

// Options of the engine context (sbft_gv_opts).
type Options struct {
	// DeviceMask selects HIP devices (bit d = device d); 0 = every visible device.
	DeviceMask uint32
	// MinSplit: batches smaller than this stay on one device (0 = 65,536).
	MinSplit uint32
	// CoalesceConsenterSigs > 1 turns on coalescing of concurrent VerifyConsenterSig calls
	// (view.go:537-541 verifies a decision's q-1 votes from q-1 goroutines): up to this many
	// calls share one GPU launch. CoalesceWaitMicros bounds how long the first call of a batch
	// waits for company.
	CoalesceConsenterSigs int
	CoalesceWaitMicros    uint32
	// OnEngineFailure is called when the engine itself fails (a negative SBFT_GV_E* code: a
	// device fault, a failed launch or copy, an allocation failure) instead of returning a
	// verdict. It must not return: nil means log.Fatalf, i.e. the node exits and the cluster sees
	// a crashed replica. Returning an error instead would read as a Byzantine leader: the library
	// treats any VerifyProposal error as a bad proposal (complain, sync, abort: view.go:386-393)
	// and a failed vote as a bad signature (view.go:839-841), so a GPU fault on the leader would
	// reject its own proposals and one on a follower would blame an honest leader.
	OnEngineFailure func(op string, err error)
}

// Verifier implements api.Verifier on the GPU engine. It is safe for concurrent use.
type Verifier struct {
	ctx    *C.sbft_gv_ctx
	v      *C.sbft_verifier
	onFail func(op string, err error)
}

// engineFailure reports whether rc says the engine itself failed (SBFT_GV_ENODEV, ENOMEM,
// ELAUNCH, EDEVICE, ESELFTEST: -2 .. -6), as opposed to a verdict (0, or SBFT_V_EVERIFY /
// EFORMAT / EKEY / ESPACE, -10 .. -13) or SBFT_GV_EINVAL (-1). EINVAL is an argument the caller
// built from its input, so it is returned as a VerifyError, never fail-stop: input a Byzantine
// client or replica controls must not be able to stop this replica. (The C entry points read an
// empty request, which cgo passes as NULL, 0, as SBFT_V_EFORMAT.)
func engineFailure(rc C.int) bool { return rc <= C.SBFT_GV_ENODEV && rc >= C.SBFT_GV_ESELFTEST }

// failStop hands an engine failure to the fail-stop hook; it does not return.
func (v *Verifier) failStop(op string, rc C.int) {
	err := &VerifyError{Code: int(rc), Index: -1, Msg: "gpu engine: " + C.GoString(C.sbft_gv_strerror(rc))}
	if v.onFail != nil {
		v.onFail(op, err)
	}
	log.Fatalf("gpuverify: %s: %v: stopping this replica (fail-stop, not a verification failure)", op, err)
}

var _ api.Verifier = (*Verifier)(nil)

// VerifyError is the error every failed verification returns; Code is the verdict
// (SBFT_V_EVERIFY, SBFT_V_EFORMAT, SBFT_V_EKEY) and Index the first failing request of a
// proposal (-1 otherwise). Engine failures (negative SBFT_GV_E* codes) are never returned as a
// VerifyError: they go to Options.OnEngineFailure (fail-stop).
type VerifyError struct {
	Code  int
	Index int64
	Msg   string
}

func (e *VerifyError) Error() string { return e.Msg }

// New creates the engine context and a verifier at the given verification sequence, with the
// consenters' 65-byte SEC1 uncompressed public keys (their comb tables are built here).
func New(opts Options, verificationSequence uint64, consenters map[uint64][]byte) (*Verifier, error) {
	o := C.sbft_gv_opts{device_mask: C.uint32_t(opts.DeviceMask), min_split: C.uint32_t(opts.MinSplit)}
	var ctx *C.sbft_gv_ctx
	if rc := C.sbft_gv_init(&o, &ctx); rc != 0 {
		return nil, fmt.Errorf("gpuverify: init: %s", C.GoString(C.sbft_gv_strerror(rc)))
	}
	v := &Verifier{ctx: ctx, v: C.sbft_verifier_new(ctx, C.uint64_t(verificationSequence)), onFail: opts.OnEngineFailure}
	if v.v == nil {
		C.sbft_gv_destroy(ctx)
		return nil, errors.New("gpuverify: verifier allocation failed")
	}
	runtime.SetFinalizer(v, (*Verifier).Close)
	for id, key := range consenters {
		if err := v.AddConsenter(id, key); err != nil {
			v.Close()
			return nil, err
		}
	}
	if opts.CoalesceConsenterSigs > 1 {
		C.sbft_verifier_coalesce_consenter_sigs(v.v, C.size_t(opts.CoalesceConsenterSigs), C.uint32_t(opts.CoalesceWaitMicros))
	}
	return v, nil
}

// Close releases the verifier and its engine context.
func (v *Verifier) Close() {
	if v.v != nil {
		C.sbft_verifier_free(v.v)
		v.v = nil
	}
	if v.ctx != nil {
		C.sbft_gv_destroy(v.ctx)
		v.ctx = nil
	}
	runtime.SetFinalizer(v, nil)
}

// AddConsenter registers (or replaces) consenter id's 65-byte SEC1 uncompressed public key.
func (v *Verifier) AddConsenter(id uint64, pubkey65 []byte) error {
	if len(pubkey65) != 65 || pubkey65[0] != 4 {
		return fmt.Errorf("gpuverify: consenter %d: key must be 65-byte SEC1 uncompressed", id)
	}
	var p pinner
	defer p.Unpin()
	if rc := C.sbft_verifier_add_consenter(v.v, C.uint64_t(id), p.bytes(pubkey65)); rc != 0 {
		return fmt.Errorf("gpuverify: consenter %d: %s", id, C.GoString(C.sbft_gv_strerror(rc)))
	}
	return nil
}

// AddClients registers client keys (65-byte SEC1 each, concatenated): a proposal whose
// requests are all signed by registered keys (at least 1,025 of them) is verified against
// their precomputed comb tables (512 KiB per key and device); others take the generic launch.
func (v *Verifier) AddClients(pubkeys65 []byte) error {
	if len(pubkeys65)%65 != 0 {
		return errors.New("gpuverify: client keys must be 65-byte SEC1 records")
	}
	var p pinner
	defer p.Unpin()
	if rc := C.sbft_verifier_add_clients(v.v, p.bytes(pubkeys65), C.size_t(len(pubkeys65)/65)); rc != 0 {
		return fmt.Errorf("gpuverify: client keys: %s", C.GoString(C.sbft_gv_strerror(rc)))
	}
	return nil
}

// SetVerificationSequence changes the sequence VerificationSequence reports (a
// reconfiguration); the library then prunes its pool (controller.go:733-746).
func (v *Verifier) SetVerificationSequence(seq uint64) {
	C.sbft_verifier_set_verification_sequence(v.v, C.uint64_t(seq))
}

// pinner pins the Go memory one C call reads through pointers stored in Go structs.
type pinner struct{ runtime.Pinner }

func (p *pinner) bytes(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	p.Pin(&b[0])
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func (p *pinner) proposal(pr types.Proposal) *C.sbft_proposal {
	cp := &C.sbft_proposal{
		payload: p.bytes(pr.Payload), payload_len: C.size_t(len(pr.Payload)),
		header: p.bytes(pr.Header), header_len: C.size_t(len(pr.Header)),
		metadata: p.bytes(pr.Metadata), metadata_len: C.size_t(len(pr.Metadata)),
		verification_sequence: C.int64_t(pr.VerificationSequence),
	}
	p.Pin(cp)
	return cp
}

func (p *pinner) signature(s types.Signature) C.sbft_signature {
	return C.sbft_signature{
		id:    C.uint64_t(s.ID),
		value: p.bytes(s.Value), value_len: C.size_t(len(s.Value)),
		msg: p.bytes(s.Msg), msg_len: C.size_t(len(s.Msg)),
	}
}

func (p *pinner) signatures(sigs []types.Signature) *C.sbft_signature {
	if len(sigs) == 0 {
		return nil
	}
	arr := make([]C.sbft_signature, len(sigs))
	for i, s := range sigs {
		arr[i] = p.signature(s)
	}
	p.Pin(&arr[0])
	return &arr[0]
}

func cchar(b []byte) *C.char { return (*C.char)(unsafe.Pointer(&b[0])) }

func errText(buf []byte) string {
	if i := bytes.IndexByte(buf, 0); i >= 0 {
		return string(buf[:i])
	}
	return string(buf)
}

// splitInfos decodes n "client_id\0id\0" records (ids hold no NUL: the engine rejects such
// requests as malformed) into RequestInfos.
func splitInfos(b []byte, n int) []types.RequestInfo {
	out := make([]types.RequestInfo, 0, n)
	for i := 0; i < n; i++ {
		j := bytes.IndexByte(b, 0)
		if j < 0 {
			break
		}
		cid := string(b[:j])
		b = b[j+1:]
		k := bytes.IndexByte(b, 0)
		if k < 0 {
			break
		}
		out = append(out, types.RequestInfo{ClientID: cid, ID: string(b[:k])})
		b = b[k+1:]
	}
	return out
}

// VerifyProposal: SHA-256 of every request body and P-256 verification of every request in
// one GPU launch (called at internal/bft/view.go:555). Any bad request rejects the proposal.
func (v *Verifier) VerifyProposal(pr types.Proposal) ([]types.RequestInfo, error) {
	var p pinner
	defer p.Unpin()
	infos := make([]byte, 64+len(pr.Payload)) // each request's ids + 2 NULs fit in its own record
	errbuf := make([]byte, 512)
	var count C.size_t
	var bad C.int64_t
	rc := C.sbft_verifier_verify_proposal(v.v, p.proposal(pr), cchar(infos), C.size_t(len(infos)), &count, &bad,
		cchar(errbuf), C.size_t(len(errbuf)))
	if engineFailure(rc) {
		v.failStop("VerifyProposal", rc)
	}
	if rc != 0 {
		return nil, &VerifyError{Code: int(rc), Index: int64(bad), Msg: errText(errbuf)}
	}
	return splitInfos(infos, int(count)), nil
}

// RequestsFromProposal parses the proposal's requests without verifying them
// (viewchanger.go:1177); nil for a malformed payload.
func (v *Verifier) RequestsFromProposal(pr types.Proposal) []types.RequestInfo {
	var p pinner
	defer p.Unpin()
	infos := make([]byte, 64+len(pr.Payload))
	var count C.size_t
	if C.sbft_verifier_requests_from_proposal(v.v, p.proposal(pr), cchar(infos), C.size_t(len(infos)), &count) != 0 {
		return nil
	}
	return splitInfos(infos, int(count))
}

// VerifyRequest verifies one signed request (controller.go:239, requestpool.go:335-354).
func (v *Verifier) VerifyRequest(val []byte) (types.RequestInfo, error) {
	var p pinner
	defer p.Unpin()
	info := make([]byte, len(val)+8)
	errbuf := make([]byte, 512)
	if rc := C.sbft_verifier_verify_request(v.v, p.bytes(val), C.size_t(len(val)), cchar(info), C.size_t(len(info)),
		cchar(errbuf), C.size_t(len(errbuf))); rc != 0 {
		if engineFailure(rc) {
			v.failStop("VerifyRequest", rc)
		}
		return types.RequestInfo{}, &VerifyError{Code: int(rc), Index: -1, Msg: errText(errbuf)}
	}
	return splitInfos(info, 1)[0], nil
}

// VerifyConsenterSig checks that the signature is consenter s.ID's over a message binding the
// proposal, and returns the message's auxiliary data (view.go:631 and :834 unmarshal it into
// protos.PreparesFrom). With Options.CoalesceConsenterSigs, concurrent calls share launches.
func (v *Verifier) VerifyConsenterSig(s types.Signature, pr types.Proposal) ([]byte, error) {
	var p pinner
	defer p.Unpin()
	cs := p.signature(s)
	p.Pin(&cs)
	aux := make([]byte, len(s.Msg)+1)
	errbuf := make([]byte, 512)
	var n C.size_t
	if rc := C.sbft_verifier_verify_consenter_sig(v.v, &cs, p.proposal(pr), (*C.uint8_t)(unsafe.Pointer(&aux[0])),
		C.size_t(len(aux)), &n, cchar(errbuf), C.size_t(len(errbuf))); rc != 0 {
		if engineFailure(rc) {
			v.failStop("VerifyConsenterSig", rc)
		}
		return nil, &VerifyError{Code: int(rc), Index: -1, Msg: errText(errbuf)}
	}
	return aux[:n], nil
}

// VerifyConsenterSigs is the batch extension the internal/bft hook detects
// (go/patches/internal_bft_prev_commits.patch): n signatures over one proposal in one launch.
// errs[i] is nil for a valid signature, whose auxiliary data is auxes[i].
func (v *Verifier) VerifyConsenterSigs(sigs []types.Signature, pr types.Proposal) (auxes [][]byte, errs []error) {
	auxes, errs = make([][]byte, len(sigs)), make([]error, len(sigs))
	if len(sigs) == 0 {
		return auxes, errs
	}
	var p pinner
	defer p.Unpin()
	status := make([]C.int32_t, len(sigs))
	if rc := C.sbft_verifier_verify_consenter_sigs(v.v, p.signatures(sigs), C.size_t(len(sigs)), p.proposal(pr),
		&status[0]); rc != 0 {
		// per-signature verdicts come back in status; a non-zero rc is the engine's, or EINVAL
		if engineFailure(rc) {
			v.failStop("VerifyConsenterSigs", rc)
		}
		for i := range errs {
			errs[i] = &VerifyError{Code: int(rc), Index: -1, Msg: "gpuverify: " + C.GoString(C.sbft_gv_strerror(rc))}
		}
		return auxes, errs
	}
	for i, st := range status {
		switch st {
		case 0:
			auxes[i] = v.AuxiliaryData(sigs[i].Msg)
		case C.SBFT_V_EKEY:
			errs[i] = &VerifyError{Code: int(st), Index: -1, Msg: fmt.Sprintf("unknown consenter %d", sigs[i].ID)}
		case C.SBFT_V_EFORMAT:
			errs[i] = &VerifyError{Code: int(st), Index: -1, Msg: "malformed signature message"}
		default:
			errs[i] = &VerifyError{Code: int(st), Index: -1, Msg: "invalid signature"}
		}
	}
	return auxes, errs
}

// VerifySignature verifies a signature over s.Msg by consenter s.ID (viewchanger.go:598, 660,
// 982, 1021, 1075).
func (v *Verifier) VerifySignature(s types.Signature) error {
	var p pinner
	defer p.Unpin()
	cs := p.signature(s)
	p.Pin(&cs)
	errbuf := make([]byte, 512)
	if rc := C.sbft_verifier_verify_signature(v.v, &cs, cchar(errbuf), C.size_t(len(errbuf))); rc != 0 {
		if engineFailure(rc) {
			v.failStop("VerifySignature", rc)
		}
		return &VerifyError{Code: int(rc), Index: -1, Msg: errText(errbuf)}
	}
	return nil
}

// VerificationSequence returns the current verification sequence.
func (v *Verifier) VerificationSequence() uint64 {
	return uint64(C.sbft_verifier_verification_sequence(v.v))
}

// AuxiliaryData extracts the auxiliary data from a consenter signature's message without
// verifying it (view.go:1032, 1074); nil for a malformed message.
func (v *Verifier) AuxiliaryData(msg []byte) []byte {
	var p pinner
	defer p.Unpin()
	m := p.bytes(msg)
	n := C.sbft_verifier_auxiliary_data(m, C.size_t(len(msg)), nil, 0)
	if n < 0 {
		return nil
	}
	out := make([]byte, int(n)+1)
	C.sbft_verifier_auxiliary_data(m, C.size_t(len(msg)), (*C.uint8_t)(unsafe.Pointer(&out[0])), C.size_t(n))
	return out[:n]
}

// PruneSet returns the indices of the pooled requests that fail VerifyRequest, verified in
// one launch: the batch form of Pool.Prune's predicate (requestpool.go:335-354).
func (v *Verifier) PruneSet(reqs [][]byte) ([]int, error) {
	if len(reqs) == 0 {
		return nil, nil
	}
	var p pinner
	defer p.Unpin()
	ptrs := make([]*C.uint8_t, len(reqs))
	lens := make([]C.size_t, len(reqs))
	for i, r := range reqs {
		ptrs[i], lens[i] = p.bytes(r), C.size_t(len(r))
	}
	p.Pin(&ptrs[0])
	idx := make([]C.size_t, len(reqs))
	var n C.size_t
	if rc := C.sbft_pool_prune(v.v, &ptrs[0], &lens[0], C.size_t(len(reqs)), &idx[0], &n); rc != 0 {
		if engineFailure(rc) {
			v.failStop("PruneSet", rc) // pruning would otherwise drop valid requests as revoked
		}
		return nil, &VerifyError{Code: int(rc), Index: -1, Msg: "gpuverify: " + C.GoString(C.sbft_gv_strerror(rc))}
	}
	out := make([]int, int(n))
	for i := range out {
		out[i] = int(idx[i])
	}
	return out, nil
}

// CommitSignaturesDigest is a drop-in for internal/bft/util.go:557-579 (called at view.go:598 to
// check the leader's PrevCommitSignatureDigest and at view.go:984 to fill it): SHA-256 of the
// Go-asn1 DER of the signatures, computed by the library on the host without copying values or
// messages. nil for no signatures, as the original.
func CommitSignaturesDigest(sigs []*protos.Signature) []byte {
	if len(sigs) == 0 {
		return nil
	}
	var p pinner
	defer p.Unpin()
	arr := make([]C.sbft_signature, len(sigs))
	for i, s := range sigs {
		arr[i] = C.sbft_signature{
			id:    C.uint64_t(s.Signer),
			value: p.bytes(s.Value), value_len: C.size_t(len(s.Value)),
			msg: p.bytes(s.Msg), msg_len: C.size_t(len(s.Msg)),
		}
	}
	p.Pin(&arr[0])
	out := make([]byte, 32)
	p.Pin(&out[0])
	if C.sbft_commit_signatures_digest(&arr[0], C.size_t(len(sigs)), (*C.uint8_t)(unsafe.Pointer(&out[0]))) != 32 {
		panic("gpuverify: CommitSignaturesDigest failed")
	}
	return out
}
