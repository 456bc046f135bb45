package gpuverify

/*
#include <stdlib.h>
#include "sbft_verifier.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	"github.com/hyperledger-labs/SmartBFT/pkg/api"
	"github.com/hyperledger-labs/SmartBFT/pkg/types"
)

// Signer implements api.Signer (pkg/api/dependencies.go:46-52) for one node key on the GPU
// engine: ECDSA P-256 over SHA-256 with RFC 6979 nonces (deterministic), signing on the GPU
// (one wavefront per signature over G's comb table). SignProposal builds the consenter
// message Msg = "SBC1" | u16 64 | Proposal.Digest() (hex) | u32 len | aux that the Verifier
// checks (include/sbft_verifier.h), so the aux round-trips into protos.PreparesFrom
// (view.go:639-643, :1032-1036).
type Signer struct {
	id uint64
	s  *C.sbft_signer
	v  *Verifier // owns the engine context the signer uses
}

var _ api.Signer = (*Signer)(nil)

// NewSigner binds a 32-byte big-endian private key in [1, n-1] to node id, on v's engine.
func NewSigner(v *Verifier, id uint64, priv32 []byte) (*Signer, error) {
	if len(priv32) != 32 {
		return nil, errors.New("gpuverify: private key must be 32 bytes")
	}
	var p pinner
	defer p.Unpin()
	s := C.sbft_signer_new(v.ctx, C.uint64_t(id), p.bytes(priv32))
	if s == nil {
		return nil, errors.New("gpuverify: invalid private key")
	}
	sg := &Signer{id: id, s: s, v: v}
	runtime.SetFinalizer(sg, (*Signer).Close)
	return sg, nil
}

// Close releases the signer.
func (sg *Signer) Close() {
	if sg.s != nil {
		C.sbft_signer_free(sg.s)
		sg.s = nil
	}
	runtime.SetFinalizer(sg, nil)
}

// Presign turns on the pre-signature pool (include/sbft_verifier.h sbft_signer_presign):
// randomized nonces whose r, k^-1 and k^-1 r d the GPU computes `pool` at a time, so Sign and
// SignProposal cost one host product and no launch. 0 returns to RFC 6979 nonces.
func (sg *Signer) Presign(pool int) error {
	if rc := C.sbft_signer_presign(sg.s, C.size_t(pool)); rc != 0 {
		return fmt.Errorf("gpuverify: presign: %s", C.GoString(C.sbft_gv_strerror(rc)))
	}
	return nil
}

// PublicKey returns the 65-byte SEC1 uncompressed public key.
func (sg *Signer) PublicKey() []byte {
	out := make([]byte, 65)
	C.sbft_signer_public_key(sg.s, (*C.uint8_t)(unsafe.Pointer(&out[0])))
	return out
}

// Sign returns r || s (64 bytes) over SHA-256(data). api.Signer has no error return: a
// failure here means the engine is gone, which the node cannot recover from.
func (sg *Signer) Sign(data []byte) []byte {
	var p pinner
	defer p.Unpin()
	sig := make([]byte, 64)
	if rc := C.sbft_signer_sign(sg.s, p.bytes(data), C.size_t(len(data)), (*C.uint8_t)(unsafe.Pointer(&sig[0]))); rc != 0 {
		panic(fmt.Sprintf("gpuverify: sign: %s", C.GoString(C.sbft_gv_strerror(rc))))
	}
	return sig
}

// SignProposal signs the consenter message binding the proposal and the auxiliary input
// (view.go:481; viewchanger.go:1259).
func (sg *Signer) SignProposal(pr types.Proposal, aux []byte) *types.Signature {
	var p pinner
	defer p.Unpin()
	msg := make([]byte, 4+2+64+4+len(aux))
	sig := make([]byte, 64)
	var n C.size_t
	if rc := C.sbft_signer_sign_proposal(sg.s, p.proposal(pr), p.bytes(aux), C.size_t(len(aux)),
		(*C.uint8_t)(unsafe.Pointer(&msg[0])), C.size_t(len(msg)), &n, (*C.uint8_t)(unsafe.Pointer(&sig[0]))); rc != 0 {
		panic(fmt.Sprintf("gpuverify: sign proposal: %s", C.GoString(C.sbft_gv_strerror(rc))))
	}
	return &types.Signature{ID: sg.id, Value: sig, Msg: msg[:n]}
}

// MakeRequest builds a signed request in the engine's format (include/sbft_verifier.h) under
// this key: a client-library helper for tests and load generators.
func (sg *Signer) MakeRequest(clientID, reqID string, payload []byte) ([]byte, error) {
	var p pinner
	defer p.Unpin()
	cid, rid := C.CString(clientID), C.CString(reqID)
	defer C.free(unsafe.Pointer(cid))
	defer C.free(unsafe.Pointer(rid))
	out := make([]byte, 200+len(clientID)+len(reqID)+len(payload))
	n := C.sbft_make_request(sg.s, cid, rid, p.bytes(payload), C.size_t(len(payload)),
		(*C.uint8_t)(unsafe.Pointer(&out[0])), C.size_t(len(out)))
	if n < 0 {
		return nil, fmt.Errorf("gpuverify: make request: code %d", int(n))
	}
	return out[:n], nil
}
