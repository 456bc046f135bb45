package gpuverify

/*
#include "sbft_verifier.h"
*/
import "C"

import (
	"runtime"
	"unsafe"

	"github.com/hyperledger-labs/SmartBFT/pkg/types"
)

// RequestVerifier is an api.Verifier whose VerifyRequest coalesces concurrent callers into
// shared GPU launches (include/sbft_verifier.h sbft_request_batcher_*). Controller.HandleRequest
// calls VerifyRequest from transport goroutines, one request each (controller.go:233-246):
// a call joins the open batch, which launches when it holds maxBatch requests or maxWaitMicros
// after its first request arrived. Every caller gets exactly what Verifier.VerifyRequest
// would return for its request. The other methods are the embedded Verifier's.
type RequestVerifier struct {
	*Verifier
	b *C.sbft_request_batcher
}

// NewRequestVerifier wraps v with a request batcher.
func NewRequestVerifier(v *Verifier, maxBatch int, maxWaitMicros uint32) *RequestVerifier {
	rv := &RequestVerifier{Verifier: v, b: C.sbft_request_batcher_new(v.v, C.size_t(maxBatch), C.uint32_t(maxWaitMicros))}
	runtime.SetFinalizer(rv, (*RequestVerifier).Close)
	return rv
}

// Close releases the batcher (not the wrapped Verifier).
func (rv *RequestVerifier) Close() {
	if rv.b != nil {
		C.sbft_request_batcher_free(rv.b)
		rv.b = nil
	}
	runtime.SetFinalizer(rv, nil)
}

// VerifyRequest verifies one request through the batcher.
func (rv *RequestVerifier) VerifyRequest(val []byte) (types.RequestInfo, error) {
	var p pinner
	defer p.Unpin()
	info := make([]byte, len(val)+8)
	errbuf := make([]byte, 512)
	if rc := C.sbft_request_batcher_verify(rv.b, p.bytes(val), C.size_t(len(val)),
		(*C.char)(unsafe.Pointer(&info[0])), C.size_t(len(info)), cchar(errbuf), C.size_t(len(errbuf))); rc != 0 {
		if engineFailure(rc) {
			rv.failStop("VerifyRequest", rc)
		}
		return types.RequestInfo{}, &VerifyError{Code: int(rc), Index: -1, Msg: errText(errbuf)}
	}
	return splitInfos(info, 1)[0], nil
}
