package gpuverify

import (
	"errors"
	"testing"
)

// newOrSkip opens the engine on the first visible device, or skips the test where there is none.
func newOrSkip(t *testing.T) *Verifier {
	t.Helper()
	v, err := New(Options{DeviceMask: 1}, 0, nil)
	if err != nil {
		t.Skipf("no usable GPU: %v", err)
	}
	t.Cleanup(v.Close)
	return v
}

// An empty request is input a client or a forwarding replica controls (Controller.HandleRequest,
// controller.go:233-246). It must come back as a verification error, never reach failStop
// (which would exit the replica).
func TestVerifyRequestEmptyIsMalformed(t *testing.T) {
	v := newOrSkip(t)
	v.onFail = func(op string, err error) { t.Fatalf("fail-stop on bad input: %s: %v", op, err) }
	for _, req := range [][]byte{nil, {}} {
		_, err := v.VerifyRequest(req)
		var ve *VerifyError
		if !errors.As(err, &ve) {
			t.Fatalf("VerifyRequest(%v): want *VerifyError, got %v", req, err)
		}
		if ve.Code != -11 { // SBFT_V_EFORMAT
			t.Fatalf("VerifyRequest(%v): code %d, want SBFT_V_EFORMAT", req, ve.Code)
		}
	}
}

func TestBatchedVerifyRequestEmptyIsMalformed(t *testing.T) {
	v := newOrSkip(t)
	v.onFail = func(op string, err error) { t.Fatalf("fail-stop on bad input: %s: %v", op, err) }
	rv := NewRequestVerifier(v, 8, 50)
	defer rv.Close()
	for _, req := range [][]byte{nil, {}} {
		_, err := rv.VerifyRequest(req)
		var ve *VerifyError
		if !errors.As(err, &ve) || ve.Code != -11 {
			t.Fatalf("batched VerifyRequest(%v): want SBFT_V_EFORMAT, got %v", req, err)
		}
	}
}
