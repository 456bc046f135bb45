"""Python view of the plugin-level mirror of SmartBFT's api.Verifier / api.Signer
(include/sbft_verifier.h, implemented in C++ in csrc/verifier.cpp). Method names follow the Go
interface (pkg/api/dependencies.go:46-71) so the tests read like the reference's own; errors
surface as VerifyError carrying the library's message text."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

from .gpuverify import GpuVerifier, load_library

_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p

EVERIFY, EFORMAT, EKEY, ESPACE = -10, -11, -12, -13


class VerifyError(Exception):
    def __init__(self, code: int, msg: str, index: int | None = None):
        super().__init__(msg)
        self.code, self.index = code, index


class _Proposal(ctypes.Structure):
    _fields_ = [("payload", _u8p), ("payload_len", ctypes.c_size_t), ("header", _u8p),
                ("header_len", ctypes.c_size_t), ("metadata", _u8p), ("metadata_len", ctypes.c_size_t),
                ("verification_sequence", ctypes.c_int64)]


class _Signature(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint64), ("value", _u8p), ("value_len", ctypes.c_size_t),
                ("msg", _u8p), ("msg_len", ctypes.c_size_t)]


class _ViewMetadata(ctypes.Structure):
    _fields_ = [("view_id", ctypes.c_uint64), ("latest_sequence", ctypes.c_uint64)]


@dataclass
class ViewMetadata:
    """The decoded protos.ViewMetadata fields ValidateLastDecision reads (viewchanger.go:689-693)."""
    ViewId: int
    LatestSequence: int


@dataclass
class Proposal:
    """types.Proposal (pkg/types/types.go:18-23)."""
    Payload: bytes = b""
    Header: bytes = b""
    Metadata: bytes = b""
    VerificationSequence: int = 0

    def Digest(self) -> str:
        out = ctypes.create_string_buffer(65)
        keep = []
        _lib().sbft_proposal_digest(ctypes.byref(_prop(self, keep)), out)
        return out.value.decode()


@dataclass
class Signature:
    """types.Signature (pkg/types/types.go:25-29)."""
    ID: int
    Value: bytes
    Msg: bytes


@dataclass
class RequestInfo:
    ClientID: str
    ID: str


def _buf(b: bytes, keep: list):
    """Borrowed read-only pointer into b (no copy; the C side never writes through it)."""
    if not b:
        return None
    a = ctypes.c_char_p(bytes(b))
    keep.append(a)
    return ctypes.cast(a, _u8p)


def _prop(p: Proposal, keep: list) -> _Proposal:
    return _Proposal(_buf(p.Payload, keep), len(p.Payload), _buf(p.Header, keep), len(p.Header),
                     _buf(p.Metadata, keep), len(p.Metadata), p.VerificationSequence)


def _sig(s: Signature, keep: list) -> _Signature:
    return _Signature(s.ID, _buf(s.Value, keep), len(s.Value), _buf(s.Msg, keep), len(s.Msg))


def _blobs(items: list[bytes], keep: list):
    arr = (_u8p * max(1, len(items)))(*[_buf(b, keep) for b in items])
    lens = (ctypes.c_size_t * max(1, len(items)))(*[len(b) for b in items])
    return arr, lens


def _infos(buf, count: int) -> list[RequestInfo]:
    parts = buf.raw.split(b"\0", 2 * count)  # bounded: the rest of the buffer is unused
    # ids are arbitrary bytes (Go strings): bytes that are not UTF-8 survive as surrogate escapes
    return [RequestInfo(parts[2 * i].decode("utf-8", "surrogateescape"),
                        parts[2 * i + 1].decode("utf-8", "surrogateescape")) for i in range(count)]


_L = None


def _lib():
    global _L
    if _L is not None:
        return _L
    L = load_library()
    P, S = ctypes.POINTER(_Proposal), ctypes.POINTER(_Signature)
    sz = ctypes.POINTER(ctypes.c_size_t)
    L.sbft_verifier_new.restype = _vp
    L.sbft_verifier_new.argtypes = [_vp, ctypes.c_uint64]
    L.sbft_verifier_free.argtypes = [_vp]
    L.sbft_verifier_free.restype = None
    L.sbft_verifier_add_consenter.argtypes = [_vp, ctypes.c_uint64, _u8p]
    L.sbft_verifier_add_clients.argtypes = [_vp, _u8p, ctypes.c_size_t]
    L.sbft_verifier_client_count.argtypes = [_vp]
    L.sbft_verifier_client_count.restype = ctypes.c_size_t
    L.sbft_verifier_verification_sequence.restype = ctypes.c_uint64
    L.sbft_verifier_verification_sequence.argtypes = [_vp]
    L.sbft_verifier_set_verification_sequence.argtypes = [_vp, ctypes.c_uint64]
    L.sbft_verifier_set_verification_sequence.restype = None
    L.sbft_verifier_verify_proposal.argtypes = [_vp, P, ctypes.c_char_p, ctypes.c_size_t, sz,
                                                ctypes.POINTER(ctypes.c_int64), ctypes.c_char_p, ctypes.c_size_t]
    L.sbft_verifier_requests_from_proposal.argtypes = [_vp, P, ctypes.c_char_p, ctypes.c_size_t, sz]
    L.sbft_verifier_verify_request.argtypes = [_vp, _u8p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                               ctypes.c_char_p, ctypes.c_size_t]
    L.sbft_verifier_verify_consenter_sig.argtypes = [_vp, S, P, _u8p, ctypes.c_size_t, sz, ctypes.c_char_p,
                                                     ctypes.c_size_t]
    L.sbft_verifier_coalesce_consenter_sigs.argtypes = [_vp, ctypes.c_size_t, ctypes.c_uint32]
    L.sbft_verifier_consenter_stats.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.sbft_verifier_consenter_stats.restype = None
    L.sbft_verifier_verify_consenter_sigs.argtypes = [_vp, S, ctypes.c_size_t, P, ctypes.POINTER(ctypes.c_int32)]
    L.sbft_verifier_verify_signature.argtypes = [_vp, S, ctypes.c_char_p, ctypes.c_size_t]
    L.sbft_verifier_auxiliary_data.restype = ctypes.c_int64
    L.sbft_verifier_auxiliary_data.argtypes = [_u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t]
    L.sbft_proposal_digest.argtypes = [P, ctypes.c_char_p]
    L.sbft_proposal_digest.restype = None
    L.sbft_commit_signatures_digest.argtypes = [S, ctypes.c_size_t, _u8p]
    L.sbft_sha256_host.argtypes = [_u8p, ctypes.c_size_t, _u8p]
    L.sbft_sha256_host.restype = None
    L.sbft_signer_new.restype = _vp
    L.sbft_signer_new.argtypes = [_vp, ctypes.c_uint64, _u8p]
    L.sbft_signer_free.argtypes = [_vp]
    L.sbft_signer_free.restype = None
    L.sbft_signer_public_key.argtypes = [_vp, _u8p]
    L.sbft_signer_sign.argtypes = [_vp, _u8p, ctypes.c_size_t, _u8p]
    L.sbft_signer_presign.argtypes = [_vp, ctypes.c_size_t]
    L.sbft_signer_sign_proposal.argtypes = [_vp, P, _u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t, sz, _u8p]
    L.sbft_make_request.restype = ctypes.c_int64
    L.sbft_make_request.argtypes = [_vp, ctypes.c_char_p, ctypes.c_char_p, _u8p, ctypes.c_size_t, _u8p,
                                    ctypes.c_size_t]
    L.sbft_compute_quorum.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.sbft_compute_quorum.restype = None
    L.sbft_verify_prev_commit_signatures.argtypes = [_vp, S, ctypes.c_size_t, P, ctypes.c_uint64,
                                                     ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_size_t]
    L.sbft_collect_commits.argtypes = [_vp, S, ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, P,
                                       ctypes.c_size_t, sz, sz, ctypes.c_char_p, ctypes.c_size_t]
    i32p = ctypes.POINTER(ctypes.c_int32)
    u8pp = ctypes.POINTER(_u8p)
    L.sbft_verifier_verify_signatures.argtypes = [_vp, S, ctypes.c_size_t, i32p]
    L.sbft_verifier_verify_requests.argtypes = [_vp, u8pp, sz, ctypes.c_size_t, i32p]
    L.sbft_validate_last_decision.argtypes = [_vp, P, ctypes.POINTER(_ViewMetadata), ctypes.c_uint64, S,
                                              ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                              ctypes.c_char_p, ctypes.c_size_t]
    L.sbft_pool_prune.argtypes = [_vp, u8pp, sz, ctypes.c_size_t, sz, sz]
    L.sbft_request_batcher_new.restype = _vp
    L.sbft_request_batcher_new.argtypes = [_vp, ctypes.c_size_t, ctypes.c_uint32]
    L.sbft_request_batcher_free.argtypes = [_vp]
    L.sbft_request_batcher_free.restype = None
    L.sbft_request_batcher_verify.argtypes = [_vp, _u8p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                              ctypes.c_char_p, ctypes.c_size_t]
    L.sbft_request_batcher_stats.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.sbft_request_batcher_stats.restype = None
    _L = L
    return L


def sha256_host(b: bytes) -> bytes:
    out = (ctypes.c_uint8 * 32)()
    keep = []
    _lib().sbft_sha256_host(_buf(b, keep), len(b), out)
    return bytes(out)


def CommitSignaturesDigest(sigs: list[Signature]) -> bytes | None:
    """internal/bft/util.go:557-579: SHA-256 of the Go-asn1 DER of the signatures; None (Go's
    nil) for an empty list."""
    keep = []
    arr = (_Signature * max(1, len(sigs)))(*[_sig(s, keep) for s in sigs])
    out = (ctypes.c_uint8 * 32)()
    rc = _lib().sbft_commit_signatures_digest(arr, len(sigs), out)
    if rc < 0:
        raise VerifyError(rc, "commit signatures digest: invalid arguments")
    return bytes(out) if rc == 32 else None


def compute_quorum(n: int) -> tuple[int, int]:
    q, f = ctypes.c_int(), ctypes.c_int()
    _lib().sbft_compute_quorum(n, ctypes.byref(q), ctypes.byref(f))
    return q.value, f.value


def AuxiliaryData(msg: bytes) -> bytes | None:
    keep = []
    n = _lib().sbft_verifier_auxiliary_data(_buf(msg, keep), len(msg), None, 0)
    if n < 0:
        return None
    out = (ctypes.c_uint8 * max(1, n))()
    _lib().sbft_verifier_auxiliary_data(_buf(msg, keep), len(msg), out, n)
    return bytes(out[:n])


def encode_payload(requests: list[bytes]) -> bytes:
    out = bytearray(len(requests).to_bytes(4, "little"))
    for r in requests:
        out += len(r).to_bytes(4, "little") + r
    return bytes(out)


class Verifier:
    """api.Verifier over the GPU engine. gv=None gives a parse-only verifier."""

    def __init__(self, gv: GpuVerifier | None, verification_sequence: int = 0):
        self.L = _lib()
        self.gv = gv
        self.h = self.L.sbft_verifier_new(gv.ctx if gv else None, verification_sequence)

    def close(self):
        if self.h:
            self.L.sbft_verifier_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_consenter(self, node_id: int, pubkey65: bytes):
        keep = []
        assert self.L.sbft_verifier_add_consenter(self.h, node_id, _buf(pubkey65, keep)) == 0

    def add_clients(self, pubkeys65: list[bytes]):
        """Register client keys: their requests take the keyed (comb-table) launch."""
        keep = []
        blob = b"".join(pubkeys65)
        rc = self.L.sbft_verifier_add_clients(self.h, _buf(blob, keep), len(pubkeys65))
        if rc:
            raise VerifyError(rc, "client key registration failed")

    def client_count(self) -> int:
        """Client keys registered so far (registration stops at the engine's table budget)."""
        return self.L.sbft_verifier_client_count(self.h)

    def VerificationSequence(self) -> int:
        return self.L.sbft_verifier_verification_sequence(self.h)

    def SetVerificationSequence(self, seq: int):
        self.L.sbft_verifier_set_verification_sequence(self.h, seq)

    def VerifyProposal(self, p: Proposal) -> list[RequestInfo]:
        keep = []
        cap = 64 + len(p.Payload)  # each request's two ids + NULs fit inside its own record
        infos = ctypes.create_string_buffer(cap)
        count, bad = ctypes.c_size_t(), ctypes.c_int64()
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_verifier_verify_proposal(self.h, ctypes.byref(_prop(p, keep)), infos, cap,
                                                  ctypes.byref(count), ctypes.byref(bad), err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode(), bad.value if bad.value >= 0 else None)
        return _infos(infos, count.value)

    def RequestsFromProposal(self, p: Proposal) -> list[RequestInfo]:
        keep = []
        cap = 64 + len(p.Payload)
        infos = ctypes.create_string_buffer(cap)
        count = ctypes.c_size_t()
        rc = self.L.sbft_verifier_requests_from_proposal(self.h, ctypes.byref(_prop(p, keep)), infos, cap,
                                                         ctypes.byref(count))
        if rc:
            return []
        return _infos(infos, count.value)

    def VerifyRequest(self, req: bytes) -> RequestInfo:
        keep = []
        info = ctypes.create_string_buffer(len(req) + 8)
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_verifier_verify_request(self.h, _buf(req, keep), len(req), info, len(req) + 8, err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode())
        return _infos(info, 1)[0]

    def VerifyConsenterSig(self, s: Signature, p: Proposal) -> bytes:
        keep = []
        aux = (ctypes.c_uint8 * (len(s.Msg) + 1))()
        alen = ctypes.c_size_t()
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_verifier_verify_consenter_sig(self.h, ctypes.byref(_sig(s, keep)),
                                                       ctypes.byref(_prop(p, keep)), aux, len(s.Msg) + 1,
                                                       ctypes.byref(alen), err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode())
        return bytes(aux[:alen.value])

    def coalesce_consenter_sigs(self, max_batch: int, max_wait_us: int):
        """Concurrent VerifyConsenterSig calls share launches (max_batch <= 1: off)."""
        assert self.L.sbft_verifier_coalesce_consenter_sigs(self.h, max_batch, max_wait_us) == 0

    def consenter_stats(self) -> tuple[int, int]:
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self.L.sbft_verifier_consenter_stats(self.h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def VerifyConsenterSigs(self, sigs: list[Signature], p: Proposal) -> list[int]:
        keep = []
        arr = (_Signature * max(1, len(sigs)))(*[_sig(s, keep) for s in sigs])
        st = (ctypes.c_int32 * max(1, len(sigs)))()
        rc = self.L.sbft_verifier_verify_consenter_sigs(self.h, arr, len(sigs), ctypes.byref(_prop(p, keep)), st)
        if rc:
            raise VerifyError(rc, "engine failure")
        return list(st[:len(sigs)])

    def VerifySignature(self, s: Signature):
        keep = []
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_verifier_verify_signature(self.h, ctypes.byref(_sig(s, keep)), err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode())

    @staticmethod
    def AuxiliaryData(msg: bytes) -> bytes | None:
        return AuxiliaryData(msg)

    # ---- batching-hook mirrors of view.go ----
    def verify_prev_commit_signatures(self, sigs: list[Signature], prev: Proposal, curr_vseq: int):
        keep = []
        arr = (_Signature * max(1, len(sigs)))(*[_sig(s, keep) for s in sigs])
        skipped = ctypes.c_int()
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_verify_prev_commit_signatures(self.h, arr, len(sigs), ctypes.byref(_prop(prev, keep)),
                                                       curr_vseq, ctypes.byref(skipped), err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode())
        return bool(skipped.value)

    def VerifySignatures(self, sigs: list[Signature]) -> list[int]:
        """Batch VerifySignature (NewView's SignedViewData, viewchanger.go:982,1021,1075)."""
        keep = []
        arr = (_Signature * max(1, len(sigs)))(*[_sig(s, keep) for s in sigs])
        st = (ctypes.c_int32 * max(1, len(sigs)))()
        rc = self.L.sbft_verifier_verify_signatures(self.h, arr, len(sigs), st)
        if rc:
            raise VerifyError(rc, "engine failure")
        return list(st[:len(sigs)])

    def VerifyRequests(self, reqs: list[bytes]) -> list[int]:
        """Batch VerifyRequest: status per request (0 ok, EFORMAT, EVERIFY)."""
        keep = []
        arr, lens = _blobs(reqs, keep)
        st = (ctypes.c_int32 * max(1, len(reqs)))()
        rc = self.L.sbft_verifier_verify_requests(self.h, arr, lens, len(reqs), st)
        if rc:
            raise VerifyError(rc, "engine failure")
        return list(st[:len(reqs)])

    def validate_last_decision(self, last_decision: Proposal | None, md: ViewMetadata | None, next_view: int,
                               sigs: list[Signature], quorum: int) -> int:
        """ValidateLastDecision (viewchanger.go:681-727): returns the last sequence, raises
        VerifyError with the reference's error text."""
        keep = []
        arr = (_Signature * max(1, len(sigs)))(*[_sig(s, keep) for s in sigs])
        cmd = _ViewMetadata(md.ViewId, md.LatestSequence) if md is not None else None
        seq = ctypes.c_uint64()
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_validate_last_decision(
            self.h, ctypes.byref(_prop(last_decision, keep)) if last_decision is not None else None,
            ctypes.byref(cmd) if cmd is not None else None, next_view, arr, len(sigs), quorum,
            ctypes.byref(seq), err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode())
        return seq.value

    def pool_prune(self, reqs: list[bytes]) -> list[int]:
        """Pool.Prune(VerifyRequest) (requestpool.go:335-354, controller.go:742-745): indices
        of the requests the pool removes."""
        keep = []
        arr, lens = _blobs(reqs, keep)
        idx = (ctypes.c_size_t * max(1, len(reqs)))()
        n = ctypes.c_size_t()
        rc = self.L.sbft_pool_prune(self.h, arr, lens, len(reqs), idx, ctypes.byref(n))
        if rc:
            raise VerifyError(rc, "engine failure")
        return list(idx[:n.value])

    def collect_commits(self, votes: list[tuple[Signature, str]], p: Proposal, need: int):
        keep = []
        arr = (_Signature * max(1, len(votes)))(*[_sig(s, keep) for s, _ in votes])
        dig = (ctypes.c_char_p * max(1, len(votes)))(*[d.encode() for _, d in votes])
        idx = (ctypes.c_size_t * max(1, len(votes)))()
        nv = ctypes.c_size_t()
        log = ctypes.create_string_buffer(8192)
        rc = self.L.sbft_collect_commits(self.h, arr, dig, len(votes), ctypes.byref(_prop(p, keep)), need, idx,
                                         ctypes.byref(nv), log, 8192)
        if rc:
            raise VerifyError(rc, "engine failure")
        return list(idx[:nv.value]), log.value.decode()


class RequestBatcher:
    """Forwarded-request micro-batching (controller.go:233-246): concurrent VerifyRequest
    calls share one launch (include/sbft_verifier.h, sbft_request_batcher_*)."""

    def __init__(self, verifier: Verifier, max_batch: int = 256, max_wait_us: int = 200):
        self.L = verifier.L
        self.verifier = verifier  # keeps the verifier alive
        self.h = self.L.sbft_request_batcher_new(verifier.h, max_batch, max_wait_us)
        assert self.h

    def close(self):
        if self.h:
            self.L.sbft_request_batcher_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def VerifyRequest(self, req: bytes) -> RequestInfo:
        keep = []
        info = ctypes.create_string_buffer(len(req) + 8)
        err = ctypes.create_string_buffer(512)
        rc = self.L.sbft_request_batcher_verify(self.h, _buf(req, keep), len(req), info, len(req) + 8, err, 512)
        if rc:
            raise VerifyError(rc, err.value.decode())
        return _infos(info, 1)[0]

    def stats(self) -> tuple[int, int]:
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self.L.sbft_request_batcher_stats(self.h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value


class Signer:
    """api.Signer for one node/client key (RFC 6979 nonces, GPU signing)."""

    def __init__(self, gv: GpuVerifier, node_id: int, priv: bytes):
        self.L = _lib()
        keep = []
        self.h = self.L.sbft_signer_new(gv.ctx, node_id, _buf(priv, keep))
        if not self.h:
            raise ValueError("invalid private key")
        self.id = node_id

    def close(self):
        if self.h:
            self.L.sbft_signer_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def public_key(self) -> bytes:
        out = (ctypes.c_uint8 * 65)()
        self.L.sbft_signer_public_key(self.h, out)
        return bytes(out)

    def presign(self, pool: int) -> None:
        """Pre-signature pool (include/sbft_verifier.h sbft_signer_presign): randomized
        nonces, r / k^-1 / k^-1 r d computed `pool` at a time on the GPU, one host product per
        signature. 0 returns to RFC 6979 nonces."""
        rc = self.L.sbft_signer_presign(self.h, pool)
        if rc:
            raise VerifyError(rc, f"presign: code {rc}")

    def Sign(self, data: bytes) -> bytes:
        keep = []
        out = (ctypes.c_uint8 * 64)()
        assert self.L.sbft_signer_sign(self.h, _buf(data, keep), len(data), out) == 0
        return bytes(out)

    def SignProposal(self, p: Proposal, aux: bytes = b"") -> Signature:
        keep = []
        cap = 80 + len(aux)
        msg = (ctypes.c_uint8 * cap)()
        mlen = ctypes.c_size_t()
        sig = (ctypes.c_uint8 * 64)()
        rc = self.L.sbft_signer_sign_proposal(self.h, ctypes.byref(_prop(p, keep)), _buf(aux, keep), len(aux),
                                              msg, cap, ctypes.byref(mlen), sig)
        assert rc == 0, rc
        return Signature(self.id, bytes(sig), bytes(msg[:mlen.value]))

    def make_request(self, client_id: str, req_id: str, payload: bytes) -> bytes:
        keep = []
        cap = 200 + len(client_id) + len(req_id) + len(payload)
        out = (ctypes.c_uint8 * cap)()
        n = self.L.sbft_make_request(self.h, client_id.encode(), req_id.encode(), _buf(payload, keep),
                                     len(payload), out, cap)
        assert n > 0, n
        return bytes(out[:n])
