"""CPU tests of the plugin-level mirror (include/sbft_verifier.h) that need no GPU: quorum
math (TestQuorum, internal/bft/util_test.go:135-163), Proposal.Digest (pkg/types/types.go:50-69)
against an independent restatement of Go encoding/asn1, and the parse-only paths."""
import hashlib

import pytest

from conftest import ROOT
from smartbft_amd import plugin


@pytest.mark.parametrize("n,f,q", [(4, 1, 3), (5, 1, 4), (6, 1, 4), (7, 2, 5), (8, 2, 6), (9, 2, 6),
                                   (10, 3, 7), (11, 3, 8), (12, 3, 8), (100, 33, 67)])
def test_quorum(n, f, q):
    assert plugin.compute_quorum(n) == (q, f)


def _der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _go_int64(v):
    # encoding/asn1 int64Length + big-endian two's complement
    n = 1
    i = v
    while i > 127:
        n += 1
        i >>= 8
    while i < -128:
        n += 1
        i >>= 8
    return (v & ((1 << (8 * n)) - 1)).to_bytes(n, "big")


def _go_digest(p):
    body = b""
    for f in (p.Payload, p.Header, p.Metadata):
        body += b"\x04" + _der_len(len(f)) + f
    iv = _go_int64(p.VerificationSequence)
    body += b"\x02" + _der_len(len(iv)) + iv
    return hashlib.sha256(b"\x30" + _der_len(len(body)) + body).hexdigest()


@pytest.mark.parametrize("size", [0, 1, 127, 128, 255, 256, 65535, 65536, 1 << 20])
@pytest.mark.parametrize("vseq", [0, 1, 127, 128, 255, 256, -1, -128, -129, (1 << 63) - 1, -(1 << 63)])
def test_proposal_digest_matches_go_asn1(size, vseq):
    p = plugin.Proposal(bytes(i % 251 for i in range(size)), b"hdr" * (size % 5), b"m" * (size % 300), vseq)
    assert p.Digest() == _go_digest(p)


def _go_commit_sigs_digest(sigs):
    # util.go:557-579: asn1.Marshal(IntDoubleBytes{A: [{int64(Signer), Value, Msg}...]})
    if not sigs:
        return None
    elems = b""
    for s in sigs:
        v = s.ID - (1 << 64) if s.ID >= 1 << 63 else s.ID  # int64(sig.Signer)
        iv = _go_int64(v)
        e = b"\x02" + _der_len(len(iv)) + iv
        e += b"\x04" + _der_len(len(s.Value)) + s.Value + b"\x04" + _der_len(len(s.Msg)) + s.Msg
        elems += b"\x30" + _der_len(len(e)) + e
    inner = b"\x30" + _der_len(len(elems)) + elems
    return hashlib.sha256(b"\x30" + _der_len(len(inner)) + inner).digest()


def test_commit_signatures_digest_matches_go_asn1():
    """CommitSignaturesDigest (internal/bft/util.go:557-579) against the Go-asn1 restatement:
    nil for no signatures, the reference tests' {Signer: 1}, {Signer: 2}, {Signer: 3}
    (view_test.go:227), signer ids across the int64 length steps and above 2^63 (the Go code
    casts to int64), and value/msg lengths across the DER short/long length forms."""
    S = plugin.Signature
    assert plugin.CommitSignaturesDigest([]) is None
    three = [S(1, b"", b""), S(2, b"", b""), S(3, b"", b"")]
    assert plugin.CommitSignaturesDigest(three) == _go_commit_sigs_digest(three)
    import random
    rng = random.Random(11)
    ids = [0, 1, 127, 128, 255, 256, 65535, (1 << 63) - 1, 1 << 63, (1 << 64) - 1]
    lens = [0, 1, 71, 72, 127, 128, 255, 256, 70000]
    for n in (1, 2, 5, 67, 300):
        sigs = [S(rng.choice(ids) if rng.random() < 0.5 else rng.randrange(1 << 64),
                  rng.randbytes(rng.choice(lens)), rng.randbytes(rng.choice(lens))) for _ in range(n)]
        assert plugin.CommitSignaturesDigest(sigs) == _go_commit_sigs_digest(sigs), n


def test_host_sha256():
    """Host SHA-256 (SHA-NI when the CPU has it) against hashlib: every length 0..300, then
    random lengths up to 200 KB."""
    import random
    rng = random.Random(3)
    m = rng.randbytes(200_000)
    for n in list(range(301)) + [rng.randrange(301, 200_000) for _ in range(60)]:
        assert plugin.sha256_host(m[:n]) == hashlib.sha256(m[:n]).digest(), n


def test_host_sha256_portable_path():
    """The portable compression (CPUs without the SHA extensions), forced by SBFT_NO_SHANI, in
    a fresh process: same digests, and Proposal.Digest unchanged."""
    import os
    import subprocess
    import sys
    code = ("import hashlib, random, sys; sys.path.insert(0, %r); from smartbft_amd import plugin; "
            "rng = random.Random(4); m = rng.randbytes(50_000); "
            "assert all(plugin.sha256_host(m[:n]) == hashlib.sha256(m[:n]).digest() "
            "for n in list(range(200)) + [777, 4096, 50_000]); "
            "print(plugin.Proposal(m, b'h', b'md', 7).Digest())") % ROOT
    env = dict(os.environ, SBFT_NO_SHANI="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    import random as _r
    m = _r.Random(4).randbytes(50_000)
    assert out.stdout.strip() == plugin.Proposal(m, b"h", b"md", 7).Digest()


def _fake_request(cid, rid, payload):
    """Format-only request (garbage key/signature): enough for the parse-only paths."""
    body = b"SBR1" + len(cid).to_bytes(2, "little") + cid.encode() + len(rid).to_bytes(2, "little") + \
        rid.encode() + len(payload).to_bytes(4, "little") + payload + b"\x04" + b"\x11" * 64
    return body + b"\x22" * 64


def test_requests_from_proposal_parse_only():
    v = plugin.Verifier(None)
    reqs = [_fake_request(f"client{i}", f"req{i}", bytes([i]) * i) for i in range(50)]
    p = plugin.Proposal(plugin.encode_payload(reqs))
    infos = v.RequestsFromProposal(p)
    assert [(r.ClientID, r.ID) for r in infos] == [(f"client{i}", f"req{i}") for i in range(50)]
    # malformed payloads parse to nothing (the reference stub returns nil on unmarshal errors)
    assert v.RequestsFromProposal(plugin.Proposal(p.Payload[:-1])) == []
    assert v.RequestsFromProposal(plugin.Proposal(b"\x05\x00\x00\x00")) == []
    # verification without an engine fails loudly, never silently accepts
    with pytest.raises(plugin.VerifyError):
        v.VerifyProposal(p)


@pytest.mark.parametrize("cid,rid", [("cl\0ient", "r1"), ("client", "r\0"), ("\0", "x")])
def test_nul_inside_an_id_is_malformed(cid, rid):
    """RequestInfos leave the C ABI as NUL-terminated "client_id\\0id\\0" records: an id holding a
    NUL would shift every later record (wrong ClientID/ID pairs for the pool). Such a request is
    malformed on every path: VerifyRequest, the batch form, and the proposal parse."""
    v = plugin.Verifier(None)
    bad = _fake_request(cid, rid, b"p")
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyRequest(bad)
    assert ei.value.code == plugin.EFORMAT
    assert v.VerifyRequests([bad]) == [plugin.EFORMAT]
    good = [_fake_request(f"c{i}", f"r{i}", b"") for i in range(3)]
    assert len(v.RequestsFromProposal(plugin.Proposal(plugin.encode_payload(good)))) == 3
    assert v.RequestsFromProposal(plugin.Proposal(plugin.encode_payload(good[:1] + [bad] + good[1:]))) == []
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(plugin.Proposal(plugin.encode_payload(good[:1] + [bad] + good[1:])))
    assert ei.value.code == plugin.EFORMAT


def test_auxiliary_data():
    aux = b"prepares-from"
    msg = b"SBC1" + (64).to_bytes(2, "little") + b"a" * 64 + len(aux).to_bytes(4, "little") + aux
    assert plugin.AuxiliaryData(msg) == aux
    assert plugin.AuxiliaryData(msg[:-1]) is None
    assert plugin.AuxiliaryData(b"") is None


def test_validate_last_decision_prechecks():
    """ValidateLastDecision's checks that precede any signature work (viewchanger.go:682-699),
    with the reference's error texts; a parse-only verifier never reaches the engine here."""
    v = plugin.Verifier(None)
    sig = plugin.Signature(1, b"\0" * 64, b"m")
    with pytest.raises(plugin.VerifyError, match="^the last decision is not set$"):
        v.validate_last_decision(None, None, 5, [sig], 3)
    p = plugin.Proposal(b"payload", b"h", b"md", 1)
    assert v.validate_last_decision(p, None, 5, [], 3) == 0  # genesis: nothing to validate
    with pytest.raises(plugin.VerifyError,
                       match="^last decision view 5 is greater or equal to requested next view 5$"):
        v.validate_last_decision(p, plugin.ViewMetadata(5, 9), 5, [sig] * 3, 3)
    with pytest.raises(plugin.VerifyError, match="^there are only 2 last decision signatures$"):
        v.validate_last_decision(p, plugin.ViewMetadata(4, 9), 5, [sig] * 2, 3)


def test_batch_entry_points_need_engine():
    """Batch forms on a parse-only verifier: malformed inputs are classified on the host, and
    anything needing a signature check fails loudly (no CPU fallback)."""
    v = plugin.Verifier(None)
    assert v.VerifyRequests([b"", b"SBR1junk"]) == [plugin.EFORMAT, plugin.EFORMAT]
    assert v.pool_prune([b"junk"]) == [0]
    assert v.VerifySignatures([plugin.Signature(9, b"\0" * 64, b"x")]) == [plugin.EKEY]
    # a syntactically valid request built by hand (no engine to sign one)
    req = (b"SBR1" + (1).to_bytes(2, "little") + b"a" + (1).to_bytes(2, "little") + b"b" +
           (0).to_bytes(4, "little") + b"\x04" + b"\1" * 64 + b"\2" * 64)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyRequests([req])
    assert ei.value.code == -2  # SBFT_GV_ENODEV


def _ref_request(r: bytes):
    """verifier.cpp parse_request restated: (client_id, id, key byte 0) or None."""
    def u(at, n):
        return int.from_bytes(r[at:at + n], "little") if at + n <= len(r) else None
    if r[:4] != b"SBR1":
        return None
    a = u(4, 2)
    if a is None or 6 + a > len(r):
        return None
    q = 6 + a
    b = u(q, 2)
    if b is None or q + 2 + b > len(r):
        return None
    cid, rid, q = r[6:6 + a], r[q + 2:q + 2 + b], q + 2 + b
    c = u(q, 4)
    if c is None or q + 4 + c + 129 != len(r) or b"\0" in cid or b"\0" in rid:
        return None
    return cid, rid, r[q + 4 + c]


def _ref_msg(m: bytes):
    """verifier.cpp parse_msg restated: the aux bytes or None."""
    if m[:4] != b"SBC1" or len(m) < 6:
        return None
    a = int.from_bytes(m[4:6], "little")
    if 6 + a + 4 > len(m):
        return None
    b = int.from_bytes(m[6 + a:10 + a], "little")
    return m[10 + a:] if 10 + a + b == len(m) else None


def test_random_request_and_message_mutations():
    """Differential fuzz of the single-request and consenter-message formats: mutated requests
    are EFORMAT in the batch form exactly when the restated format (or the SEC1 key prefix)
    rejects them, and AuxiliaryData returns exactly the restated aux bytes."""
    import numpy as np
    rng = np.random.default_rng(23)
    v = plugin.Verifier(None)
    base = _fake_request("client-7", "req-19", b"payload bytes")
    base = base[:-129] + b"\x04" + base[-128:]
    aux = b"prepares-from"
    msg = b"SBC1" + (32).to_bytes(2, "little") + b"d" * 32 + len(aux).to_bytes(4, "little") + aux
    reqs, msgs = [], []
    for n in range(400):
        for src, dst in ((base, reqs), (msg, msgs)):
            b = bytearray(src)
            for _ in range(int(rng.integers(1, 3))):
                at = int(rng.integers(0, len(b)))
                k = int(rng.integers(0, 3))
                if k == 0:
                    b[at] ^= 1 << int(rng.integers(0, 8))
                elif k == 1:
                    del b[at]
                else:
                    b.insert(at, int(rng.integers(0, 256)))
            dst.append(bytes(b))
    for r in reqs:
        want = _ref_request(r)
        try:  # a well-formed request needs the engine: the parse-only verifier raises ENODEV
            code = v.VerifyRequests([r])[0]
        except plugin.VerifyError as e:
            code = e.code
        assert (code == plugin.EFORMAT) == (want is None or want[2] != 0x04)
        assert code in (plugin.EFORMAT, -2)
    for m in msgs:
        assert plugin.AuxiliaryData(m) == _ref_msg(m)
    v.close()
