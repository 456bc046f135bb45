"""GPU parity tests at the workloads of BASELINE.json configs 1, 3 and 5, through the C ABI,
against the oracle (oracle/p256_oracle.c, the C restatement of Go crypto/ecdsa.Verify) and
hashlib-independent SHA-256 (the oracle's).

Config 3: VerifyProposal (view.go:555) over a 10,000-request proposal, a distinct client key
per request, corrupted requests at the first, middle and last index: the whole proposal is
rejected (view.go:386-393) and the reported index is the first request the oracle rejects.
Both the generic launch and the registered-client (keyed) launch.

Config 5: hash + verify of payloads uniform in [1 KiB, 64 KiB] with corrupted signatures and
tampered payloads, fused (tuples passed in) and framed (tuples gathered on the device from the
signed-request layout), on the one-lane throughput kernel and the two-lane latency kernel,
and streamed from host memory (sbft_gv_sha256_verify_p256_stream).

Config 1: the naive_chain shape (4 nodes, 1k requests per proposal) driven through the plugin
mirror in the library's call sequence (Go is absent: the protocol itself is out of scope)."""
import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

KERNEL_OPTS = {"lane": dict(pair_max=-1, half_max=-1),
               "pair": dict(pair_max=1 << 30, half_max=-1),
               "half": dict(half_max=1 << 30, halfq_max=-1),
               "halfw": dict(halfq_max=1 << 30)}


# ---------------------------------------------------------------- config 3
@pytest.fixture(scope="module")
def requests_10k(gpu):
    from smartbft_amd.workload import make_signed_requests
    return make_signed_requests(gpu, 10_000, start=31337)


def _tuples(reqs):
    """The (digest, r, s, qx, qy) each request's signature check verifies (signed-request
    format of include/sbft_verifier.h: the body ends with the 65-byte SEC1 key, r || s follows)."""
    n = len(reqs)
    out = [np.zeros((n, 32), dtype=np.uint8) for _ in range(5)]
    for i, q in enumerate(reqs):
        body, sig = q[:-64], q[-64:]
        pub = body[-65:]
        for k, b in enumerate((hashlib.sha256(body).digest(), sig[:32], sig[32:], pub[1:33], pub[33:])):
            out[k][i] = np.frombuffer(b, dtype=np.uint8)
    return out


def _corrupt(reqs, where, kind):
    out = list(reqs)
    for i in where:
        q = bytearray(out[i])
        if kind == "sig":
            q[-40] ^= 0x10                       # a bit of s
        elif kind == "payload":
            q[-64 - 65 - 10] ^= 0x01             # inside the payload (signed body)
        elif kind == "key":
            q[-64 - 1] ^= 0x01                   # qy's last byte: off the curve
        out[i] = bytes(q)
    return out


CASES = [([0], "sig"), ([5000], "sig"), ([9999], "sig"), ([9999, 5000, 0], "payload"), ([4321], "key"),
         ([7777, 9998], "sig")]


def _check_proposal(v, reqs, where, kind):
    from smartbft_amd import plugin
    bad = _corrupt(reqs, where, kind)
    want = oracle.verify_batch(*_tuples(bad))
    first = int(np.nonzero(want == 0)[0][0])
    assert first == min(where) and int((want == 0).sum()) == len(set(where))
    p = plugin.Proposal(plugin.encode_payload(bad), b"header", b"metadata", 1)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.code == plugin.EVERIFY and ei.value.index == first
    assert f"request {first} (client{31337 + first}:tx{31337 + first}) has an invalid signature" in str(ei.value)


def test_config3_verify_proposal_10k_generic(gpu, requests_10k):
    from smartbft_amd import plugin
    reqs = requests_10k
    assert len({q[-129:-64] for q in reqs}) == 10_000  # a distinct client key per request
    assert oracle.verify_batch(*_tuples(reqs)).all()
    v = plugin.Verifier(gpu, 1)
    p = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
    infos = v.VerifyProposal(p)
    assert [(i.ClientID, i.ID) for i in infos] == [(f"client{31337 + i}", f"tx{31337 + i}") for i in range(10_000)]
    assert v.RequestsFromProposal(p) == infos
    for where, kind in CASES:
        _check_proposal(v, reqs, where, kind)
    v.close()


def test_config3_verify_proposal_10k_registered_clients(gpu, requests_10k):
    """The same proposals with every client key registered (keyed comb-table launch), then with
    half of them registered (the proposal is split over the keyed and the generic launch)."""
    from smartbft_amd import plugin
    reqs = requests_10k
    p = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
    half = plugin.Verifier(gpu, 1)
    half.add_clients([q[-129:-64] for q in reqs[::2]])
    want = [(f"client{31337 + i}", f"tx{31337 + i}") for i in range(10_000)]
    assert [(i.ClientID, i.ID) for i in half.VerifyProposal(p)] == want
    for where, kind in CASES:
        _check_proposal(half, reqs, where, kind)
    half.close()
    full = plugin.Verifier(gpu, 1)
    full.add_clients([q[-129:-64] for q in reqs])
    assert [(i.ClientID, i.ID) for i in full.VerifyProposal(p)] == want
    for where, kind in CASES:
        _check_proposal(full, reqs, where, kind)
    full.close()


def test_config3_client_table_budget(requests_10k):
    """The client-key registry under an HBM budget: with room for 3,000 clients'
    tables, registering all 10,000 registers 3,000 and leaves the rest on the generic path -- no
    error, now or at proposal time -- and a proposal mixing registered and unregistered clients
    gets the oracle's verdicts. Consenter keys are not budgeted. With 2 slots per device each key
    costs two tables, so the same budget holds half as many clients."""
    from smartbft_amd import GpuVerifier, plugin
    reqs = requests_10k
    tb = 512 << 10
    gv = GpuVerifier(device_mask=1, client_table_bytes=3000 * tb)
    try:
        v = plugin.Verifier(gv, 1)
        v.add_clients([q[-129:-64] for q in reqs])
        assert v.client_count() == 3000
        v.add_clients([q[-129:-64] for q in reqs[::-1]])  # budget spent: nothing more, no error
        assert v.client_count() == 3000
        ids = gv.register_keys(np.stack([np.frombuffer(q[-128:-96], np.uint8) for q in reqs[:5]]),
                               np.stack([np.frombuffer(q[-96:-64], np.uint8) for q in reqs[:5]]), client=True)
        assert (ids != 0).all()  # keys already registered keep their ids
        p = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
        want = [(f"client{31337 + i}", f"tx{31337 + i}") for i in range(10_000)]
        assert [(i.ClientID, i.ID) for i in v.VerifyProposal(p)] == want
        for where, kind in CASES:
            _check_proposal(v, reqs, where, kind)
        sg = plugin.Signer(gv, 7, (12345).to_bytes(32, "big"))
        v.add_consenter(7, sg.public_key())  # past the client budget: consenters still register
        assert v.VerifyConsenterSigs([sg.SignProposal(p, b"x")], p) == [0]
        sg.close()
        v.close()
    finally:
        gv.close()
    gv2 = GpuVerifier(device_mask=1, slots_per_device=2, client_table_bytes=3000 * tb)
    try:
        v2 = plugin.Verifier(gv2, 1)
        v2.add_clients([q[-129:-64] for q in reqs[:4000]])
        assert v2.client_count() == 1500
        p = plugin.Proposal(plugin.encode_payload(reqs[:4000]), b"header", b"metadata", 1)
        assert len(v2.VerifyProposal(p)) == 4000
        v2.close()
    finally:
        gv2.close()


# ---------------------------------------------------------------- config 5
def _config5_batch(n, seed, sign_with_gpu=None):
    """n messages, lengths uniform in [1 KiB, 64 KiB], each signed under its own key; ~1/5 with
    a corrupted signature, ~1/7 with the payload tampered after signing, a few with s = 0 / r >= n.
    Returns blob, off, len, (r, s, qx, qy), and the oracle's verdicts over SHA-256 of the
    messages as they are in the blob."""
    rng = np.random.default_rng(seed)
    ln = rng.integers(1024, 65537, size=n).astype(np.uint32)
    gaps = rng.integers(0, 4, size=n)  # unaligned message starts
    off = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += int(ln[i])
    blob = rng.integers(0, 256, size=pos, dtype=np.uint8)
    dig = oracle.sha256_batch(blob, off, ln)
    d = [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(n)]
    k = [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(n)]
    b32 = lambda xs: np.frombuffer(b"".join(x.to_bytes(32, "big") for x in xs), dtype=np.uint8).reshape(-1, 32)
    if sign_with_gpu is not None:
        qx, qy, r, s, st = sign_with_gpu.sign(b32(d), b32(k), dig)
        assert st.all()
    else:
        qx, qy, r, s = (np.zeros((n, 32), dtype=np.uint8) for _ in range(4))
        for i in range(n):
            x, y = oracle.pubkey(d[i])
            rr, ss = oracle.sign(d[i], k[i], bytes(dig[i]))
            qx[i], qy[i], r[i], s[i] = (np.frombuffer(b, dtype=np.uint8) for b in (x, y, rr, ss))
    for i in range(n):
        if i % 5 == 1:
            r[i, int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
        elif i % 7 == 2:
            blob[int(off[i]) + int(rng.integers(0, int(ln[i])))] ^= 0x40  # tampered after signing
        elif i % 97 == 3:
            s[i] = 0
        elif i % 89 == 4:
            r[i] = np.frombuffer(oracle.N.to_bytes(32, "big"), dtype=np.uint8)
    dig = oracle.sha256_batch(blob, off, ln)
    want = oracle.verify_batch(dig, r, s, qx, qy)
    return blob, off, ln, (r, s, qx, qy), dig, want


@pytest.mark.parametrize("mode", list(KERNEL_OPTS))
def test_config5_fused_hash_verify_1_to_64_kib(mode):
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available()
    gv = GpuVerifier(**KERNEL_OPTS[mode])
    blob, off, ln, cols, dig, want = _config5_batch(700, seed=55)
    assert 0.5 < want.mean() < 0.8
    ok, got_dig = gv.sha256_verify(blob, off, ln, *cols, want_digests=True)
    assert np.array_equal(got_dig, dig)
    assert np.array_equal(ok, want)
    gv.close()


@pytest.mark.parametrize("mode", list(KERNEL_OPTS))
def test_config5_framed_hash_verify_1_to_64_kib(mode):
    """The same payload sizes in the signed-request layout: each message is payload || qx || qy
    (the key closes the signed body) followed by r || s; the device gathers the tuple."""
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available()
    gv = GpuVerifier(**KERNEL_OPTS[mode])
    rng = np.random.default_rng(56)
    n = 400
    parts, off, lens, exp = [], [], [], []
    pos = 1
    for i in range(n):
        d = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        k = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        qx, qy = oracle.pubkey(d)
        body = rng.bytes(int(rng.integers(1024, 65537))) + qx + qy
        r, s = oracle.sign(d, k, hashlib.sha256(body).digest())
        sig = r + s
        if i % 6 == 1:
            sig = sig[:40] + bytes([sig[40] ^ 4]) + sig[41:]
        if i % 9 == 2:
            body = body[:100] + bytes([body[100] ^ 1]) + body[101:]
        cols = (hashlib.sha256(body).digest(), sig[:32], sig[32:], body[-64:-32], body[-32:])
        exp.append(oracle.verify_batch(*[np.frombuffer(x, dtype=np.uint8).reshape(1, 32) for x in cols])[0])
        off.append(pos)
        lens.append(len(body))
        parts.append(body + sig)
        pos += len(body) + 64
    exp = np.array(exp, dtype=np.uint8)
    blob = np.frombuffer(b"\0" + b"".join(parts), dtype=np.uint8)
    got = gv.sha256_verify_framed(blob, np.array(off), np.array(lens), 0, -64)
    assert np.array_equal(got, exp)
    assert 0 < exp.sum() < n
    gv.close()


def test_config5_large_batch_throughput_kernel(gpu):
    """40,000 messages of 1-64 KiB (~1.3 GB): above the latency kernel's 32,768-tuple limit, so
    the one-lane kernel with its launch-wide s^-1 batching runs; signed by the engine's signer
    (itself pinned to the oracle byte for byte in test_gpu_verify.py), verdicts vs the oracle."""
    blob, off, ln, cols, dig, want = _config5_batch(40_000, seed=57, sign_with_gpu=gpu)
    ok, got_dig = gpu.sha256_verify(blob, off, ln, *cols, want_digests=True)
    assert np.array_equal(got_dig, dig)
    assert np.array_equal(ok, want)


# ---------------------------------------------------------------- config 5, streamed
@pytest.fixture(scope="module")
def config5_batch():
    return _config5_batch(600, seed=58)


@pytest.mark.parametrize("window", [0, 1 << 20, 300_000, 16_384])
def test_config5_streamed_pageable(gpu, config5_batch, window):
    """sbft_gv_sha256_verify_p256_stream from pageable memory: windows gathered on the host
    into double-buffered pinned staging. Small windows force many windows, windows of one
    message, and messages longer than the window (16 KiB < 64 KiB)."""
    blob, off, ln, cols, dig, want = config5_batch
    ok, got = gpu.sha256_verify_stream(blob, off, ln, *cols, window_bytes=window, want_digests=True)
    assert np.array_equal(got, dig)
    assert np.array_equal(ok, want)
    assert np.array_equal(gpu.sha256_verify_stream(blob, off, ln, *cols, window_bytes=window), want)


def test_config5_streamed_pinned_blob(gpu, config5_batch):
    """A page-locked blob with dense windows is DMA'd in place; with the messages listed in a
    permuted order the windows are sparse and gathered on the host instead. Same verdicts."""
    from smartbft_amd import PinnedArray
    blob, off, ln, cols, dig, want = config5_batch
    pin = PinnedArray(blob.shape)
    try:
        pin.array[:] = blob
        ok, got = gpu.sha256_verify_stream(pin.array, off, ln, *cols, window_bytes=2 << 20, want_digests=True)
        assert np.array_equal(got, dig) and np.array_equal(ok, want)
        perm = np.random.default_rng(1).permutation(len(off))
        ok2 = gpu.sha256_verify_stream(pin.array, off[perm], ln[perm], *[c[perm] for c in cols],
                                       window_bytes=2 << 20)
        assert np.array_equal(ok2, want[perm])
    finally:
        pin.close()


def test_config5_streamed_edges(gpu, config5_batch):
    blob, off, ln, cols, dig, want = config5_batch
    assert np.array_equal(gpu.sha256_verify_stream(blob, off[:1], ln[:1], *[c[:1] for c in cols]), want[:1])
    z = np.zeros((0, 32), dtype=np.uint8)
    assert gpu.sha256_verify_stream(blob, off[:0], ln[:0], z, z, z, z).shape == (0,)
    with pytest.raises(Exception):  # a message past the blob's end is rejected, not read
        gpu.sha256_verify_stream(blob[:100], off[:2], ln[:2], *[c[:2] for c in cols])


# ---------------------------------------------------------------- config 1 (plumbing shape)
def test_config1_four_nodes_1k_requests(gpu):
    """BASELINE config 1's shape (examples/naive_chain: 4 nodes, f = 1, 1k signed requests per
    proposal) driven through the plugin mirror the way the library drives an api.Verifier
    (Go and the library are absent here; the call sequence follows view.go): every node
    verifies the leader's proposal (view.go:555), signs it (SignProposal, view.go:481),
    collects q-1 = 2 commit votes from the others (processCommits, view.go:519-551), and the next
    proposal carries the previous decision's q signatures, which every node re-verifies
    (verifyPrevCommitSignatures, view.go:606-647). A proposal with one forged request is
    rejected by every node at the same index (view.go:386-393)."""
    import hashlib
    from smartbft_amd import plugin
    q, f = plugin.compute_quorum(4)
    assert (q, f) == (3, 1)
    priv = lambda tag: (int.from_bytes(hashlib.sha256(b"c1-" + tag).digest(), "big") % oracle.N).to_bytes(32, "big")
    signers = [plugin.Signer(gpu, i, priv(b"node%d" % i)) for i in range(1, 5)]
    nodes = [plugin.Verifier(gpu, 1) for _ in range(4)]
    for v in nodes:
        for s in signers:
            v.add_consenter(s.id, s.public_key())
    clients = [plugin.Signer(gpu, 100 + c, priv(b"client%d" % c)) for c in range(16)]
    prev_sigs, prev_prop = None, None
    for seq in range(3):
        reqs = [clients[i % 16].make_request(f"c{i % 16}", f"s{seq}-r{i}", b"tx-%d-%d" % (seq, i) * 4)
                for i in range(1000)]
        prop = plugin.Proposal(plugin.encode_payload(reqs), b"hdr-%d" % seq, b"md-%d" % seq, 1)
        infos = [v.VerifyProposal(prop) for v in nodes]
        assert all(x == infos[0] for x in infos) and len(infos[0]) == 1000
        if prev_sigs is not None:
            for v in nodes:
                assert v.verify_prev_commit_signatures(prev_sigs, prev_prop, curr_vseq=1) is False
        votes = [s.SignProposal(prop, b"prepares-from-%d" % s.id) for s in signers]
        digest = prop.Digest()
        decided = []
        for k, v in enumerate(nodes):
            others = [(votes[j], digest) for j in range(4) if j != k]
            idx, log = v.collect_commits(others, prop, need=q - 1)
            assert len(idx) == q - 1 and log == ""
            decided.append([others[i][0] for i in idx] + [votes[k]])
        prev_sigs, prev_prop = decided[0], prop
    # a forged request: every node rejects the proposal at the same index
    bad = list(reqs)
    bad[517] = bad[517][:-1] + bytes([bad[517][-1] ^ 1])
    badp = plugin.Proposal(plugin.encode_payload(bad), b"hdr-x", b"md-x", 1)
    for v in nodes:
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyProposal(badp)
        assert ei.value.index == 517 and ei.value.code == plugin.EVERIFY
    for v in nodes:
        v.close()
