"""GPU tests of the api.Verifier / api.Signer mirror: every verification goes through the
engine (one fused launch per proposal / per consenter batch). Expectations follow the
reference's own tests where they pin behaviour: any bad request rejects the whole proposal
(view.go:386-393, TestBadPrePrepare), the prev-commit error text (view.go:637), the
commit-vote log text (view.go:840, TestBadCommit), dedupe per signer (util.go:123-136)."""
import hashlib
import hmac

import numpy as np
import pytest

import oracle
from smartbft_amd import plugin

pytestmark = pytest.mark.gpu


def _priv(tag):
    return (int.from_bytes(hashlib.sha256(b"node" + str(tag).encode()).digest(), "big") % oracle.N).to_bytes(32, "big")


@pytest.fixture(scope="module")
def net(gpu):
    nodes = [plugin.Signer(gpu, i, _priv(i)) for i in range(1, 5)]
    v = plugin.Verifier(gpu, verification_sequence=3)
    for s in nodes:
        v.add_consenter(s.id, s.public_key())
    clients = [plugin.Signer(gpu, 1000 + i, _priv(("client", i))) for i in range(8)]
    return v, nodes, clients


def _proposal(clients, n, tamper=None):
    reqs = []
    for i in range(n):
        r = clients[i % len(clients)].make_request(f"client{i % len(clients)}", f"tx{i}", b"payload-%d" % i)
        if tamper == i:
            r = r[:30] + bytes([r[30] ^ 1]) + r[31:]
        reqs.append(r)
    return plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 3), reqs


def test_verify_proposal_accepts_and_lists_requests(net):
    v, nodes, clients = net
    p, reqs = _proposal(clients, 300)
    infos = v.VerifyProposal(p)
    assert [(i.ClientID, i.ID) for i in infos] == [(f"client{i % 8}", f"tx{i}") for i in range(300)]
    assert v.RequestsFromProposal(p) == infos


def test_verify_proposal_rejects_any_bad_request(net):
    v, nodes, clients = net
    p, _ = _proposal(clients, 100, tamper=37)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.index == 37 and "has an invalid signature" in str(ei.value)
    assert ei.value.code == plugin.EVERIFY


def test_verify_request(net):
    v, nodes, clients = net
    r = clients[0].make_request("alice", "42", b"hello")
    info = v.VerifyRequest(r)
    assert (info.ClientID, info.ID) == ("alice", "42")
    with pytest.raises(plugin.VerifyError):
        v.VerifyRequest(r[:-1] + bytes([r[-1] ^ 0x80]))
    with pytest.raises(plugin.VerifyError):
        v.VerifyRequest(r[:10])


def test_empty_request_is_malformed_not_an_engine_error(net):
    """An empty request (Go's nil / []byte{}, passed as NULL, 0) is a malformed request from the
    network: SBFT_V_EFORMAT, which the Go binding returns as a VerifyError. Before round 5 it was
    SBFT_GV_EINVAL, which the binding's fail-stop would have turned into a replica exit."""
    v, nodes, clients = net
    for req in (b"", None):
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyRequest(req or b"")
        assert ei.value.code == plugin.EFORMAT
    b = plugin.RequestBatcher(v, max_batch=4, max_wait_us=100)
    with pytest.raises(plugin.VerifyError) as ei:
        b.VerifyRequest(b"")
    assert ei.value.code == plugin.EFORMAT
    assert b.stats() == (0, 0)  # refused before joining a batch
    r = clients[0].make_request("alice", "43", b"hi")
    assert b.VerifyRequest(r).ID == "43"
    b.close()


def test_requests_signatures_verify_under_oracle(net):
    """The engine's RFC 6979 signatures are valid ECDSA under the independent oracle."""
    v, nodes, clients = net
    r = clients[3].make_request("c3", "x", b"abc")
    body, sig = r[:-64], r[-64:]
    pub = clients[3].public_key()
    assert oracle.verify(hashlib.sha256(body).digest(), sig[:32], sig[32:], pub[1:33], pub[33:])


def _rfc6979_k(x: bytes, h1: bytes) -> int:
    """Independent restatement of RFC 6979 3.2 with Python's hmac."""
    q = oracle.N
    h = (int.from_bytes(h1, "big") % q).to_bytes(32, "big")
    V, K = b"\x01" * 32, b"\x00" * 32
    K = hmac.new(K, V + b"\x00" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    K = hmac.new(K, V + b"\x01" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    while True:
        V = hmac.new(K, V, hashlib.sha256).digest()
        k = int.from_bytes(V, "big")
        if 1 <= k < q:
            return k
        K = hmac.new(K, V + b"\x00", hashlib.sha256).digest()
        V = hmac.new(K, V, hashlib.sha256).digest()


def test_signer_rfc6979_known_answer(gpu):
    # RFC 6979 A.2.5, P-256 with SHA-256, message "sample"
    x = bytes.fromhex("C9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721")
    s = plugin.Signer(gpu, 9, x)
    pub = s.public_key()
    assert pub[1:].hex().upper() == (
        "60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6"
        "7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299")
    sig = s.Sign(b"sample")
    k = _rfc6979_k(x, hashlib.sha256(b"sample").digest())
    assert k == 0xA6E3C57DD01ABE90086538398355DD4C3B17AA873382B0F24D6129493D8AAD60
    assert sig.hex().upper() == (
        "EFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716"
        "F7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8")


def test_presign_pool_signatures(gpu):
    """Pooled signer (sbft_signer_presign): randomized signatures, valid under the oracle,
    through pool refills (pool 5, 23 signatures), and SignProposal verifies on the keyed path;
    presign(0) returns to the RFC 6979 known answer."""
    x = bytes.fromhex("C9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721")
    s = plugin.Signer(gpu, 9, x)
    pub = s.public_key()
    qx, qy = pub[1:33], pub[33:]
    s.presign(5)
    sigs = []
    for i in range(23):
        m = b"pooled-%d" % i
        sig = s.Sign(m)
        sigs.append(sig)
        e = hashlib.sha256(m).digest()
        assert oracle.verify_batch(*[np.frombuffer(b, dtype=np.uint8).reshape(1, 32)
                                     for b in (e, sig[:32], sig[32:], qx, qy)])[0], i
    assert len({sg[:32] for sg in sigs}) == len(sigs)  # fresh nonce per signature
    assert s.Sign(b"sample") != s.Sign(b"sample")    # randomized
    v = plugin.Verifier(gpu, 1)
    v.add_consenter(9, pub)
    p = plugin.Proposal(b"pooled-block" * 50, b"h", b"m", 1)
    sp = s.SignProposal(p, b"aux")
    assert v.VerifyConsenterSig(sp, p) == b"aux"
    s.presign(0)
    assert s.Sign(b"sample").hex().upper() == (
        "EFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716"
        "F7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8")
    v.close()


def test_consenter_sig_roundtrip_and_binding(net):
    v, nodes, clients = net
    p, _ = _proposal(clients, 10)
    other, _ = _proposal(clients, 11)
    sig = nodes[1].SignProposal(p, b"aux-bytes")
    assert v.VerifyConsenterSig(sig, p) == b"aux-bytes"
    assert plugin.AuxiliaryData(sig.Msg) == b"aux-bytes"
    with pytest.raises(plugin.VerifyError, match="does not bind"):
        v.VerifyConsenterSig(sig, other)
    bad = plugin.Signature(sig.ID, sig.Value[:-1] + bytes([sig.Value[-1] ^ 1]), sig.Msg)
    with pytest.raises(plugin.VerifyError, match="invalid signature"):
        v.VerifyConsenterSig(bad, p)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyConsenterSig(plugin.Signature(77, sig.Value, sig.Msg), p)
    assert ei.value.code == plugin.EKEY
    v.VerifySignature(plugin.Signature(nodes[2].id, nodes[2].Sign(b"view-data"), b"view-data"))
    with pytest.raises(plugin.VerifyError):
        v.VerifySignature(plugin.Signature(nodes[2].id, nodes[2].Sign(b"view-data"), b"view-datA"))


def test_consenter_batch_statuses(net):
    v, nodes, clients = net
    p, _ = _proposal(clients, 5)
    sigs = [n.SignProposal(p, b"a%d" % n.id) for n in nodes]
    sigs[2] = plugin.Signature(sigs[2].ID, sigs[1].Value, sigs[2].Msg)  # wrong value
    st = v.VerifyConsenterSigs(sigs, p)
    assert st == [0, 0, plugin.EVERIFY, 0]


def test_prev_commit_signatures_mirror(net):
    v, nodes, clients = net
    prev, _ = _proposal(clients, 7)
    sigs = [n.SignProposal(prev, b"") for n in nodes[:3]]
    assert v.verify_prev_commit_signatures(sigs, prev, curr_vseq=3) is False
    assert v.verify_prev_commit_signatures(sigs, prev, curr_vseq=4) is True  # skipped: seq advanced
    sigs[1] = plugin.Signature(sigs[1].ID, sigs[0].Value, sigs[1].Msg)
    with pytest.raises(plugin.VerifyError,
                       match=f"failed verifying consenter signature of {sigs[1].ID}: invalid signature"):
        v.verify_prev_commit_signatures(sigs, prev, curr_vseq=3)


def test_collect_commits_quorum_n100(gpu):
    """Commit collection at n = 100 (q = 67, 66 votes needed besides our own), one launch."""
    q, f = plugin.compute_quorum(100)
    assert (q, f) == (67, 33)
    nodes = [plugin.Signer(gpu, i, _priv(("n100", i))) for i in range(1, 101)]
    v = plugin.Verifier(gpu, 1)
    for s in nodes:
        v.add_consenter(s.id, s.public_key())
    p = plugin.Proposal(b"block", b"h", b"m", 1)
    dig = p.Digest()
    votes = [(n.SignProposal(p, b""), dig) for n in nodes[1:80]]
    votes[3] = (plugin.Signature(votes[3][0].ID, votes[4][0].Value, votes[3][0].Msg), dig)  # bad sig
    votes[7] = (votes[7][0], "ff" * 32)                                                      # wrong digest
    votes.insert(10, votes[9])                                                              # duplicate
    idx, log = v.collect_commits(votes, p, need=q - 1)
    assert len(idx) == q - 1
    assert 3 not in idx and 7 not in idx and 10 not in idx
    assert f"Couldn't verify {votes[3][0].ID}'s signature: invalid signature" in log
    assert "Got wrong digest at processCommits" in log


# ---- N1: view change --------------------------------------------------------------------
def test_validate_last_decision(net):
    """ValidateLastDecision (viewchanger.go:681-727), one launch; the cases of
    TestValidateLastDecision (viewchanger_test.go:1415-1522): dedupe by signer, any invalid
    signature fails, fewer valid than quorum fails."""
    v, nodes, clients = net
    prev, _ = _proposal(clients, 4)
    md = plugin.ViewMetadata(ViewId=1, LatestSequence=7)
    sigs = [n.SignProposal(prev, b"") for n in nodes[:3]]
    assert v.validate_last_decision(prev, md, 2, sigs, 3) == 7
    # a duplicate of a valid signer does not count twice
    with pytest.raises(plugin.VerifyError, match="^there are only 2 valid last decision signatures$"):
        v.validate_last_decision(prev, md, 2, [sigs[0], sigs[1], sigs[0]], 3)
    bad = list(sigs)
    bad[1] = plugin.Signature(sigs[1].ID, sigs[0].Value, sigs[1].Msg)
    with pytest.raises(plugin.VerifyError,
                       match="^last decision signature is invalid, error: invalid signature$"):
        v.validate_last_decision(prev, md, 2, bad, 3)
    other, _ = _proposal(clients, 5)
    with pytest.raises(plugin.VerifyError, match="does not bind"):
        v.validate_last_decision(other, md, 2, sigs, 3)


def test_verify_signatures_batch(net):
    """NewView's SignedViewData signatures (viewchanger.go:982,1021,1075) in one launch; each
    status equals what the single VerifySignature call returns."""
    v, nodes, clients = net
    sigs = [plugin.Signature(n.id, n.Sign(b"view-data-%d" % n.id), b"view-data-%d" % n.id) for n in nodes]
    sigs.append(plugin.Signature(nodes[0].id, sigs[1].Value, sigs[0].Msg))   # wrong value
    sigs.append(plugin.Signature(99, sigs[0].Value, sigs[0].Msg))            # unknown signer
    sigs.append(plugin.Signature(nodes[0].id, sigs[0].Value[:63], sigs[0].Msg))  # short value
    st = v.VerifySignatures(sigs)
    assert st == [0, 0, 0, 0, plugin.EVERIFY, plugin.EKEY, plugin.EFORMAT]
    for s, want in zip(sigs, st):
        if want == 0:
            v.VerifySignature(s)
        else:
            with pytest.raises(plugin.VerifyError) as ei:
                v.VerifySignature(s)
            assert ei.value.code == want


# ---- N2: pool re-verification -------------------------------------------------------------
def test_pool_prune_and_verify_requests(net):
    """MaybePruneRevokedRequests -> Pool.Prune(VerifyRequest) (controller.go:733-746,
    requestpool.go:335-354): one launch over the pool; pruned = the requests whose
    VerifyRequest fails, in pool order."""
    v, nodes, clients = net
    pool = [clients[i % 8].make_request(f"c{i % 8}", f"r{i}", b"x" * (i % 97)) for i in range(400)]
    bad = {3, 77, 200, 399}
    for i in bad:
        r = pool[i]
        pool[i] = r[:-1] + bytes([r[-1] ^ 4])
    pool[150] = pool[150][:20]  # malformed
    st = v.VerifyRequests(pool)
    assert [i for i, s in enumerate(st) if s] == sorted(bad | {150})
    assert st[150] == plugin.EFORMAT and st[3] == plugin.EVERIFY
    assert v.pool_prune(pool) == sorted(bad | {150})
    for i in (0, 3, 150):  # same verdict as the single call
        if st[i]:
            with pytest.raises(plugin.VerifyError):
                v.VerifyRequest(pool[i])
        else:
            v.VerifyRequest(pool[i])


# ---- N3: forwarded-request micro-batching ------------------------------------------------
def test_request_batcher_coalesces_concurrent_callers(net):
    """HandleRequest's VerifyRequest from concurrent transport goroutines (controller.go:233-246):
    64 threads, one request each, coalesce into few launches; every caller gets its own verdict."""
    import threading
    v, nodes, clients = net
    reqs = [clients[i % 8].make_request(f"c{i % 8}", f"fw{i}", b"p%d" % i) for i in range(64)]
    reqs[9] = reqs[9][:-1] + bytes([reqs[9][-1] ^ 1])
    b = plugin.RequestBatcher(v, max_batch=64, max_wait_us=20000)
    out = [None] * len(reqs)
    start = threading.Barrier(len(reqs))

    def call(i):
        start.wait()
        try:
            out[i] = b.VerifyRequest(reqs[i])
        except plugin.VerifyError as e:
            out[i] = e

    th = [threading.Thread(target=call, args=(i,)) for i in range(len(reqs))]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert isinstance(out[9], plugin.VerifyError) and out[9].code == plugin.EVERIFY
    assert "has an invalid signature" in str(out[9])
    for i, o in enumerate(out):
        if i != 9:
            assert (o.ClientID, o.ID) == (f"c{i % 8}", f"fw{i}")
    launches, served = b.stats()
    assert served == 64 and launches < 16, (launches, served)
    # a lone caller is served after its deadline, with one launch
    assert b.VerifyRequest(reqs[0]).ID == "fw0"
    assert b.stats() == (launches + 1, 65)
    b.close()


# ---- client-key registry: VerifyProposal on the keyed launch ------------------------------
def test_verify_proposal_registered_clients(gpu, net):
    """With the clients' keys registered (sbft_verifier_add_clients), VerifyProposal verifies
    a proposal whose keys are all registered on the comb-table launch (>= 1,025 requests): same
    RequestInfos, same rejection (index and text) as the generic path; a proposal mixing
    registered and unregistered clients, or a small one, takes the generic launch."""
    _, nodes, clients = net
    v = plugin.Verifier(gpu, 3)
    p, reqs = _proposal(clients, 120)
    generic = v.VerifyProposal(p)
    v.add_clients([c.public_key() for c in clients[:5]] + [b"\x04" + b"\x01" * 64])  # last: off-curve
    assert v.VerifyProposal(p) == generic
    bad, _ = _proposal(clients, 120, tamper=41)   # client 41 % 8 = 1: registered
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(bad)
    assert ei.value.index == 41 and "has an invalid signature" in str(ei.value)
    bad, _ = _proposal(clients, 120, tamper=46)   # client 6: not registered
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(bad)
    assert ei.value.index == 46
    v.add_clients([c.public_key() for c in clients])  # all registered (re-registering is a no-op)
    assert v.VerifyProposal(p) == generic
    # >= 1,025 requests, every key registered: the keyed four-lane launch over the payload
    # (bodies hashed on a fifth wavefront, r || s read in place), against the generic verifier
    g = plugin.Verifier(gpu, 3)
    big, _ = _proposal(clients, 1100)
    assert v.VerifyProposal(big) == g.VerifyProposal(big)
    for t in (0, 1037, 1099):
        bad, _ = _proposal(clients, 1100, tamper=t)
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyProposal(bad)
        assert ei.value.index == t and "has an invalid signature" in str(ei.value)
    g.close()
    v.close()


@pytest.mark.parametrize("registered", [False, True])
def test_verify_proposal_format_checked_during_verify(gpu, net, registered):
    """VerifyProposal launches after the chain of length prefixes alone and runs the full format
    check while the GPU verifies (verifier.cpp walk_payload / check): a request malformed inside
    (magic, a NUL in an id, a compressed key) under an intact length chain gets the format
    verdict, ahead of any signature verdict, on the generic and the registered-key launch; a good
    proposal after them verifies."""
    _, nodes, clients = net
    v = plugin.Verifier(gpu, 3)
    good, reqs = _proposal(clients, 1100)
    if registered:
        v.add_clients([q[-129:-64] for q in reqs[:len(clients)]])

    def enc(rs):
        return plugin.Proposal(plugin.encode_payload(rs), b"header", b"metadata", 3)

    def expect(rs, text, index=None):
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyProposal(enc(rs))
        assert ei.value.code == plugin.EFORMAT and text in str(ei.value), str(ei.value)
        if index is not None:
            assert ei.value.index == index
        if index is None:
            assert v.RequestsFromProposal(enc(rs)) == []

    _, bad_sig = _proposal(clients, 1100, tamper=100)
    for at in (0, 700, 1099):
        rs = list(bad_sig)
        rs[at] = b"X" + rs[at][1:]                     # broken magic, same length
        expect(rs, "malformed proposal payload")
        rs = list(bad_sig)
        rs[at] = rs[at][:6] + b"\0" + rs[at][7:]      # NUL inside the client id
        expect(rs, "malformed proposal payload")
        rs = list(bad_sig)
        rs[at] = rs[at][:-129] + b"\x02" + rs[at][-128:]  # compressed-key prefix
        expect(rs, "public key is not SEC1 uncompressed", index=at)
    # a request shorter than the smallest well-formed one fails the walk (no launch)
    rs = list(reqs)
    rs[5] = rs[5][:100]
    expect(rs, "malformed proposal payload")
    # the walk's own length checks (with clients registered the key lookups trail the walk on a
    # second thread and must stop at its last whole request): payload cut inside the last
    # request, one trailing byte, a count one higher than the requests present
    pl = plugin.encode_payload(reqs)
    for raw in (pl[:-1], pl + b"\0", (len(reqs) + 1).to_bytes(4, "little") + pl[4:]):
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyProposal(plugin.Proposal(raw, b"header", b"metadata", 3))
        assert ei.value.code == plugin.EFORMAT and "malformed proposal payload" in str(ei.value)
    assert len(v.VerifyProposal(good)) == 1100
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(enc(bad_sig))
    assert ei.value.code == plugin.EVERIFY and ei.value.index == 100
    v.close()


def test_verify_proposal_format_errors_and_concurrent_callers(net):
    """The overlapped path (parse on the engine's helper thread): format errors found there come
    back with their own code and text, and concurrent callers (helper busy -> inline parse)
    each get their own proposal's verdicts."""
    import threading
    v, nodes, clients = net
    good, _ = _proposal(clients, 60)
    bad, _ = _proposal(clients, 40, tamper=11)
    trunc = plugin.Proposal(good.Payload[:-1], good.Header, good.Metadata, good.VerificationSequence)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(trunc)
    assert ei.value.code == plugin.EFORMAT and "malformed" in str(ei.value)
    results, errors = {}, []

    def worker(k):
        try:
            for it in range(6):
                if (k + it) % 2:
                    assert len(v.VerifyProposal(good)) == 60
                else:
                    with pytest.raises(plugin.VerifyError) as e:
                        v.VerifyProposal(bad)
                    assert e.value.index == 11 and e.value.code == plugin.EVERIFY
            results[k] = True
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    assert len(results) == 4


# ---- config 4 as the stock library drives it: concurrent single VerifyConsenterSig calls ----
def test_consenter_sig_coalescer_concurrent_callers(gpu):
    """view.go:537-541 spawns one goroutine per commit vote, each calling VerifyConsenterSig
    (:834). With coalescing on, 66 concurrent single calls share few launches; every caller
    still gets its own verdict, aux, and error text (view.go:840 logs "Couldn't verify %d's
    signature: %v" with it)."""
    import threading
    q, f = plugin.compute_quorum(100)
    nodes = [plugin.Signer(gpu, i, _priv(("co", i))) for i in range(1, q + 1)]
    v = plugin.Verifier(gpu, 1)
    for s in nodes:
        v.add_consenter(s.id, s.public_key())
    blocks = [plugin.Proposal(b"blk-%d" % k * 50, b"h", b"m", 1) for k in range(2)]
    votes = [nodes[i].SignProposal(blocks[i % 2], b"aux-%d" % i) for i in range(1, q)]  # two proposals mixed
    bad = 17
    votes[bad] = plugin.Signature(votes[bad].ID, votes[bad - 2].Value, votes[bad].Msg)
    v.coalesce_consenter_sigs(max_batch=q - 1, max_wait_us=20000)
    l0, c0 = v.consenter_stats()
    out = [None] * len(votes)
    start = threading.Barrier(len(votes))

    def call(i):
        start.wait()
        try:
            out[i] = v.VerifyConsenterSig(votes[i], blocks[(i + 1) % 2])
        except plugin.VerifyError as e:
            out[i] = e

    th = [threading.Thread(target=call, args=(i,)) for i in range(len(votes))]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    for i, o in enumerate(out):
        if i == bad:
            assert isinstance(o, plugin.VerifyError) and o.code == plugin.EVERIFY
            assert f"Couldn't verify {votes[i].ID}'s signature: {o}" == \
                f"Couldn't verify {votes[i].ID}'s signature: invalid signature"
        else:
            assert o == b"aux-%d" % (i + 1), (i, o)
    l1, c1 = v.consenter_stats()
    assert c1 - c0 == len(votes) and l1 - l0 <= 8, (l1 - l0, c1 - c0)
    # a lone call after its deadline, and coalescing off again: one launch per call
    assert v.VerifyConsenterSig(votes[0], blocks[1]) == b"aux-1"
    v.coalesce_consenter_sigs(0, 0)
    with pytest.raises(plugin.VerifyError, match="does not bind"):
        v.VerifyConsenterSig(votes[0], blocks[0])
    assert v.consenter_stats() == (l1 + 2, c1 + 2)
    v.close()


def test_consenter_batches_concurrent_on_zero_copy_lanes(gpu):
    """Small keyed batches take one of four zero-copy lanes (own stream, mapped buffer, lock)
    instead of the device lock, so concurrent quorum checks run side by side. 12 threads x 6
    uncoalesced batches each (more callers than lanes: some wait for a lane), every batch with
    its own proposal and a different bad signature: each caller gets exactly its statuses."""
    import threading
    nodes = [plugin.Signer(gpu, i, _priv(("zl", i))) for i in range(1, 18)]
    v = plugin.Verifier(gpu, 1)
    for s in nodes:
        v.add_consenter(s.id, s.public_key())
    T, R = 12, 6
    props = [plugin.Proposal(b"zl-block-%d" % k * 20, b"h", b"m", 1) for k in range(T * R)]
    jobs = []
    for k, p in enumerate(props):
        sigs = [n.SignProposal(p, b"x") for n in nodes]
        bad = k % len(sigs)
        sigs[bad] = plugin.Signature(sigs[bad].ID, sigs[(bad + 1) % len(sigs)].Value, sigs[bad].Msg)
        want = [0] * len(sigs)
        want[bad] = plugin.EVERIFY
        jobs.append((sigs, p, want))
    errors = []
    start = threading.Barrier(T)

    def worker(t):
        start.wait()
        for r in range(R):
            sigs, p, want = jobs[t * R + r]
            got = v.VerifyConsenterSigs(sigs, p)
            if got != want:
                errors.append((t, r, got, want))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    assert not errors, errors[:3]
    v.close()
