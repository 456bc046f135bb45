"""The multi-device split, run on one GPU.

A host-buffer batch is cut into contiguous shares, one per engine slot, each enqueued and
synchronised by a host worker of its own; there is no collective. `slots_per_device = K`
gives one GPU K slots, each with its own stream, staging, G comb table and registered-key
tables, so every piece of the split runs here as it would on K GPUs:
  - the share plan (sbft_gv_plan_split) and the per-share launches;
  - offset rebasing of hashed / framed messages (each share copies only its slice of the blob);
  - verdict placement (ok_out + share begin) and, for VerifyProposal, the first rejected
    request across shares (view.go:555, the error path view.go:386-393);
  - per-slot comb and key tables (registered clients, consenter keys);
  - the persistent per-share host workers, also under concurrent callers.
Every verdict is checked against the oracle (oracle/p256_oracle.c, Go crypto/ecdsa.Verify
restated) or the golden fixtures, with corruptions placed on both sides of every share edge."""
import threading

import numpy as np
import pytest

import oracle
from conftest import split_fields
from test_gpu_configs import _config5_batch, _corrupt, _tuples

pytestmark = pytest.mark.gpu

SLOTS = [2, 4, 8]


def _gv(k, **kw):
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    gv = GpuVerifier(slots_per_device=k, **kw)
    assert gv.device_count == k * torch.cuda.device_count()
    return gv


def _edges(n, k, min_split=0):
    """Indices on both sides of every internal share boundary, plus the ends."""
    from smartbft_amd.gpuverify import plan_split
    parts = plan_split(n, k, min_split)
    assert len(parts) == (k if n >= (min_split or 65536) else 1)
    out = {0, n - 1}
    for b, c in parts[1:]:
        out |= {b - 1, b}
    return sorted(out), parts


# ---------------------------------------------------------------- config 2: 1M split 8 ways
@pytest.fixture(scope="module")
def workload_1m(gpu):
    from smartbft_amd.workload import make_workload
    wl = make_workload(gpu, 1_000_000, start=777_000)
    return wl.host_fields(), (~wl.corrupted).cpu().numpy().astype(np.uint8)


def test_config2_1m_split_eight_slots(workload_1m):
    """BASELINE config 2 (1M tuples, ~10% corrupted) through sbft_gv_verify_p256 split over 8
    slots (125,000 tuples each, one-lane kernel): every verdict = the construction, the share
    edges = the oracle."""
    f, want = workload_1m
    gv = _gv(8)
    try:
        ok = gv.verify(*f)
        assert np.array_equal(ok, want)
        edges, parts = _edges(len(want), 8)
        assert len(parts) == 8 and all(c == 125_000 for _, c in parts)
        assert np.array_equal(oracle.verify_batch(*[x[edges] for x in f]), ok[edges])
    finally:
        gv.close()


def test_config2_pipelined_shares_two_slots(workload_1m):
    """1.1M tuples over 2 slots: each 550,000-tuple share takes the pipelined path (page-locked
    staging, copy stream overlapped with sub-batch launches on two compute streams), from
    pageable and from page-locked inputs."""
    from smartbft_amd import PinnedArray
    f, want = workload_1m
    extra = 100_000
    f2 = [np.ascontiguousarray(np.concatenate([x, x[:extra]])) for x in f]
    w2 = np.concatenate([want, want[:extra]])
    gv = _gv(2)
    pins = []
    try:
        assert np.array_equal(gv.verify(*f2), w2)
        pins = [PinnedArray(a.shape) for a in f2]
        for p, a in zip(pins, f2):
            p.array[:] = a
        assert np.array_equal(gv.verify(*[p.array for p in pins]), w2)
    finally:
        for p in pins:
            p.close()
        gv.close()


def test_golden_vectors_split_every_slot_count(p256_vectors):
    """The 3,263 golden vectors (18 categories) tiled to 70,000 tuples, split 2 / 4 / 8 ways
    with the default split threshold, and every verdict = the fixture."""
    f, exp, cat, names = p256_vectors
    n = 70_000
    idx = np.arange(n) % len(exp)
    cols = [np.ascontiguousarray(c[idx]) for c in split_fields(f)]
    for k in SLOTS:
        gv = _gv(k)
        try:
            assert np.array_equal(gv.verify(*cols), exp[idx]), k
        finally:
            gv.close()


# ---------------------------------------------------------------- config 3: VerifyProposal
@pytest.fixture(scope="module")
def requests_10k(gpu):
    from smartbft_amd.workload import make_signed_requests
    return make_signed_requests(gpu, 10_000, start=31337)


def _reject_at(v, reqs, where, kind="sig"):
    from smartbft_amd import plugin
    bad = _corrupt(reqs, where, kind)
    want = oracle.verify_batch(*_tuples(bad))
    first = int(np.nonzero(want == 0)[0][0])
    assert first == min(where)
    p = plugin.Proposal(plugin.encode_payload(bad), b"header", b"metadata", 1)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.code == plugin.EVERIFY and ei.value.index == first, (where, ei.value.index)


@pytest.mark.parametrize("k", SLOTS)
@pytest.mark.parametrize("clients", ["generic", "registered"])
def test_config3_verify_proposal_split(requests_10k, k, clients):
    """A 10,000-request proposal split over k slots (min_split = 1): the framed launch per
    share hashes its slice of the payload (offsets rebased) and gathers the tuples in place;
    with every client key registered each share takes the keyed launch over its own slot's
    client tables. A bad request on either side of every share edge, and all of them at once,
    is reported at the oracle's first rejected index."""
    from smartbft_amd import plugin
    reqs = requests_10k
    gv = _gv(k, min_split=1)
    v = plugin.Verifier(gv, 1)
    try:
        if clients == "registered":
            v.add_clients([q[-129:-64] for q in reqs])
        p = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
        infos = v.VerifyProposal(p)
        assert [(i.ClientID, i.ID) for i in infos] == [(f"client{31337 + i}", f"tx{31337 + i}") for i in range(10_000)]
        edges, parts = _edges(10_000, k, 1)
        assert len(parts) == k
        for e in edges:
            _reject_at(v, reqs, [e])
        _reject_at(v, reqs, [e for e in edges if e > 0], "payload")  # first bad one in a later share
        _reject_at(v, reqs, edges, "key")
    finally:
        v.close()
        gv.close()


# ---------------------------------------------------------------- hashing and config 5
@pytest.fixture(scope="module")
def config5_small():
    return _config5_batch(600, seed=61)


@pytest.mark.parametrize("k", SLOTS)
def test_hash_and_fused_verify_split(config5_small, k):
    """sbft_gv_sha256 and sbft_gv_sha256_verify_p256 split over k slots (min_split = 1): each
    share copies only its span of the blob and rebases its offsets; digests and verdicts land
    at their global indices."""
    blob, off, ln, cols, dig, want = config5_small
    gv = _gv(k, min_split=1)
    try:
        assert np.array_equal(gv.sha256(blob, off, ln), dig)
        ok, got = gv.sha256_verify(blob, off, ln, *cols, want_digests=True)
        assert np.array_equal(got, dig) and np.array_equal(ok, want)
        # a permuted listing: shares cover scattered spans of the blob
        perm = np.random.default_rng(k).permutation(len(off))
        ok2 = gv.sha256_verify(blob, off[perm], ln[perm], *[c[perm] for c in cols])
        assert np.array_equal(ok2, want[perm])
    finally:
        gv.close()


@pytest.mark.parametrize("k", SLOTS)
def test_config5_streamed_split(config5_small, k):
    """BASELINE config 5's streamed hash -> verify with the messages split over k slots
    (min_split = 1), each slot streaming its share through its own six stages; 1 MiB windows
    force many windows per share."""
    blob, off, ln, cols, dig, want = config5_small
    gv = _gv(k, min_split=1)
    try:
        ok, got = gv.sha256_verify_stream(blob, off, ln, *cols, window_bytes=1 << 20, want_digests=True)
        assert np.array_equal(got, dig) and np.array_equal(ok, want)
    finally:
        gv.close()


# ---------------------------------------------------------------- registered keys, signer
@pytest.mark.parametrize("n", [2000, 5000])
def test_keyed_split_golden(p256_vectors, n):
    """Registered-key verify split over 4 slots (min_split = 1): every slot builds the tables
    of every key; shares of 500 take the zero-copy lanes, shares of 1,250 the pinned four-lane
    launch. Verdicts = the fixtures (an unregistrable key verifies false, as the fixture says)."""
    f, exp, cat, names = p256_vectors
    sub = f[:1500]
    gv = _gv(4, min_split=1)
    try:
        ids = gv.register_keys(np.ascontiguousarray(sub[:, 96:128]), np.ascontiguousarray(sub[:, 128:160]))
        idx = np.arange(n) % len(sub)
        g = sub[idx]
        ok = gv.verify_keyed(np.ascontiguousarray(g[:, 0:32]), np.ascontiguousarray(g[:, 32:64]),
                             np.ascontiguousarray(g[:, 64:96]), ids[idx])
        assert np.array_equal(ok, exp[:1500][idx])
    finally:
        gv.close()


def test_sign_split_matches_oracle():
    """10,000 signatures (past the wavefront signer's 4,096) split over 4 slots: r, s and Q
    byte for byte the oracle's."""
    rng = np.random.default_rng(9)
    n = 10_000
    d = [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(n)]
    k = [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(n)]
    b32 = lambda xs: np.frombuffer(b"".join(x.to_bytes(32, "big") for x in xs), dtype=np.uint8).reshape(-1, 32)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    gv = _gv(4, min_split=1)
    try:
        qx, qy, r, s, st = gv.sign(b32(d), b32(k), e)
        assert st.all()
        for i in (0, 2499, 2500, 4999, 5000, 7499, 7500, n - 1):
            x, y = oracle.pubkey(d[i])
            rr, ss = oracle.sign(d[i], k[i], bytes(e[i]))
            assert (bytes(qx[i]), bytes(qy[i]), bytes(r[i]), bytes(s[i])) == (x, y, rr, ss), i
        assert oracle.verify_batch(e, r, s, qx, qy).all()
    finally:
        gv.close()


def test_concurrent_split_callers(p256_vectors):
    """Six threads issuing split calls on one 4-slot context at once: shares of different calls
    queue on the same per-share workers and slot locks; every caller gets its own verdicts."""
    f, exp, cat, names = p256_vectors
    gv = _gv(4, min_split=1)
    errs = []

    def run(t):
        try:
            rng = np.random.default_rng(100 + t)
            for _ in range(3):
                idx = rng.integers(0, len(exp), size=int(rng.integers(1000, 40_000)))
                cols = [np.ascontiguousarray(c[idx]) for c in split_fields(f)]
                if not np.array_equal(gv.verify(*cols), exp[idx]):
                    errs.append(t)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(repr(e))

    try:
        th = [threading.Thread(target=run, args=(t,)) for t in range(6)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs
    finally:
        gv.close()
