"""The proposal parse over several threads (verifier.cpp parse_payload_par): large proposals are
walked from several candidate request boundaries at once and joined where the chains meet. It
must accept and reject exactly the payloads the sequential parse does, report the same first
bad request, and survive payloads crafted to defeat the speculation (request-looking bytes
inside payloads). CPU only: RequestsFromProposal and a parse-only VerifyProposal (no engine).
RequestsFromProposal and VerifyProposal parse on 1 thread by default (verifier.cpp
parse_threads_for); SBFT_PARSE_THREADS sets both, once per process, so every case runs again in a
child process with 3 threads."""
import os
import subprocess
import sys

import numpy as np
import pytest

from smartbft_amd import plugin


def _req(i: int, rng, pl: bytes | None = None, key0: int = 0x04) -> bytes:
    cid, rid = f"client{i}".encode(), f"tx{i}".encode()
    if pl is None:
        pl = rng.bytes(int(rng.integers(64, 257)))
    key = bytes([key0]) + rng.bytes(64)
    body = (b"SBR1" + len(cid).to_bytes(2, "little") + cid + len(rid).to_bytes(2, "little") + rid +
            len(pl).to_bytes(4, "little") + pl + key)
    return body + rng.bytes(64)


def _want(n):
    return [(f"client{i}", f"tx{i}") for i in range(n)]


def _ids(infos):
    return [(x.ClientID, x.ID) for x in infos]


@pytest.fixture(scope="module")
def reqs():
    rng = np.random.default_rng(11)
    return [_req(i, rng) for i in range(6000)]  # ~1.8 MB: the parallel path (>= 2048 requests, >= 256 KB)


def test_large_proposal_parses_in_order(reqs):
    v = plugin.Verifier(None)
    p = plugin.Proposal(plugin.encode_payload(reqs), b"h", b"m", 0)
    assert _ids(v.RequestsFromProposal(p)) == _want(len(reqs))
    # no engine: the parse and the format checks run, then the call reports the missing GPU
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.code != plugin.EFORMAT
    v.close()


@pytest.mark.parametrize("where", [0.0, 0.33, 0.34, 0.5, 0.66, 0.67, 0.999])
def test_false_boundaries_inside_payloads(where):
    """Some requests carry, inside their payload, bytes that form a complete length-prefixed
    request (a speculative walker starting there follows a false chain): the join must reject it
    and the list must still be exact."""
    rng = np.random.default_rng(int(where * 1000) + 5)
    out = []
    n = 5000
    fake_at = int(where * n)
    for i in range(n):
        if fake_at - 40 <= i <= fake_at + 40:
            inner = _req(10_000 + i, rng)
            pl = rng.bytes(int(rng.integers(0, 40))) + len(inner).to_bytes(4, "little") + inner + rng.bytes(8)
            out.append(_req(i, rng, pl=pl))
        else:
            out.append(_req(i, rng))
    v = plugin.Verifier(None)
    p = plugin.Proposal(plugin.encode_payload(out), b"h", b"m", 0)
    assert _ids(v.RequestsFromProposal(p)) == _want(n)
    v.close()


def test_every_payload_full_of_fake_headers(reqs):
    """Every request's payload is request-looking bytes: the candidate scan is bounded and the
    list still exact."""
    rng = np.random.default_rng(3)
    fake = _req(99, rng)
    out = [_req(i, rng, pl=(len(fake).to_bytes(4, "little") + fake)[: int(rng.integers(64, 257))]) for i in range(4000)]
    v = plugin.Verifier(None)
    assert _ids(v.RequestsFromProposal(plugin.Proposal(plugin.encode_payload(out), b"h", b"m", 0))) == _want(4000)
    v.close()


def _malformed(v, payload):
    p = plugin.Proposal(payload, b"h", b"m", 0)
    assert v.RequestsFromProposal(p) == []
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(p)
    assert ei.value.code == plugin.EFORMAT and "malformed proposal payload" in str(ei.value)


def test_malformed_large_payloads(reqs):
    v = plugin.Verifier(None)
    good = plugin.encode_payload(reqs)
    n = len(reqs)
    _malformed(v, (n + 1).to_bytes(4, "little") + good[4:])          # count says one more
    _malformed(v, (n - 1).to_bytes(4, "little") + good[4:])          # count says one fewer
    _malformed(v, good[:-1])                                          # truncated
    _malformed(v, good + b"\0")                                       # trailing byte
    for frac in (0.1, 0.5, 0.9):                                      # a bad length prefix late on
        k = int(frac * n)
        off = 4 + sum(4 + len(r) for r in reqs[:k])
        bad = bytearray(good)
        bad[off:off + 4] = (len(reqs[k]) + 3).to_bytes(4, "little")
        _malformed(v, bytes(bad))
        bad = bytearray(good)
        bad[off + 4] = ord("X")                                       # a broken magic
        _malformed(v, bytes(bad))
    v.close()


@pytest.mark.parametrize("bad", [[4999], [1200, 4700], [3001]])
def test_first_bad_key_reported_in_order(bad):
    rng = np.random.default_rng(17)
    out = [_req(i, rng, key0=0x02 if i in bad else 0x04) for i in range(5000)]
    v = plugin.Verifier(None)
    with pytest.raises(plugin.VerifyError) as ei:
        v.VerifyProposal(plugin.Proposal(plugin.encode_payload(out), b"h", b"m", 0))
    i = min(bad)
    assert ei.value.code == plugin.EFORMAT and ei.value.index == i
    assert f"request {i} (client{i}:tx{i}): public key is not SEC1 uncompressed" in str(ei.value)
    v.close()


def test_verify_proposal_parallel_prepare_in_child():
    """Every case above with SBFT_PARSE_THREADS=3: the parallel walk and join of
    RequestsFromProposal, and VerifyProposal's parallel prepare (per-range format checks, first
    bad key by atomic minimum)."""
    env = dict(os.environ, SBFT_PARSE_THREADS="3")
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r); import pytest; "
            "sys.exit(pytest.main(['-q', '-p', 'no:cacheprovider', %r, '-k', "
            "'not in_child']))" % (here, os.path.join(here, "test_parse_parallel.py")))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600,
                       cwd=os.path.dirname(here))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def _ref_parse(payload: bytes, keys=None):
    """The payload format restated (verifier.cpp parse_payload / parse_request): u32 count, then
    count x (u32 length, request); a request is "SBR1", u16 + client id, u16 + request id, u32 +
    body, 65-byte key, 64-byte signature, nothing after it; ids without NUL bytes. Any deviation
    rejects the whole payload (None)."""
    def u(b, at, n):
        return int.from_bytes(b[at:at + n], "little") if at + n <= len(b) else None
    keys = [] if keys is None else keys
    count = u(payload, 0, 4)
    if count is None or count > len(payload) // 4:
        return None
    at, out = 4, []
    for _ in range(count):
        ln = u(payload, at, 4)
        if ln is None or at + 4 + ln > len(payload):
            return None
        r = payload[at + 4:at + 4 + ln]
        at += 4 + ln
        if r[:4] != b"SBR1":
            return None
        a = u(r, 4, 2)
        if a is None or 6 + a > len(r):
            return None
        cid, q = r[6:6 + a], 6 + a
        b = u(r, q, 2)
        if b is None or q + 2 + b > len(r):
            return None
        rid, q = r[q + 2:q + 2 + b], q + 2 + b
        c = u(r, q, 4)
        if c is None or q + 4 + c + 65 + 64 != len(r) or b"\0" in cid or b"\0" in rid:
            return None
        out.append((cid.decode("utf-8", "surrogateescape"), rid.decode("utf-8", "surrogateescape")))
        keys.append(r[q + 4 + c])
    return out if at == len(payload) else None


def _parsed(v, payload):
    infos = v.RequestsFromProposal(plugin.Proposal(payload, b"h", b"m", 0))
    return [(x.ClientID, x.ID) for x in infos]


@pytest.mark.parametrize("seed", range(4))
def test_random_mutations_match_the_format(reqs, seed):
    """Differential fuzz: a large proposal (the 3-thread parse) with 1-3 random edits -- byte
    flips, inserted or deleted bytes, some aimed at length prefixes and ids -- is accepted with
    exactly the requests the restated format yields, or rejected exactly when it rejects."""
    rng = np.random.default_rng(100 + seed)
    good = plugin.encode_payload(reqs)
    starts = np.cumsum([4] + [4 + len(r) for r in reqs[:-1]])
    v = plugin.Verifier(None)
    accepted = rejected = 0
    for _ in range(40):
        b = bytearray(good)
        for _ in range(int(rng.integers(1, 4))):
            kind = int(rng.integers(0, 5))
            k = int(rng.integers(0, len(reqs)))
            if kind == 0:    # a length prefix
                at = int(starts[k]) + int(rng.integers(0, 4))
            elif kind == 1:  # inside the ids
                at = int(starts[k]) + 4 + int(rng.integers(4, 20))
            else:            # anywhere
                at = int(rng.integers(0, len(b)))
            at = min(at, len(b) - 1)
            if kind == 3:
                del b[at]
            elif kind == 4:
                b.insert(at, int(rng.integers(0, 256)))
            else:
                b[at] ^= 1 << int(rng.integers(0, 8))
        keys = []
        want = _ref_parse(bytes(b), keys)
        got = _parsed(v, bytes(b))
        assert got == (want or []), "mutation parsed differently"
        # VerifyProposal's format verdict (parse-only verifier: a well-formed proposal reaches
        # the missing engine instead): malformed payload, else the first non-SEC1 key in order
        with pytest.raises(plugin.VerifyError) as ei:
            v.VerifyProposal(plugin.Proposal(bytes(b), b"h", b"m", 0))
        bad_key = next((i for i, k0 in enumerate(keys) if k0 != 0x04), None)
        if want is None or bad_key is not None:
            assert ei.value.code == plugin.EFORMAT
            if want is not None:
                assert ei.value.index == bad_key
        else:
            assert ei.value.code != plugin.EFORMAT
        accepted += want is not None
        rejected += want is None
    assert rejected > 0
    v.close()


def test_random_small_payloads_match_the_format():
    """The sequential parse on short random and near-valid payloads (no crash, same verdict)."""
    rng = np.random.default_rng(7)
    v = plugin.Verifier(None)
    base = plugin.encode_payload([_req(i, rng) for i in range(5)])
    for n in range(300):
        if n % 3 == 0:
            pl = rng.bytes(int(rng.integers(0, 64)))
        else:
            b = bytearray(base)
            for _ in range(int(rng.integers(1, 3))):
                b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            pl = bytes(b[: int(rng.integers(len(b) - 8, len(b) + 1))]) if n % 3 == 2 else bytes(b)
        want = _ref_parse(pl)
        assert _parsed(v, pl) == (want or [])
    v.close()
