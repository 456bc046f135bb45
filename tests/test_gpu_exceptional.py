"""Crafted exceptional tuples (tests/golden/p256_crafted.bin, made by tests/golden/gen_crafted.py):
signatures whose scalars make a lean addition of the verify ladders meet acc == +-addend, at
every place one can (p256_f29.hpp add_aff_fix, p256_verify.hip):
  - the last addition of the u2 Q ladder (u2 = n - 2|d|: P + P);
  - each of the 13 comb additions of u1 G (12 windows of 22 bits + 2^264 G), which land on top of u2 Q: with a key Q = q G of
    known q the attacker picks q so that u2 q + (the comb's partial sum) = +-(the next entry),
    giving a doubling (P + P) or the point at infinity (P + (-P)) at that step; at the last
    entry the infinity case is R = infinity itself.
A client controls Q, r and s of its own request (and hence u1 = e/s, u2 = r/s), so each of these
is reachable by a crafted proposal; they are verified in place (no fix-up pass). Verdicts
against the fixture and the oracle (oracle/p256_oracle.c, Go crypto/ecdsa.Verify restated), on
the one-lane throughput kernel and the two-lane latency kernel, one by one and tiled into a
10k batch, and as framed requests."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

N = oracle.N


def _b(x: int) -> bytes:
    return (x % (1 << 256)).to_bytes(32, "big")


def load_crafted():
    raw = np.fromfile(os.path.join(GOLDEN, "p256_crafted.bin"), dtype=np.uint8).reshape(-1, 162)
    names = json.load(open(os.path.join(GOLDEN, "p256_crafted.json")))["tags"]
    cols = [np.ascontiguousarray(raw[:, 32 * k:32 * k + 32]) for k in range(5)]
    return cols, [names[i] for i in raw[:, 161]], raw[:, 160].copy()


@pytest.fixture(scope="module")
def crafted():
    cols, tags, want = load_crafted()
    assert np.array_equal(oracle.verify_batch(*cols), want)
    return cols, tags, want


MODE_OPTS = {"lane": dict(pair_max=-1, half_max=-1),
             "pair": dict(pair_max=1 << 30, half_max=-1),
             "half": dict(half_max=1 << 30, halfq_max=-1),
             "halfw": dict(halfq_max=1 << 30)}


@pytest.mark.parametrize("mode", ["lane", "pair", "half", "halfw"])
def test_crafted_exceptional_verdicts(crafted, mode):
    from smartbft_amd import GpuVerifier
    opts = MODE_OPTS[mode]
    gv = GpuVerifier(**opts)
    try:
        cols, tags, want = crafted
        got = gv.verify(*cols)
        bad = [t for t, g, w in zip(tags, got, want) if g != w]
        assert not bad, bad
        # tiled into an adversarial proposal-sized batch, and mixed with honest tuples
        idx = np.arange(10_000) % len(tags)
        assert np.array_equal(gv.verify(*[c[idx] for c in cols]), want[idx])
    finally:
        gv.close()


@pytest.mark.parametrize("mode", ["pair", "half", "halfw"])
def test_crafted_exceptional_framed(crafted, mode):
    """The same tuples as framed requests (VerifyProposal's fused hash + verify launch): the
    digest is SHA-256 of the body, so the crafted scalars need e = SHA-256(body): re-derive s and
    r for each body (u1 = e/s, u2 = r/s kept by choosing s = e/u1, r = u2 s)."""
    from smartbft_amd import GpuVerifier
    cols, tags, want = crafted
    gv = GpuVerifier(**MODE_OPTS[mode])
    try:
        rng = np.random.default_rng(3)
        parts, off, lens, exp = [], [], [], []
        pos = 0
        for i in range(len(tags)):
            e0, r0, s0 = (int.from_bytes(bytes(cols[k][i]), "big") for k in range(3))
            u1 = e0 * pow(s0, -1, N) % N
            u2 = r0 * pow(s0, -1, N) % N
            qx, qy = bytes(cols[3][i]), bytes(cols[4][i])
            body = rng.bytes(int(rng.integers(64, 300))) + qx + qy
            e = int.from_bytes(hashlib.sha256(body).digest(), "big") % N
            if e == 0 or u1 == 0:
                continue
            s = e * pow(u1, -1, N) % N
            r = u2 * s % N
            if r == 0:
                continue
            exp.append(oracle.verify_batch(*[np.frombuffer(x, dtype=np.uint8).reshape(1, 32) for x in
                                             (hashlib.sha256(body).digest(), _b(r), _b(s), qx, qy)])[0])
            off.append(pos)
            lens.append(len(body))
            parts.append(body + _b(r) + _b(s))
            pos += len(body) + 64
        blob = np.frombuffer(b"".join(parts), dtype=np.uint8)
        got = gv.sha256_verify_framed(blob, np.array(off), np.array(lens), 0, -64)
        assert np.array_equal(got, np.array(exp, dtype=np.uint8))
    finally:
        gv.close()


def _sbr1(i: int, pl: bytes, qx: bytes, qy: bytes) -> bytes:
    cid, rid = f"c{i}".encode(), f"r{i}".encode()
    return (b"SBR1" + len(cid).to_bytes(2, "little") + cid + len(rid).to_bytes(2, "little") + rid +
            len(pl).to_bytes(4, "little") + pl + b"\x04" + qx + qy)


@pytest.mark.parametrize("mode", ["pair", "half", "halfw"])
def test_crafted_exceptional_proposal(crafted, mode):
    """The crafted tuples as signed requests inside a VerifyProposal of honest ones
    (sbft_gv_framed_overlapped: fused hash + verify launch, verdicts in mapped host memory).
    SBR1 signs the client's key, so a crafted request keeps u1 = e/s and u2 = r/s (the scalars
    that make the ladder or the comb meet an exceptional addition) but not a valid r: each is a
    rejection. The two-lane kernel repairs them in place; the half-size-scalar kernel meets no
    exceptional addition on its 128-bit ladders and repairs its comb join in place, and any tuple
    either flags goes to the fix-up kernel, launched only because the verify kernel raised the
    mapped flag. Each crafted request replaces an honest one of an all-valid proposal of the same size
    verified just before (whose verdict bytes, all 1, are still in the mapped buffer), so a
    skipped fix-up would show as an accepted proposal; the error must name that request."""
    from smartbft_amd import GpuVerifier, plugin
    cols, tags, want = crafted
    opts = MODE_OPTS[mode]
    gv = GpuVerifier(**opts)
    v = plugin.Verifier(gv)
    try:
        rng = np.random.default_rng(5)
        honest = []
        for i in range(96):
            d = int.from_bytes(rng.bytes(32), "big") % N or 1
            k = int.from_bytes(rng.bytes(32), "big") % N or 1
            qx, qy = oracle.pubkey(d)
            body = _sbr1(i, rng.bytes(int(rng.integers(16, 200))), qx, qy)
            r, s = oracle.sign(d, k, hashlib.sha256(body).digest())
            honest.append(body + r + s)
        assert len(v.VerifyProposal(plugin.Proposal(plugin.encode_payload(honest)))) == len(honest)
        tried = 0
        for j in range(0, len(tags), max(1, len(tags) // 12)):
            e0, r0, s0 = (int.from_bytes(bytes(cols[k][j]), "big") for k in range(3))
            u1, u2 = e0 * pow(s0, -1, N) % N, r0 * pow(s0, -1, N) % N
            qx, qy = bytes(cols[3][j]), bytes(cols[4][j])
            body = _sbr1(1000 + j, rng.bytes(int(rng.integers(16, 200))), qx, qy)
            e = int.from_bytes(hashlib.sha256(body).digest(), "big") % N
            if e == 0 or u1 == 0:
                continue
            s = e * pow(u1, -1, N) % N
            r = u2 * s % N
            if r == 0:
                continue
            assert not oracle.verify_batch(*[np.frombuffer(x, dtype=np.uint8).reshape(1, 32) for x in
                                             (hashlib.sha256(body).digest(), _b(r), _b(s), qx, qy)])[0]
            at = (7 * j) % len(honest)
            reqs = honest[:at] + [body + _b(r) + _b(s)] + honest[at + 1:]
            with pytest.raises(plugin.VerifyError) as ei:
                v.VerifyProposal(plugin.Proposal(plugin.encode_payload(reqs)))
            assert ei.value.index == at, (tags[j], at, ei.value.index)
            # the all-valid proposal again (its verdict bytes back to 1 for the next round)
            assert len(v.VerifyProposal(plugin.Proposal(plugin.encode_payload(honest)))) == len(honest)
            tried += 1
        assert tried >= 8
    finally:
        v.close()
        gv.close()
