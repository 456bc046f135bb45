"""Crafted exceptional tuples (tests/golden/p256_crafted.bin, made by tests/golden/gen_crafted.py):
signatures whose scalars make a lean addition of the verify ladders meet acc == +-addend, at
every place one can (p256_f29.hpp add_aff_fix, p256_verify.hip):
  - the last addition of the u2 Q ladder (u2 = n - 2|d|: P + P);
  - each of the 17 comb additions of u1 G, which land on top of u2 Q: with a key Q = q G of
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
KG = 16


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


@pytest.mark.parametrize("mode", ["lane", "pair"])
def test_crafted_exceptional_verdicts(crafted, mode):
    from smartbft_amd import GpuVerifier
    opts = dict(pair_max=-1, quad_max=-1) if mode == "lane" else dict(pair_max=1 << 30, quad_max=-1)
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


def test_crafted_exceptional_framed(crafted):
    """The same tuples as framed requests (VerifyProposal's fused hash + verify launch): the
    digest is SHA-256 of the body, so the crafted scalars need e = SHA-256(body): re-derive s and
    r for each body (u1 = e/s, u2 = r/s kept by choosing s = e/u1, r = u2 s)."""
    from smartbft_amd import GpuVerifier
    cols, tags, want = crafted
    gv = GpuVerifier()
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
