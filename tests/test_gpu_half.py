"""The half-size-scalar kernel's own edge cases (p256_verify_half_kernel): signatures
built around a prescribed u2 = r / s, so that the Euclid reduction to (v, w) meets its limits --
u2 below 2^128 (no step), quotients at and past the 2^31 give-up bound (the in-kernel classic
fallback), long all-ones quotient runs, u2 near n -- each valid and corrupted, mixed into one
batch so that fallback and half-size lanes share wavefronts. Verdicts must equal the oracle's on
every kernel (the half kernel forced on, the pair and throughput kernels for comparison)."""
import random

import numpy as np
import pytest

import oracle
from oracle import pyref

pytestmark = pytest.mark.gpu

N = pyref.N
MODES = {"half": dict(half_max=1 << 30), "pair": dict(pair_max=1 << 30, half_max=-1),
         "lane": dict(pair_max=-1, half_max=-1)}


def _signature_for(u1: int, u2: int, q: int):
    """A valid (e, r, s, Q) whose scalars are u1 = e / s and u2 = r / s (key recovery:
    R = (u1 + u2 q) G, r = x(R) mod n, s = r / u2, e = u1 s); None if r came out 0."""
    Q = pyref.mul(q, pyref.G)
    R = pyref.mul((u1 + u2 * q) % N, pyref.G)
    if R is None:
        return None
    r = R[0] % N
    if r == 0:
        return None
    s = r * pow(u2, -1, N) % N
    e = u1 * s % N
    return e, r, s, Q[0], Q[1]


def _u2_cases(rng):
    fib = [1, 2]
    while fib[-1] < N:
        fib.append(fib[-1] + fib[-2])
    out = [1, 2, 3, 5, (1 << 127) + 1, (1 << 128) - 1, 1 << 128, (1 << 128) + 1, N - 1, N - 2, N // 2,
           N // ((1 << 31) - 1), N // (1 << 31), N // (1 << 31) + 1, N // (1 << 40), N // (1 << 100),
           N // 3 + 1, fib[-2] % N, fib[-3] % N]
    out += [(N * k) // ((1 << 33) + k) for k in range(1, 6)]  # a large quotient a few steps in
    out += [rng.randrange(1, N) for _ in range(24)]
    return [u % N or 1 for u in out]


@pytest.fixture(scope="module")
def crafted_u2():
    rng = random.Random(404)
    recs, want = [], []
    for u2 in _u2_cases(rng):
        for _ in range(2):
            t = _signature_for(rng.randrange(1, N), u2, rng.randrange(1, N))
            if t is None:
                continue
            e, r, s, qx, qy = t
            recs.append((e, r, s, qx, qy))
            recs.append((e, r, (s + 1) % N or 1, qx, qy))  # corrupted: u2 moves
            recs.append((e ^ 1, r, s, qx, qy))              # corrupted: u1 moves, u2 kept
    cols = [np.zeros((len(recs), 32), dtype=np.uint8) for _ in range(5)]
    for i, rec in enumerate(recs):
        for k, v in enumerate(rec):
            cols[k][i] = np.frombuffer(int(v).to_bytes(32, "big"), dtype=np.uint8)
    want = oracle.verify_batch(*cols)
    assert want.sum() >= len(recs) // 3 - 2  # the valid third verifies
    return cols, want


@pytest.mark.parametrize("mode", list(MODES))
def test_prescribed_u2_edges(crafted_u2, mode):
    from smartbft_amd import GpuVerifier
    cols, want = crafted_u2
    gv = GpuVerifier(device_mask=1, **MODES[mode])
    try:
        got = gv.verify(*cols)
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
        # tiled into a proposal-sized batch, shuffled among honest-looking ones: fallback and
        # half-size lanes share wavefronts and workgroups
        rng = np.random.default_rng(7)
        idx = rng.permutation(np.arange(4000) % len(want))
        assert np.array_equal(gv.verify(*[c[idx] for c in cols]), want[idx])
    finally:
        gv.close()
