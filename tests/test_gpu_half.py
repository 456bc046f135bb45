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
MODES = {"half": dict(half_max=1 << 30, halfq_max=-1), "halfw": dict(halfq_max=1 << 30),
         "pair": dict(pair_max=1 << 30, half_max=-1),
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


def _twist_small_order_r(rng, q):
    """r such that x = r lies on the quadratic twist (r^3 - 3r + b a non-square) as the x of a
    point of order q (q | the twist's order: 3, 5, 13, 179). The half kernel's pair B then runs on
    E_c, c = r^3 - 3r + b, from P' = (c r, c^2) -- a point of order q on the twist -- so its table
    build and ladder meet infinity and doublings of equal points by construction."""
    P, B = pyref.P, pyref.B
    nt = 2 * P + 2 - N  # the twist's order
    assert nt % q == 0
    d = next(x for x in range(2, 100) if pow(x, (P - 1) // 2, P) == P - 1)  # a non-square
    a, b = (-3 * d * d) % P, B * d ** 3 % P  # E_d: y^2 = x^3 + a x + b, the twist

    def add(p1, p2):
        if p1 is None:
            return p2
        if p2 is None:
            return p1
        (x1, y1), (x2, y2) = p1, p2
        if x1 == x2 and (y1 + y2) % P == 0:
            return None
        if p1 == p2:
            lam = (3 * x1 * x1 + a) * pow(2 * y1, -1, P) % P
        else:
            lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
        x3 = (lam * lam - x1 - x2) % P
        return x3, (lam * (x1 - x3) - y1) % P

    def mul(k, pt):
        acc = None
        while k:
            if k & 1:
                acc = add(acc, pt)
            pt = add(pt, pt)
            k >>= 1
        return acc

    while True:
        x = rng.randrange(P)
        rhs = (x ** 3 + a * x + b) % P
        y = pow(rhs, (P + 1) // 4, P)
        if y * y % P != rhs:
            continue
        T = mul(nt // q, (x, y))
        if T is None:
            continue
        r = T[0] * pow(d, -1, P) % P  # the x-line of the curve: x_E = x_{E_d} / d
        c = (r ** 3 - 3 * r + B) % P
        assert pow(c, (P - 1) // 2, P) == P - 1  # no point of the curve has x = r
        if r < N:
            return r


def test_twist_small_order_r():
    """Pair B's arithmetic on the twist must only ever be discarded: r from small-order twist
    points (the table's 3P', 5P', ... hit infinity), with valid-looking s, Q and digest, mixed with
    honest signatures in one batch. Every kernel must reject them, as the oracle (Go) does, and
    leave the honest neighbours' verdicts alone."""
    from smartbft_amd import GpuVerifier
    rng = random.Random(31337)
    recs = []
    for q in (3, 5, 13, 179):
        for _ in range(3):
            r = _twist_small_order_r(rng, q)
            Q = pyref.mul(rng.randrange(1, N), pyref.G)
            recs.append((rng.randrange(N), r, rng.randrange(1, N), Q[0], Q[1]))
    honest = []
    while len(honest) < len(recs):
        t = _signature_for(rng.randrange(1, N), rng.randrange(1, N), rng.randrange(1, N))
        if t is not None:
            honest.append(t)
    recs = [x for pair in zip(honest, recs) for x in pair]  # honest, crafted, honest, ...
    cols = [np.zeros((len(recs), 32), dtype=np.uint8) for _ in range(5)]
    for i, rec in enumerate(recs):
        for k, v in enumerate(rec):
            cols[k][i] = np.frombuffer(int(v).to_bytes(32, "big"), dtype=np.uint8)
    want = oracle.verify_batch(*cols)
    assert np.array_equal(want, np.arange(len(recs)) % 2 == 0)
    for mode in MODES:
        gv = GpuVerifier(device_mask=1, **MODES[mode])
        try:
            got = gv.verify(*cols)
            assert np.array_equal(got, want), (mode, np.nonzero(got != want)[0][:10])
            idx = np.random.default_rng(5).permutation(np.arange(2000) % len(want))
            assert np.array_equal(gv.verify(*[c[idx] for c in cols]), want[idx]), mode
        finally:
            gv.close()
