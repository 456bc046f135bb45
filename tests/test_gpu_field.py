"""GPU unit tests of the field / scalar primitives (sbft_gv_selftest_field) against Python
big integers, on edge values the ECDSA vectors do not all reach (lazy-reduced inputs in
[p, 2^256), carries out of the top limb, zero)."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
R = 1 << 256
EDGE = [0, 1, 2, 3, P - 1, P, P + 1, P + 2, R - 1, R - 2, N - 1, N, N + 1, 1 << 255, 1 << 224,
        (1 << 224) - 1, R - P, R - P - 1, 0xFFFFFFFF, 1 << 32, (1 << 192) + 1, 2 * (R - P),
        R - 1 - (1 << 96)]


def _inputs(n_rand=3000, lo=0, hi=R, seed=1):
    rng = random.Random(seed)
    pairs = [(a, b) for a in EDGE for b in EDGE]
    pairs += [(rng.randrange(lo, hi), rng.randrange(lo, hi)) for _ in range(n_rand)]
    pairs += [(rng.randrange(P, R), rng.randrange(P, R)) for _ in range(300)]  # lazy range
    return pairs


def _run(gpu, op, pairs):
    a = np.frombuffer(b"".join(x.to_bytes(32, "big") for x, _ in pairs), dtype=np.uint8).reshape(-1, 32)
    b = np.frombuffer(b"".join(y.to_bytes(32, "big") for _, y in pairs), dtype=np.uint8).reshape(-1, 32)
    out = gpu.selftest_field(op, a, b)
    return [int.from_bytes(o.tobytes(), "big") for o in out]


def _check(pairs, got, ref, mod, name):
    bad = [(hex(a), hex(b), hex(g)) for (a, b), g in zip(pairs, got) if (g - ref(a, b)) % mod]
    assert not bad, (name, len(bad), bad[:3])


def test_fp_mul_sqr(gpu):
    pairs = _inputs()
    rinv = pow(R, -1, P)
    _check(pairs, _run(gpu, 0, pairs), lambda a, b: a * b * rinv, P, "fp_mul")
    _check(pairs, _run(gpu, 1, pairs), lambda a, b: a * a * rinv, P, "fp_sqr")


def test_fp_add_sub(gpu):
    pairs = _inputs()
    _check(pairs, _run(gpu, 2, pairs), lambda a, b: a + b, P, "fp_add")
    _check(pairs, _run(gpu, 3, pairs), lambda a, b: a - b, P, "fp_sub")


def test_fn_mul(gpu):
    pairs = _inputs()
    rinv = pow(R, -1, N)
    _check(pairs, _run(gpu, 4, pairs), lambda a, b: a * b * rinv, N, "fn_mul")


def test_inversions(gpu):
    rng = random.Random(7)
    xs = [1, 2, P - 1, N - 1, R - 1, 1 << 255] + [rng.randrange(1, P) for _ in range(500)]
    pairs = [(x, 0) for x in xs]
    got = _run(gpu, 5, pairs)
    for (x, _), g in zip(pairs, got):
        if x % P:
            assert (g * x - R * R) % P == 0, hex(x)
    xs = [x for x in xs if x % N]
    pairs = [(x, 0) for x in xs]
    got = _run(gpu, 6, pairs)
    for (x, _), g in zip(pairs, got):
        assert (g * x - R * R) % N == 0, hex(x)


def test_canonical_forms(gpu):
    pairs = _inputs(500)
    assert _run(gpu, 7, pairs) == [a % P for a, _ in pairs]
    assert _run(gpu, 8, pairs) == [a % N for a, _ in pairs]
    small = [(a % N, b % N) for a, b in pairs]
    assert _run(gpu, 9, small) == [(a + b) % N for a, b in small]
