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


# ---- radix-2^29 ladder layer (p256_f29.hpp): ops 11..19 ------------------------------------
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5


def _add(p1, p2):
    if p1 is None:
        return p2
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 - 3) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def _mul(k, pt):
    acc = None
    for bit in bin(k)[2:]:
        acc = _add(acc, acc) if acc else None
        if bit == "1":
            acc = _add(acc, pt)
    return acc


def test_f29_mul_sqr_inv(gpu):
    """f29_mul / f29_sqr (Montgomery, R = 2^261) and the safegcd inversion mod p."""
    pairs = [(a % P, b % P) for a, b in _inputs(n_rand=3000, seed=11)]
    _check(pairs, _run(gpu, 11, pairs), lambda a, b: a * b, P, "f29_mul")
    _check(pairs, _run(gpu, 12, pairs), lambda a, b: a * a, P, "f29_sqr")
    xs = [(x, 0) for x, _ in pairs if x % P]
    got = _run(gpu, 13, xs)
    bad = [hex(x) for (x, _), g in zip(xs, got) if g != pow(x, -1, P)]
    assert not bad, bad[:3]


def test_f29_point_ops(gpu):
    """The ladder's lean doubling / mixed / Jacobian additions on random curve points, with the
    doubling loop both rolled and unrolled (same source the verify kernel inlines)."""
    rng = random.Random(5)
    pts = [(GX, GY)] + [_mul(rng.randrange(1, N), (GX, GY)) for _ in range(60)]
    pts += [_mul(k, (GX, GY)) for k in (2, 3, N - 1, N - 2, (N + 1) // 2)]
    x32 = [_mul(32, p) for p in pts]
    assert _run(gpu, 14, pts) == [q[0] for q in x32], "x(32P), rolled doubling loop"
    assert _run(gpu, 15, pts) == [q[0] for q in x32], "x(32P), unrolled doubling loop"
    assert _run(gpu, 16, pts) == [q[1] for q in x32], "y(32P)"
    assert _run(gpu, 17, pts) == [_mul(3, p)[0] for p in pts], "x(2P + P), mixed addition"
    assert _run(gpu, 18, pts) == [_mul(6, p)[1] for p in pts], "y(4P + 2P), Jacobian addition"
    assert _run(gpu, 19, pts) == [_mul(3, p)[1] for p in pts], "y(2P + P), negated twice"


def test_pair_inversion(gpu):
    """inv::inv_mod_pair (the half kernel's table inversion, split over a lane pair: the even lane
    keeps f, g, the odd lane d, e) mod p and mod n, on element 2t's input in both lanes of the pair;
    odd element counts leave the last pair half outside the batch (the kernel still runs it)."""
    rng = random.Random(23)
    for op, mod in ((23, P), (24, N)):
        xs = [0, 1, 2, 3, mod - 1, mod - 2, (1 << 255) % mod, (1 << 224) % mod, 0xFFFFFFFF]
        xs += [rng.randrange(1, mod) for _ in range(1200)]
        for count in (len(xs), len(xs) - 1):
            pairs = [(x, 0) for x in xs[:count]]
            got = _run(gpu, op, pairs)
            want = [pow(xs[i & ~1], -1, mod) if xs[i & ~1] else 0 for i in range(count)]
            bad = [(i, hex(xs[i & ~1])) for i in range(count) if got[i] != want[i]]
            assert not bad, (op, count, bad[:3])


def test_pair_w_ladder(gpu):
    """The half kernel's lane-local W ladder (p29_dbl_plw x5, then the five-step p29_add_aff_plw
    with P itself; c = 1, so W = Z^2) against the group law: x and y of 33P on element 2t's point,
    in both lanes of the pair."""
    rng = random.Random(33)
    pts = [(GX, GY)] + [_mul(rng.randrange(1, N), (GX, GY)) for _ in range(40)]
    pts += [_mul(k, (GX, GY)) for k in (2, 3, N - 1, (N + 1) // 2)]
    want = [_mul(33, pts[i & ~1]) for i in range(len(pts))]
    assert _run(gpu, 25, pts) == [q[0] for q in want], "x(33P)"
    assert _run(gpu, 26, pts) == [q[1] for q in want], "y(33P)"


def test_quad_w_ladder(gpu):
    """The wide half kernel's quad W ladder (p256_f29.hpp q4_dbl / q4_add_rest / q4_add_full; c = 1,
    so W = Z^2) against the group law, on element 4t's point in all four lanes of the quad:
    x and y of 33P (four doublings, a fifth carrying the addition's first step on lanes 2-3, the
    addition's rest with P itself) and of 32P = 33P + (-P) (then a whole addition from the first
    one's N+- Y). Ragged counts leave a partial last quad."""
    rng = random.Random(34)
    pts = [(GX, GY)] + [_mul(rng.randrange(1, N), (GX, GY)) for _ in range(60)]
    pts += [_mul(k, (GX, GY)) for k in (2, 3, 5, N - 1, N - 2, (N + 1) // 2)]
    for count in (len(pts), len(pts) - 1, len(pts) - 2):
        sub = pts[:count]
        want33 = [_mul(33, sub[i & ~3]) for i in range(count)]
        want32 = [_mul(32, sub[i & ~3]) for i in range(count)]
        assert _run(gpu, 27, sub) == [q[0] for q in want33], ("x(33P)", count)
        assert _run(gpu, 28, sub) == [q[1] for q in want33], ("y(33P)", count)
        assert _run(gpu, 29, sub) == [q[0] for q in want32], ("x(32P)", count)
        assert _run(gpu, 30, sub) == [q[1] for q in want32], ("y(32P)", count)
