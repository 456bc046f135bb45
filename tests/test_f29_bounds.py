"""Overflow and limb-range model of the radix-2^29 field arithmetic (smartbft_amd/csrc/p256_f29.hpp),
run on the CPU: every product column, every 64-bit accumulator and every 32-bit limb of the
throughput kernel's doubling (p29_dbl_f) and mixed addition (p29_add_aff_lean_f), including the
products with addends (f29_mulsq_add) and the carry-only tripling (f29_triple), is restated here
in Python integers and checked against the int64 / int32 widths the GPU computes in, while the
values are checked against the curve (oracle/pyref.py, the group law in Python big integers).

The inputs are not just canonical: before every operation each value is re-limbed at random
inside its stated contract (N: limbs 0..7 in [0, 2^29); N': limbs 0..7 in (-2^26, 2^29 + 2^26),
limb 8 in [0, 2^24); N+-: |limb| < 2^29), value unchanged, so the column bounds are exercised
near the edges the comments at each use site claim. The lane-pair forms (p29_dbl_pl,
p29_add_aff_pl) compute the same products on the same operands, in a different summation order
whose partial sums the per-column sum of |terms| bounds as well (checked here)."""
import random

import pytest

from oracle import pyref

P = pyref.P
R = 1 << 261
RINV = pow(R, -1, P)
MASK = (1 << 29) - 1
I64 = 1 << 63
I32 = 1 << 31


def i32(u):
    u &= 0xFFFFFFFF
    return u - (1 << 32) if u & 0x80000000 else u


def val(limbs):
    return sum(i32(w) << (29 * i) for i, w in enumerate(limbs))


def to_limbs(x):  # canonical limbs of 0 <= x < 2^261 (limb 8 holds the top 29 bits)
    return [(x >> (29 * i)) & MASK for i in range(8)] + [x >> 232]


def fits64(v):
    assert -I64 <= v < I64, "64-bit accumulator overflow"
    return v


def fits32(v):
    assert -I32 <= v < I32, "32-bit limb overflow"
    return v & 0xFFFFFFFF


# ---- the device primitives (p256_f29.hpp) -------------------------------------------------
RED = ((3, 1 << 9), (6, 1 << 18), (7, 0x1FE00000), (8, 0x00FFFFFF))  # (column offset, multiplier)


def mont(a, b, sq=False, addends=(), fold=False):
    """f29_mul / f29_sqr / f29_mulsq_add (chain form): Mont(a b) + sum c v, columns checked."""
    d = [fits32(2 * i32(x)) for x in a] if sq else None
    m = [0] * 9
    out = [0] * 9
    acc = 0
    for k in range(17):
        terms = []
        for i in range(9):
            j = k - i
            if sq:
                if i < j <= 8:
                    terms.append(i32(a[i]) * i32(d[j]))
                if j == i:
                    terms.append(i32(a[i]) * i32(a[i]))
            elif 0 <= j <= 8:
                terms.append(i32(a[i]) * i32(b[j]))
        for off, c in RED:
            if k >= off and k - off <= 8:
                terms.append(i32(m[k - off]) * c)
        if k >= 9:
            for v, c in addends:
                terms.append(i32(v[k - 9]) * c)
        # any summation order (chain, ILP columns first, pipelined) stays below this
        fits64(abs(acc) + sum(abs(t) for t in terms))
        acc = fits64(acc + sum(terms))
        if k < 9:
            m[k] = acc & MASK
        else:
            out[k - 9] = acc & MASK
        acc >>= 29
    for v, c in addends:
        acc += i32(v[8]) * c
    top = fits32(acc)
    if fold:
        h = i32(top) >> 24
        out[8] = (top - (h << 24)) & 0xFFFFFFFF
        out[7] = fits32(out[7] + (h << 21))
        out[6] = fits32(out[6] - (h << 18))
        out[3] = fits32(out[3] - (h << 9))
        out[0] = fits32(out[0] + h)
    else:
        out[8] = top
    return out


def mul_sub(a, b, c, d):  # f29_mul_sub: a b - c d, one reduction
    nd = [fits32(-i32(x)) for x in d]
    m = [0] * 9
    out = [0] * 9
    acc = 0
    for k in range(17):
        terms = []
        for i in range(9):
            j = k - i
            if 0 <= j <= 8:
                terms += [i32(a[i]) * i32(b[j]), i32(c[i]) * i32(nd[j])]
        for off, cc in RED:
            if k >= off and k - off <= 8:
                terms.append(i32(m[k - off]) * cc)
        fits64(abs(acc) + sum(abs(t) for t in terms))
        acc = fits64(acc + sum(terms))
        if k < 9:
            m[k] = acc & MASK
        else:
            out[k - 9] = acc & MASK
        acc >>= 29
    out[8] = fits32(acc)
    return out


def add(a, b):
    return [fits32(i32(x) + i32(y)) for x, y in zip(a, b)]


def sub(a, b):
    return [fits32(i32(x) - i32(y)) for x, y in zip(a, b)]


def normalize(a):  # f29_normalize
    c = [i32(a[i]) >> 29 for i in range(8)]
    t = [a[0] & MASK] + [fits32((a[i] & MASK) + c[i - 1]) for i in range(1, 8)] + [0]
    top = fits32(i32(a[8]) + c[7])
    h = i32(top) >> 24
    t[8] = top & 0x00FFFFFF
    t[7] = fits32(i32(t[7]) + (h << 21))
    t[6] = fits32(i32(t[6]) - (h << 18))
    t[3] = fits32(i32(t[3]) - (h << 9))
    t[0] = fits32(i32(t[0]) + h)
    return t


def triple(a):  # f29_triple (a product output)
    t = [fits32(3 * i32(x)) for x in a]
    c = [(t[i] & 0xFFFFFFFF) >> 29 for i in range(8)]
    return [t[0] & MASK] + [fits32((t[i] & MASK) + c[i - 1]) for i in range(1, 8)] + [fits32(i32(t[8]) + c[7])]


def mul_sqsub(a, b, c):  # f29_mul_sqsub: Mont(a b - c^2), c's terms negated in the same columns
    nc = [fits32(-i32(x)) for x in c]
    nc2 = [fits32(-2 * i32(x)) for x in c]
    m = [0] * 9
    out = [0] * 9
    acc = 0
    for k in range(17):
        terms = []
        for i in range(9):
            j = k - i
            if 0 <= j <= 8:
                terms.append(i32(a[i]) * i32(b[j]))
            if i < j <= 8:
                terms.append(i32(c[i]) * i32(nc2[j]))
            if j == i:
                terms.append(i32(c[i]) * i32(nc[i]))
        for off, cc in RED:
            if k >= off and k - off <= 8:
                terms.append(i32(m[k - off]) * cc)
        fits64(abs(acc) + sum(abs(t) for t in terms))
        acc = fits64(acc + sum(terms))
        if k < 9:
            m[k] = acc & MASK
        else:
            out[k - 9] = acc & MASK
        acc >>= 29
    out[8] = fits32(acc)
    return out


P29 = [0x1fffffff, 0x1fffffff, 0x1fffffff, 0x000001ff, 0, 0, 0x00040000, 0x1fe00000, 0x00ffffff]


def triple_half(a):  # f29_triple_half: 3 a / 2 mod p for a product output
    odd = a[0] & 1
    t = [(a[i] + (P29[i] if odd else 0)) * 3 for i in range(8)]
    assert all(0 <= x < 1 << 32 for x in t), "32-bit limb overflow"
    t.append(fits32(3 * (i32(a[8]) + (P29[8] if odd else 0))))
    c = [(t[i] & 0xFFFFFFFF) >> 29 for i in range(8)]
    w = [t[0] & MASK] + [fits32((t[i] & MASK) + c[i - 1]) for i in range(1, 8)] + [fits32(i32(t[8]) + c[7])]
    assert w[0] & 1 == 0
    return [fits32((w[i] >> 1) + ((w[i + 1] & 1) << 28)) for i in range(8)] + [fits32(i32(w[8]) >> 1)]


# ---- contracts ------------------------------------------------------------------------------
def check_N(a):  # product output
    assert all(0 <= a[i] <= MASK for i in range(8)) and abs(val(a)) < 1 << 258


def check_Np(a):  # f29_normalize / fold output
    assert all(-(1 << 26) < i32(a[i]) < (1 << 29) + (1 << 26) for i in range(8))
    assert 0 <= i32(a[8]) < 1 << 24 and abs(val(a)) < 1 << 257


def relimb(a, rng, lo, hi, top_lo=None, top_hi=None):
    """The same value with limbs 0..7 moved at random inside [lo, hi) (limb 8 absorbs)."""
    v = [i32(x) for x in a]
    for i in range(8):
        k = rng.choice((-2, -1, 0, 1, 2))
        nv = v[i] + k * (1 << 29)
        if lo <= nv < hi:
            v[i] = nv
            v[i + 1] -= k
    if top_lo is not None and not top_lo <= v[8] < top_hi:
        return a
    return [x & 0xFFFFFFFF for x in v]


def mont_of(x):
    return to_limbs(x * R % P)


def plain(a):
    return val(a) * RINV % P


# ---- the formulas (p256_f29.hpp p29_dbl_f, p29_add_aff_lean_f) ------------------------------
def dbl_f(X, Y, Z):
    y2 = add(Y, Y)
    d = mont(Z, Z, sq=True)
    g = mont(Y, Y, sq=True)
    t0 = add(g, g)
    b2 = mont(X, t0)
    t1 = sub(X, d)
    a1 = add(X, d)
    a1 = mont(t1, a1)
    al = triple(a1)
    Z3 = mont(y2, Z)
    X3 = mont(al, al, sq=True, addends=[(b2, -4)], fold=True)
    l = mont(g, g, sq=True)
    t0 = [fits32((i32(b) << 1) - i32(x)) for b, x in zip(b2, X3)]
    Y3 = mont(al, t0, addends=[(l, -8)], fold=True)
    for v in (d, g, b2, a1, Z3, l):
        check_N(v)
    check_Np(X3)
    check_Np(Y3)
    return X3, Y3, Z3


def dbl_h(X, Y, Z):  # p29_dbl_h: the representative scaled by 1/2
    d = mont(Z, Z, sq=True)
    g = mont(Y, Y, sq=True)
    b = mont(X, g)
    t1 = sub(X, d)
    a1 = add(X, d)
    a1 = mont(t1, a1)
    al = triple_half(a1)
    assert all(0 <= al[i] < (1 << 29) + 3 for i in range(8)) and abs(val(al)) < 2 ** 258.1
    Z3 = mont(Y, Z)
    X3 = mont(al, al, sq=True, addends=[(b, -2)], fold=True)
    t = sub(b, X3)
    Y3 = mul_sqsub(al, t, g)
    for v in (d, g, b, a1, Z3, Y3):
        check_N(v)
    check_Np(X3)
    return X3, Y3, Z3


def add_aff_f(X, Y, Z, x2, y2):
    z1z1 = mont(Z, Z, sq=True)
    u2 = mont(x2, z1z1)
    t = mont(Z, z1z1)
    h = sub(u2, X)
    s2 = mont(y2, t)
    hh = mont(h, h, sq=True)
    rr = sub(s2, Y)
    hhh = mont(hh, h)
    V = mont(X, hh)
    Z3 = mont(Z, h)
    X3 = mont(rr, rr, sq=True, addends=[(hhh, -1), (V, -2)], fold=True)
    t = sub(V, X3)
    Y3 = mul_sub(rr, t, Y, hhh)
    for v in (z1z1, u2, hh, hhh, V, Z3, Y3):
        check_N(v)
    check_Np(X3)
    return X3, Y3, Z3


def dbl_w(X, Y, Z, W):
    """p29_dbl_plw (the half kernel's lane-local doubling with W = c Z^2 carried along, on E_c:
    y^2 = x^3 - 3 c^2 x + b c^3; c = 1 is the curve itself), halved representative:
      a' = (X - W)(X + W) | g = Y^2;  b = X g | W3 = g W;  X3 = h^2 - 2b | L = g^2 (h = 3a'/2);
      Y3 = h (b - X3) - L | Z3 = Y Z.  Every product is a general one (one lane's is a square)."""
    a1 = mont(sub(X, W), add(X, W))
    g = mont(Y, Y)
    b = mont(X, g)
    W3 = mont(W, g)
    h = triple_half(a1)
    assert all(0 <= h[i] < (1 << 29) + 3 for i in range(8)) and abs(val(h)) < 2 ** 258.1
    X3 = mont(h, h, sq=True, addends=[(b, -2)], fold=True)
    L = mont(g, g, sq=True, addends=[(b, 0)], fold=True)  # the odd lane: the same call, c = 0
    t = sub(b, X3)
    Y3 = mont(h, t, addends=[(L, -1)], fold=True)
    Z3 = mont(Y, Z, addends=[(L, 0)])                      # odd lane: c = 0, no fold
    for v in (a1, g, b, W3, Z3):
        check_N(v)
    for v in (X3, L, Y3):
        check_Np(v)
    return X3, Y3, Z3, W3


def add_aff_w(X, Y, Z, W, x2, y2):
    """p29_add_aff_plw5: the mixed addition with W = c Z1^2 for the table entries (x/c, y/c):
      U2 = x2 W | T = Z1 W;  HH = H^2 | S2 = y2 T;  V = X1 HH | HHH;  Z3 = Z1 H | X3 = r^2 - HHH - 2V;
      W3 = W HH | Y3 = r (V - X3) - Y1 HHH (f29_mul_sub_ilp; the even lane's second product is Z1 0)."""
    u2 = mont(x2, W)
    T = mont(Z, W)
    h = sub(u2, X)
    hh = mont(h, h)
    s2 = mont(y2, T)
    V = mont(X, hh)
    hhh = mont(h, hh)
    rr = sub(s2, Y)
    Z3 = mont(Z, h, addends=[(hhh, 0), (V, 0)])
    X3 = mont(rr, rr, addends=[(hhh, -1), (V, -2)], fold=True)
    t = sub(V, X3)
    Y3 = mul_sub(rr, t, Y, hhh)
    W3 = mul_sub(W, hh, Z, [0] * 9)
    for v in (u2, T, hh, s2, V, hhh, Z3, Y3, W3):
        check_N(v)
    check_Np(X3)
    return X3, Y3, Z3, W3


def jac_to_affine(X, Y, Z):
    x, y, z = plain(X), plain(Y), plain(Z)
    zi = pow(z, -1, P)
    return x * zi * zi % P, y * zi * zi * zi % P


@pytest.mark.parametrize("dbl", ["f", "h"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_ladder_bounds_and_values(seed, dbl):
    """200 doublings and 50 mixed additions per seed, every operand re-limbed at the edges of
    its contract before use: no int64 column or int32 limb overflows, every output meets its
    stated contract, and the point matches the Python group law."""
    rng = random.Random(seed)
    G = pyref.G
    k = rng.randrange(1, pyref.N)
    pt = pyref.mul(k, G)
    X, Y, Z = mont_of(pt[0]), mont_of(pt[1]), mont_of(1)
    ref = pt
    for step in range(250):
        X = relimb(X, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
        Y = relimb(Y, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
        if step % 5 == 4:
            q = pyref.mul(rng.randrange(1, pyref.N), G)
            x2, y2 = mont_of(q[0]), mont_of(q[1])
            if rng.random() < 0.5:  # a negated table entry: N+- limbs
                y2 = [(-i32(w)) & 0xFFFFFFFF for w in y2]
                q = (q[0], (-q[1]) % P)
            X, Y, Z = add_aff_f(X, Y, Z, x2, y2)
            ref = pyref.add(ref, q)
            Y = relimb(Y, rng, -(1 << 29) + 1, 1 << 29)  # N+- (a difference of products)
        else:
            if dbl == "h":
                Y = relimb(Y, rng, -(1 << 29) + 1, 1 << 29)  # N+- (dbl_h's own Y3 is N)
            X, Y, Z = (dbl_h if dbl == "h" else dbl_f)(X, Y, Z)
            ref = pyref.add(ref, ref)
        assert jac_to_affine(X, Y, Z) == ref, step


def test_extreme_operands():
    """The doubling and the addition on operands whose every limb sits at the top of its
    contract (the worst case of each column), values then reduced: no overflow anywhere."""
    top = (1 << 29) + (1 << 26) - 1
    Np_max = [top] * 8 + [(1 << 24) - 1]
    N_max = [MASK] * 8 + [(1 << 24) - 1]
    X3, Y3, Z3 = dbl_f(Np_max, Np_max, N_max)
    add_aff_f(X3, Y3, Z3, N_max, [(-MASK) & 0xFFFFFFFF] * 8 + [0])
    X3, Y3, Z3 = dbl_h(Np_max, Np_max, N_max)
    dbl_h(X3, Y3, Z3)
    dbl_h(Np_max, [(-MASK) & 0xFFFFFFFF] * 8 + [(1 << 24) - 1], N_max)
    add_aff_f(X3, Y3, Z3, N_max, [(-MASK) & 0xFFFFFFFF] * 8 + [0])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_w_ladder_on_the_isomorphic_curve(seed):
    """The half kernel's v R0 side without the square root (p29_dbl_plw / p29_add_aff_plw): R0 =
    (r, y0) on the curve, c = r^3 - 3r + b = y0^2, and the ladder runs on E_c: y^2 = x^3 - 3c^2 x +
    b c^3 from P' = (c r, c^2), the image of R0 under (x, y) -> (c x, c y0 y), with W = c Z^2 and
    the table entries (x/c, y/c) = (x_E, y0 y_E). Checked: no overflow, every contract, W = c Z^2
    all along, and X / W = x(k R0) on the curve (the comparison the kernel makes) -- no y0 needed.
    c = 1 (the base on the curve itself, pair A) runs the same code."""
    rng = random.Random(seed)
    G = pyref.G
    for c_is_one in (False, True):
        R0 = pyref.mul(rng.randrange(1, pyref.N), G)
        r, y0 = R0
        c = 1 if c_is_one else (r ** 3 - 3 * r + pyref.B) % P
        yscale = 1 if c_is_one else y0
        if c_is_one:
            X, Y = mont_of(r), mont_of(y0)
        else:
            X, Y = mont_of(c * r % P), mont_of(c * c % P)
        Z, W = mont_of(1), mont_of(c)
        ref = R0
        for step in range(150):
            X = relimb(X, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
            W = relimb(W, rng, 0, 1 << 29)                                           # N
            if step % 5 == 4:
                q = pyref.mul(rng.randrange(1, pyref.N), R0)
                x2, y2 = mont_of(q[0]), mont_of(yscale * q[1] % P)
                if rng.random() < 0.5:  # a negated table entry: N+- limbs
                    y2 = [(-i32(w)) & 0xFFFFFFFF for w in y2]
                    q = (q[0], (-q[1]) % P)
                X, Y, Z, W = add_aff_w(X, Y, Z, W, x2, y2)
                ref = pyref.add(ref, q)
                Y = relimb(Y, rng, -(1 << 29) + 1, 1 << 29)  # N+-
            else:
                Y = relimb(Y, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
                X, Y, Z, W = dbl_w(X, Y, Z, W)
                ref = pyref.add(ref, ref)
            z = plain(Z)
            assert plain(W) == c * z * z % P, step
            assert plain(X) * pow(plain(W), -1, P) % P == ref[0], step


def _ec_add(A, p1, p2):
    """Affine addition on y^2 = x^3 + A x + B' (None = infinity); B' never enters the formulas."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2 and (y1 + y2) % P == 0:
        return None
    if p1 == p2:
        lam = (3 * x1 * x1 + A) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


@pytest.mark.parametrize("seed", [5, 6])
def test_w_ladder_on_the_twist_never_matches(seed):
    """Why the half kernel needs no square test (round 5): when c = r^3 - 3r + b is NOT a square,
    pair B's ladder runs on E_c, now the quadratic twist, from P' = (c r, c^2), and the x it ends
    with, X / W = x(V) / c, has f(x) = x^3 - 3x + b a non-square at every step -- the x of no point
    of the curve, so the final comparison with T (a curve point) fails, as Go's x(R) = r does when
    no point has x = r. Same kernel model (dbl_w / add_aff_w, limb contracts, W = c Z^2), with the
    reference ladder on E_c itself."""
    rng = random.Random(seed)
    done = 0
    while done < 2:
        r = rng.randrange(1, P)
        c = (r ** 3 - 3 * r + pyref.B) % P
        if pow(c, (P - 1) // 2, P) != P - 1:
            continue  # c a square: covered by test_w_ladder_on_the_isomorphic_curve
        done += 1
        A = (-3 * c * c) % P  # E_c: y^2 = x^3 - 3 c^2 x + b c^3
        base = (c * r % P, c * c % P)
        assert (base[1] ** 2 - base[0] ** 3 - A * base[0] - pyref.B * c ** 3) % P == 0
        X, Y = mont_of(base[0]), mont_of(base[1])
        Z, W = mont_of(1), mont_of(c)
        ref = base
        for step in range(80):
            X = relimb(X, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
            W = relimb(W, rng, 0, 1 << 29)                                           # N
            if step % 5 == 4:
                q = base
                for _ in range(rng.randrange(1, 8)):
                    q = _ec_add(A, q, base)
                x2, y2 = mont_of(q[0] * pow(c, -1, P) % P), mont_of(q[1] * pow(c, -1, P) % P)  # entry / c
                X, Y, Z, W = add_aff_w(X, Y, Z, W, x2, y2)
                ref = _ec_add(A, ref, q)
                Y = relimb(Y, rng, -(1 << 29) + 1, 1 << 29)  # N+-
            else:
                Y = relimb(Y, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
                X, Y, Z, W = dbl_w(X, Y, Z, W)
                ref = _ec_add(A, ref, ref)
            z = plain(Z)
            assert plain(W) == c * z * z % P, step
            xv = plain(X) * pow(plain(W), -1, P) % P
            assert xv == ref[0] * pow(c, -1, P) % P, step
            fx = (xv ** 3 - 3 * xv + pyref.B) % P
            assert pow(fx, (P - 1) // 2, P) == P - 1, step  # the x of no curve point


def test_w_extreme_operands():
    top = (1 << 29) + (1 << 26) - 1
    Np_max = [top] * 8 + [(1 << 24) - 1]
    N_max = [MASK] * 8 + [(1 << 24) - 1]
    X3, Y3, Z3, W3 = dbl_w(Np_max, Np_max, N_max, N_max)
    add_aff_w(X3, Y3, Z3, W3, N_max, [(-MASK) & 0xFFFFFFFF] * 8 + [0])
    dbl_w(Np_max, [(-MASK) & 0xFFFFFFFF] * 8 + [(1 << 24) - 1], N_max, N_max)
    add_aff_w(Np_max, [(-MASK) & 0xFFFFFFFF] * 8 + [0], N_max, N_max, N_max, N_max)


def dbl_q4(X, Y, Z, W):
    """q4_dbl (the wide half kernel's quad doubling, p256_f29.hpp): the products of dbl_w, three
    steps of four lanes:  a' | g | Z3;  h^2 | L = g^2 | b = X g | W3 = W g;
    Y3 = h (3b - h^2) - L | X3 = h^2 - 2b  (b - X3 = 3b - h^2, so Y3 needs no X3; its operand's
    limbs reach 3 2^29, the widest any product here takes)."""
    a1 = mont(sub(X, W), add(X, W))
    g = mont(Y, Y)
    Z3 = mont(Y, Z)
    h = triple_half(a1)
    h2 = mont(h, h)
    L = mont(g, g)
    b = mont(X, g)
    W3 = mont(W, g)
    t = [fits32(3 * i32(bb) - i32(hh)) for bb, hh in zip(b, h2)]
    Y3 = mont(h, t, addends=[(L, -1)], fold=True)
    X3 = mont(h, h, addends=[(b, -2)], fold=True)
    for v in (a1, g, Z3, h2, L, b, W3):
        check_N(v)
    for v in (X3, Y3):
        check_Np(v)
    return X3, Y3, Z3, W3


def add_aff_q4(X, Y, Z, W, x2, y2):
    """q4_dbl<true> + q4_add_rest: U2 = x2 W | T = Z1 W (on the doubling's spare lanes);
    HH = H^2 | Z3 = Z1 H | S2 = y2 T;  V = X1 HH | HHH | W3 = W HH | r^2;  X3 = r^2 - HHH - 2V
    (normalised limb arithmetic);  r (V - X3) | Y1 HHH, Y3 their difference (N+-)."""
    u2 = mont(x2, W)
    T = mont(Z, W)
    h = sub(u2, X)
    hh = mont(h, h)
    Z3 = mont(Z, h)
    s2 = mont(y2, T)
    rr = sub(s2, Y)
    V = mont(X, hh)
    hhh = mont(h, hh)
    W3 = mont(W, hh)
    r2 = mont(rr, rr)
    X3 = normalize(sub(sub(r2, hhh), add(V, V)))
    t = sub(V, X3)
    p0 = mont(rr, t)
    p1 = mont(Y, hhh)
    Y3 = sub(p0, p1)
    for v in (u2, T, hh, Z3, s2, V, hhh, W3, r2, p0, p1):
        check_N(v)
    check_Np(X3)
    assert all(abs(i32(y)) < 1 << 29 for y in Y3)  # N+-
    return X3, Y3, Z3, W3


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_quad_ladder_on_the_isomorphic_curve(seed):
    """The quad forms on the same walk as test_w_ladder_on_the_isomorphic_curve: pair B's E_c from
    P' = (c r, c^2) and pair A's curve (c = 1), operands re-limbed at the edges of their contracts
    (Y into the doubling as N' or N+-, into the addition as N': the kernel normalises Y before an
    addition that follows an addition). No overflow, every contract, W = c Z^2, X / W = x(k R0)."""
    rng = random.Random(seed)
    G = pyref.G
    for c_is_one in (False, True):
        R0 = pyref.mul(rng.randrange(1, pyref.N), G)
        r, y0 = R0
        c = 1 if c_is_one else (r ** 3 - 3 * r + pyref.B) % P
        yscale = 1 if c_is_one else y0
        X, Y = (mont_of(r), mont_of(y0)) if c_is_one else (mont_of(c * r % P), mont_of(c * c % P))
        Z, W = mont_of(1), mont_of(c)
        ref = R0
        for step in range(150):
            X = relimb(X, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
            W = relimb(W, rng, 0, 1 << 29)                                           # N
            if step % 5 == 4:
                q = pyref.mul(rng.randrange(1, pyref.N), R0)
                x2, y2 = mont_of(q[0]), mont_of(yscale * q[1] % P)
                if rng.random() < 0.5:
                    y2 = [(-i32(w)) & 0xFFFFFFFF for w in y2]
                    q = (q[0], (-q[1]) % P)
                Y = relimb(Y, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
                X, Y, Z, W = add_aff_q4(X, Y, Z, W, x2, y2)
                ref = pyref.add(ref, q)
                Y = relimb(Y, rng, -(1 << 29) + 1, 1 << 29)  # N+-
            else:
                if rng.random() < 0.5:
                    Y = relimb(Y, rng, -(1 << 29) + 1, 1 << 29)                          # N+-
                else:
                    Y = relimb(Y, rng, -(1 << 26) + 1, (1 << 29) + (1 << 26), 0, 1 << 24)   # N'
                X, Y, Z, W = dbl_q4(X, Y, Z, W)
                ref = pyref.add(ref, ref)
            z = plain(Z)
            assert plain(W) == c * z * z % P, step
            assert plain(X) * pow(plain(W), -1, P) % P == ref[0], step


def test_quad_extreme_operands():
    """Every limb at the top of its contract; and 3b - h^2's product at its analytic worst case
    (h limbs 2^29 + 2, the operand's 3 (2^29 - 1), the reduction's m limbs 2^29 - 1)."""
    top = (1 << 29) + (1 << 26) - 1
    Np_max = [top] * 8 + [(1 << 24) - 1]
    N_max = [MASK] * 8 + [(1 << 24) - 1]
    neg = [(-MASK) & 0xFFFFFFFF] * 8 + [(1 << 24) - 1]
    dbl_q4(Np_max, Np_max, N_max, N_max)
    dbl_q4(Np_max, neg, N_max, N_max)
    add_aff_q4(Np_max, Np_max, N_max, N_max, N_max, [(-MASK) & 0xFFFFFFFF] * 8 + [0])
    h = [(1 << 29) + 2] * 8 + [(1 << 26)]
    t = [3 * MASK] * 8 + [3 << 26]
    worst = 9 * ((1 << 29) + 2) * 3 * MASK + MASK * sum(c for _, c in RED)
    assert worst < I64
    mont(h, t, addends=[(N_max, -1)], fold=True)
