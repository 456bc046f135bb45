"""CPU tests of header-only device algorithms compiled for the host with g++ (same source the
HIP kernels include): the safegcd inversion mod n and mod p (smartbft_amd/csrc/p256_inv.hpp) against
Python's pow(x, -1, m)."""
import os
import random
import subprocess

import pytest

from conftest import ROOT

N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
P = 2**256 - 2**224 + 2**192 + 2**96 - 1


@pytest.fixture(scope="module")
def inv_exe(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("native") / "inv_test")
    subprocess.run(["g++", "-O2", "-Wall", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "inv_test.cpp")], check=True)
    return exe


@pytest.mark.parametrize("mod", ["n", "p", "nR"])
def test_safegcd_inverse_matches_pow(inv_exe, mod):
    M = P if mod == "p" else N
    scale = (1 << 256) % N if mod == "nR" else 1
    rng = random.Random(1)
    xs = [1, 2, 3, M - 1, M - 2, M // 2, M // 3, 1 << 255, (1 << 256) % M, (1 << 128) - 1, 0xFFFFFFFF]
    xs += [1 << k for k in range(0, 256, 7)]
    xs += [(1 << 256) - 1 - (1 << k) for k in range(0, 255, 13) if (1 << 256) - 1 - (1 << k) < M]
    xs += [rng.randrange(1, M) for _ in range(20000)]
    # adversarial-ish: long runs of equal low bits (many divsteps with g even)
    xs += [((1 << 200) * rng.randrange(1, 1 << 55)) % M or 1 for _ in range(200)]
    out = subprocess.run([inv_exe, mod], input="".join("%064x\n" % x for x in xs), capture_output=True,
                         text=True, check=True).stdout.split()
    assert len(out) == len(xs)
    bad = [hex(x) for x, o in zip(xs, out) if int(o, 16) != scale * pow(x, -1, M) % M]
    assert not bad, bad[:4]


def test_host_mod_n_arithmetic(tmp_path):
    """modn_host.hpp (the pooled signer's online s = A e + B) against Python big integers."""
    exe = str(tmp_path / "modn_test")
    subprocess.run(["g++", "-O2", "-Wall", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "modn_test.cpp")], check=True)
    rng = random.Random(7)
    edge = [0, 1, 2, N - 1, N - 2, N // 2, 2**255, 2**256 - 1, 2**256 - N, N, N + 1, 2**128 - 1]
    pairs = [(a, b) for a in edge for b in edge]
    pairs += [(rng.randrange(2**256), rng.randrange(2**256)) for _ in range(20000)]
    out = subprocess.run([exe], input="".join("%064x %064x\n" % p for p in pairs), capture_output=True,
                         text=True, check=True).stdout.split("\n")
    assert len([l for l in out if l]) == len(pairs)
    for (a, b), line in zip(pairs, out):
        # inputs are reduced once on load (any 256-bit value is < 2n)
        ar, br = (a - N if a >= N else a), (b - N if b >= N else b)
        m, s = line.split()
        assert int(m, 16) == ar * br % N, (hex(a), hex(b))
        assert int(s, 16) == (ar + br) % N, (hex(a), hex(b))


def _euclid_half(u):
    """Exact restatement: Euclid on (n, u) stopped at the first remainder below 2^128 -> (w, v)
    with v u = w (mod n), plus the largest quotient met (the kernel gives up at >= 2^31)."""
    a, b, ta, tb, qmax = N, u, 0, 1, 0
    while b >= 1 << 128:
        q = a // b
        qmax = max(qmax, q)
        a, b, ta, tb = b, a - q * b, tb, ta - q * tb
    return b, tb, qmax


@pytest.mark.parametrize("rounds", [16, 0])
def test_half_gcd_matches_euclid(tmp_path, rounds):
    """p256_halfgcd.hpp (the half-size scalars of p256_verify_half_kernel) against exact Euclid:
    the same (w, v) whenever every quotient is below 2^31, a give-up otherwise, and always
    v u = w (mod n), 0 < w < 2^128, |v| < 2^128 on success."""
    exe = str(tmp_path / "hgcd_test")
    # rounds: SBFT_HGCD_K, Lehmer rounds of exactly that many candidate steps (0: the variable loop)
    subprocess.run(["g++", "-O2", "-Wall", "-Werror", f"-DSBFT_HGCD_K={rounds}", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "hgcd_test.cpp")], check=True)
    rng = random.Random(11)
    us = [1, 2, 3, N - 1, N - 2, N // 2, N // 3, (N + 1) // 2, (1 << 128) - 1, 1 << 128, (1 << 128) + 1,
          (1 << 255) % N, 0xFFFFFFFF, 1 << 200, N - (1 << 128)]
    us += [N // k for k in (5, 7, 1000, 1 << 20, (1 << 31) - 1, 1 << 31, (1 << 31) + 1, 1 << 40)]
    us += [rng.randrange(1, N) for _ in range(20000)]
    # Fibonacci-like (all quotients 1: the longest runs) and near-multiples (large quotients)
    f0, f1 = 1, 2
    while f1 < N:
        f0, f1 = f1, f0 + f1
    us += [f0 % N, (f0 * 3) % N]
    us += [(N * k) // (k * 1000 + 1) for k in range(1, 50)]
    us += [(rng.randrange(1, 1 << 100) << 150) % N or 1 for _ in range(200)]
    out = subprocess.run([exe], input="".join("%064x\n" % u for u in us), capture_output=True, text=True,
                         check=True).stdout.split("\n")
    nfail = 0
    for u, line in zip(us, out):
        w_x, v_x, qmax = _euclid_half(u)
        f = line.split()
        if f[0] == "0":
            assert qmax >= 1 << 31, (hex(u), "gave up although every quotient is small")
            nfail += 1
            continue
        assert qmax < 1 << 31, hex(u)
        w, v, neg = int(f[1], 16), int(f[2], 16), f[3] == "1"
        sv = -v if neg else v
        assert (w, sv) == (w_x, v_x), hex(u)
        assert (sv * u - w) % N == 0 and 0 < w < 1 << 128 and 0 < v < 1 << 128, hex(u)
    assert nfail < 60  # only the crafted large-quotient inputs


@pytest.mark.parametrize("count", [1, 2, 67, 96, 500])
def test_host_batch_sinv(tmp_path, count):
    """modn::sinv_batch_mont (sinv_host.hpp): the keyed path's host-side s^-1 for a batch, by
    Montgomery's trick and one safegcd, in the Montgomery form the keyed kernel takes
    (s^-1 2^256 mod n); s = 0 and s >= n stand in as 1."""
    exe = str(tmp_path / "sinv_test")
    subprocess.run(["g++", "-O2", "-Wall", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "sinv_test.cpp")], check=True)
    rng = random.Random(count)
    n = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    edge = [1, 2, n - 1, n, n + 1, 0, (1 << 256) - 1, 1 << 255, 0xFFFFFFFF]
    ss = (edge + [rng.randrange(1, n) for _ in range(count)])[:count] if count > len(edge) else \
        [rng.randrange(1, n) for _ in range(count)]
    out = subprocess.run([exe], input="".join("%064x\n" % x for x in ss), capture_output=True, text=True,
                         check=True).stdout.split()
    assert len(out) == count
    for x, got in zip(ss, out):
        v = x if 0 < x < n else 1
        assert int(got, 16) == pow(v, -1, n) * (1 << 256) % n, hex(x)
