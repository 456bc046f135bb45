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
