"""GPU parity tests of the registered-key path (p256_keyed.hip): per-key comb tables, the
wavefront-per-signature verify and the safegcd scalar inversion — bit-exact against the
oracle (Go crypto/ecdsa.Verify restated) and the golden fixtures."""
import hashlib
import random

import numpy as np
import pytest

import oracle
from conftest import split_fields
from smartbft_amd import GpuVerifyError

pytestmark = pytest.mark.gpu

N = oracle.N
P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF


def _be(x: int) -> bytes:
    return x.to_bytes(32, "big")


def test_safegcd_inverse_mod_n(gpu):
    rng = random.Random(7)
    xs = [1, 2, 3, N - 1, N - 2, 1 << 255, (1 << 256) % N, 0xFFFFFFFF, 1 << 224, N // 2]
    xs += [rng.randrange(1, N) for _ in range(4000)]
    a = np.frombuffer(b"".join(_be(x) for x in xs), dtype=np.uint8).reshape(-1, 32)
    out = gpu.selftest_field(10, a, a)
    got = [int.from_bytes(bytes(r), "big") for r in out]
    bad = [hex(x) for x, g in zip(xs, got) if g != pow(x, -1, N)]
    assert not bad, bad[:4]


def test_register_key_validation(gpu):
    qx, qy = oracle.pubkey(12345)
    k1 = gpu.register_key(qx, qy)
    assert k1 >= 1
    assert gpu.register_key(qx, qy) == k1  # idempotent
    bad_y = (int.from_bytes(qy, "big") + 1) % P
    with pytest.raises(GpuVerifyError):
        gpu.register_key(qx, _be(bad_y))           # off curve
    with pytest.raises(GpuVerifyError):
        gpu.register_key(_be(P + 3), qy)                # non-canonical x >= p
    with pytest.raises(GpuVerifyError):
        gpu.register_key(bytes(32), bytes(32))      # (0, 0) is not on the curve
    qx2, qy2 = oracle.pubkey(999)
    k2 = gpu.register_key(qx2, qy2)
    assert k2 > k1
    # batch registration: known keys keep their id, invalid ones map to 0, new ones get ids
    qx3, qy3 = oracle.pubkey(4242)
    ids = gpu.register_keys([qx, _be(P + 3), qx3, qx3], [qy, qy, qy3, qy3])
    assert ids[0] == k1 and ids[1] == 0 and ids[2] > k2 and ids[3] == ids[2]


def _register_all(gpu, f):
    """Register every distinct key of the rows; rows whose key is invalid get id 0 (unknown)."""
    ids, cache = np.zeros(len(f), dtype=np.uint32), {}
    for i, row in enumerate(f):
        k = bytes(row[96:160])
        if k not in cache:
            try:
                cache[k] = gpu.register_key(k[:32], k[32:])
            except GpuVerifyError:
                cache[k] = 0
        ids[i] = cache[k]
    return ids


def test_golden_vectors_keyed(gpu, p256_vectors):
    f, exp, cat, names = p256_vectors
    # every category, the big random ones subsampled (one comb table per distinct key)
    rng = np.random.default_rng(3)
    keep = []
    for c in np.unique(cat):
        idx = np.nonzero(cat == c)[0]
        keep.extend(idx if len(idx) <= 160 else rng.choice(idx, 60, replace=False))
    keep = np.sort(np.array(keep))
    g = f[keep]
    ids = _register_all(gpu, g)
    d, r, s, _, _ = split_fields(g)
    got = gpu.verify_keyed(d, r, s, ids)
    bad = np.nonzero(got != exp[keep])[0]
    assert len(bad) == 0, {names[c]: int((cat[keep][bad] == c).sum()) for c in np.unique(cat[keep][bad])}
    # invalid keys never verify
    assert not got[ids == 0].any()


@pytest.mark.parametrize("path", ["wave", "lanes"])
def test_golden_vectors_keyed_paths(p256_vectors, path, monkeypatch):
    """Every golden category (R = infinity and Shamir-exceptional included) through each keyed
    kernel on its own: the wavefront per signature (zero-copy latency path) and the four-lane
    kernel with the batched s^-1 (large batches), whichever the batch size would pick."""
    from smartbft_amd import GpuVerifier
    if path == "wave":
        monkeypatch.setenv("SBFT_KEYED_ZC_MAX", "100000")
        monkeypatch.setenv("SBFT_KEYED_LANES_MIN", "0")
    else:
        monkeypatch.setenv("SBFT_KEYED_ZC_MAX", "0")
        monkeypatch.setenv("SBFT_KEYED_LANES_MIN", "1")
    g = GpuVerifier(device_mask=1)
    f, exp, cat, names = p256_vectors
    rng = np.random.default_rng(11)
    keep = []
    for c in np.unique(cat):
        idx = np.nonzero(cat == c)[0]
        keep.extend(idx if len(idx) <= 160 else rng.choice(idx, 40, replace=False))
    keep = np.sort(np.array(keep))
    rows = f[keep]
    ids = _register_all(g, rows)
    d, r, s, _, _ = split_fields(rows)
    for n in (len(keep), 1, 2, 1025):  # whole set, tiny and just past the zero-copy bound
        sel = np.arange(min(n, len(keep)))
        got = g.verify_keyed(d[sel], r[sel], s[sel], ids[sel])
        bad = np.nonzero(got != exp[keep][sel])[0]
        assert len(bad) == 0, (n, {names[c]: int((cat[keep][sel][bad] == c).sum()) for c in np.unique(cat[keep][sel][bad])})
    g.close()


@pytest.mark.parametrize("host_sinv_max", ["96", "0"])
def test_golden_vectors_keyed_host_sinv(p256_vectors, host_sinv_max, monkeypatch):
    """The zero-copy wavefront path with s^-1 from the host (batches of at most keyed_host_sinv_max
    = 96 signatures, modn::sinv_batch_mont; s = 0 and s >= n are swapped for 1 there and rejected
    by the kernel's `valid` flag) and with it off (SBFT_KEYED_HOST_SINV_MAX=0: the kernel inverts),
    every golden category -- out-of-range s included -- in batches of 96 and of odd sizes."""
    from smartbft_amd import GpuVerifier
    monkeypatch.setenv("SBFT_KEYED_ZC_MAX", "100000")
    monkeypatch.setenv("SBFT_KEYED_LANES_MIN", "0")
    monkeypatch.setenv("SBFT_KEYED_HOST_SINV_MAX", host_sinv_max)
    g = GpuVerifier(device_mask=1)
    f, exp, cat, names = p256_vectors
    rng = np.random.default_rng(12)
    keep = []
    for c in np.unique(cat):
        idx = np.nonzero(cat == c)[0]
        keep.extend(idx if len(idx) <= 96 else rng.choice(idx, 24, replace=False))
    keep = np.sort(np.array(keep))
    rows = f[keep]
    ids = _register_all(g, rows)
    d, r, s, _, _ = split_fields(rows)
    want = exp[keep]
    for size in (96, 67, 1):
        for lo in range(0, len(keep), size):
            sel = np.arange(lo, min(lo + size, len(keep)))
            got = g.verify_keyed(d[sel], r[sel], s[sel], ids[sel])
            bad = np.nonzero(got != want[sel])[0]
            assert len(bad) == 0, (host_sinv_max, size, lo,
                                   {names[c]: int((cat[keep][sel][bad] == c).sum()) for c in np.unique(cat[keep][sel][bad])})
            if size == 1 and lo > 40:
                break
    g.close()


def _signed(n, nkeys, seed, corrupt=0.3):
    rng = random.Random(seed)
    keys = [rng.randrange(1, N) for _ in range(nkeys)]
    pubs = [oracle.pubkey(d) for d in keys]
    rows, msgs, which = [], [], []
    for i in range(n):
        j = rng.randrange(nkeys)
        m = rng.randbytes(rng.randrange(0, 300))
        e = hashlib.sha256(m).digest()
        r, s = oracle.sign(keys[j], rng.randrange(1, N), e)
        r, s = bytearray(r), bytearray(s)
        if rng.random() < corrupt:
            kind = rng.randrange(5)
            if kind == 0:
                r[rng.randrange(32)] ^= 1 << rng.randrange(8)
            elif kind == 1:
                s[rng.randrange(32)] ^= 1 << rng.randrange(8)
            elif kind == 2:
                m = m + b"x"
            elif kind == 3:
                s = bytearray(_be(N))
            else:
                r = bytearray(bytes(32))
        rows.append(hashlib.sha256(m).digest() + bytes(r) + bytes(s) + pubs[j][0] + pubs[j][1])
        msgs.append(m)
        which.append(j)
    f = np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(n, 160)
    return f, msgs, which, pubs


@pytest.mark.parametrize("n", [1, 2, 67, 333])
def test_random_keyed_matches_oracle(gpu, n):
    f, msgs, which, pubs = _signed(n, 12, seed=n)
    kid = [gpu.register_key(*p) for p in pubs]
    ids = np.array([kid[j] for j in which], dtype=np.uint32)
    exp = oracle.verify_batch(*split_fields(f))
    d, r, s, _, _ = split_fields(f)
    assert np.array_equal(gpu.verify_keyed(d, r, s, ids), exp)
    # fused: the messages are hashed inside the keyed launch
    ln = np.array([len(m) for m in msgs], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8)
    assert np.array_equal(gpu.sha256_verify_keyed(blob, off, ln, r, s, ids), exp)
    if n > 1:
        assert 0 < exp.sum() < n


def test_wrong_or_unknown_key_id_rejects(gpu):
    f, msgs, which, pubs = _signed(40, 3, seed=5, corrupt=0.0)
    kid = [gpu.register_key(*p) for p in pubs]
    d, r, s, _, _ = split_fields(f)
    right = np.array([kid[j] for j in which], dtype=np.uint32)
    assert gpu.verify_keyed(d, r, s, right).all()
    wrong = np.array([kid[(j + 1) % 3] for j in which], dtype=np.uint32)
    assert not gpu.verify_keyed(d, r, s, wrong).any()
    for bogus in (0, 1 << 30):
        assert not gpu.verify_keyed(d, r, s, np.full(40, bogus, dtype=np.uint32)).any()
