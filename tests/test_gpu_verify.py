"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the golden
fixtures, bit-exact. Marked gpu; they fail — never skip — when the HIP library or the GPU
is missing."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, split_fields

pytestmark = pytest.mark.gpu


def _rand_tuples(n, seed, corrupt_frac=0.25):
    """Oracle-signed tuples with a seeded mix of corruptions (test-side generator)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 160), dtype=np.uint8)
    for i in range(n):
        d = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        k = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        e = hashlib.sha256(rng.bytes(64)).digest()
        qx, qy = oracle.pubkey(d)
        r, s = oracle.sign(d, k, e)
        rec = bytearray(e + r + s + qx + qy)
        if rng.random() < corrupt_frac:
            kind = int(rng.integers(0, 7))
            if kind == 0:
                rec[32 + int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 1:
                rec[64 + int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 2:
                rec[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 3:
                rec[32:64] = bytes(32)
            elif kind == 4:
                rec[64:96] = oracle.N.to_bytes(32, "big")
            elif kind == 5:
                rec[159] ^= 1  # Qy + 1 -> off curve
            else:
                rec[32:64] = (oracle.N + int(rng.integers(0, 1000))).to_bytes(32, "big")
        out[i] = np.frombuffer(bytes(rec), dtype=np.uint8)
    return out


def test_golden_vectors_host_api(gpu, p256_vectors):
    f, exp, cat, names = p256_vectors
    got = gpu.verify(*split_fields(f))
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, {names[c]: int((cat[bad] == c).sum()) for c in np.unique(cat[bad])}


def test_golden_vectors_device_api(gpu, p256_vectors):
    import torch
    f, exp, cat, names = p256_vectors
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in split_fields(f)]
    ok = torch.zeros(len(exp), dtype=torch.uint8, device=dev)
    gpu.verify_dev(*t, ok)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), exp)


def test_random_batch_matches_oracle(gpu):
    f = _rand_tuples(3000, seed=11)
    exp = oracle.verify_batch(*split_fields(f))
    got = gpu.verify(*split_fields(f))
    assert np.array_equal(got, exp)
    assert 0 < exp.sum() < len(exp)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 255, 256, 257, 1000])
def test_ragged_batch_sizes(gpu, p256_vectors, n):
    f, exp, cat, names = p256_vectors
    idx = np.arange(n) * 7 % len(exp)
    got = gpu.verify(*split_fields(f[idx]))
    assert np.array_equal(got, exp[idx])


def test_empty_batch(gpu):
    z = np.zeros((0, 32), dtype=np.uint8)
    assert gpu.verify(z, z, z, z, z).shape == (0,)


def test_large_tiled_batch_against_fixtures(gpu, p256_vectors):
    """Size-independent property at scale: 128 tiled copies of the fixture set must give the
    fixture verdict in every copy (exercises many blocks and the multi-chunk split)."""
    f, exp, cat, names = p256_vectors
    reps = 128
    big = np.tile(f, (reps, 1))
    got = gpu.verify(*split_fields(big))
    assert np.array_equal(got.reshape(reps, -1), np.tile(exp, (reps, 1)))


def _sha_msg(length, tag, seed=b"SBFT-GPUV-FIXTURES-1"):
    out = bytearray()
    ctr = 0
    while len(out) < length:
        out += hashlib.sha256(seed + b"shamsg" + str(tag).encode() + ctr.to_bytes(8, "little")).digest()
        ctr += 1
    return bytes(out[:length])


def test_sha256_kats(gpu):
    d = json.load(open(os.path.join(GOLDEN, "sha256_vectors.json")))
    msgs = [bytes.fromhex(v["msg_hex"]) for v in d["fips180_4"]] + \
           [_sha_msg(v["len"], v["tag"]) for v in d["seeded"]]
    want = [v["sha256"] for v in d["fips180_4"]] + [v["sha256"] for v in d["seeded"]]
    lens = np.array([len(m) for m in msgs], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    got = gpu.sha256(blob, off, lens)
    assert [g.tobytes().hex() for g in got] == want


def test_sha256_random_lengths_and_alignment(gpu):
    rng = np.random.default_rng(3)
    n = 2000
    lens = rng.integers(0, 3000, size=n).astype(np.uint32)
    gaps = rng.integers(0, 5, size=n)  # odd gaps -> unaligned starts
    off = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += int(lens[i])
    blob = rng.integers(0, 256, size=pos, dtype=np.uint8)
    got = gpu.sha256(blob, off, lens)
    exp = oracle.sha256_batch(blob, off, lens)
    assert np.array_equal(got, exp)


def test_sha256_dev_explicit_order(gpu):
    """Device entry with a caller permutation (lane t hashes message order[t]): digests still
    land at their own message's index, for an arbitrary (not length-sorted) permutation too."""
    import torch
    rng = np.random.default_rng(4)
    n = 1500
    lens = rng.integers(0, 5000, size=n).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
    blob = rng.integers(0, 256, size=int(lens.sum()) + 256, dtype=np.uint8)  # SBFT_GV_SHA_BLOB_PAD
    exp = oracle.sha256_batch(blob, off, lens)
    dev = torch.device("cuda:0")
    d_blob = torch.from_numpy(blob).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    for order in (np.argsort(-lens.astype(np.int64), kind="stable"), rng.permutation(n)):
        d_dig = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
        d_ord = torch.from_numpy(order.astype(np.int32)).to(dev)
        gpu.sha256_dev(d_blob, d_off, d_len, d_dig, d_order=d_ord)
        torch.cuda.synchronize()
        assert np.array_equal(d_dig.cpu().numpy(), exp)


@pytest.mark.parametrize("n", [65_535, 65_536, 100_003, 70_001])
def test_sha256_longest_first_batches(gpu, n):
    """Batches of >= 65,536 messages (no caller order) are hashed longest first: a device-side
    counting sort of the lengths into 128 classes picks the order (sha256.hip). Digests land at
    their own index on the device entry and the host entry, for lengths spanning empty, one-
    block, padding-edge and multi-KiB messages at unaligned offsets, on both sides of the cut-in."""
    import torch
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 1500, size=n).astype(np.uint32)
    lens[:: 97] = rng.integers(4000, 9000, size=len(lens[:: 97]))  # a spread of long messages
    lens[1::1009] = 0
    lens[2::1013] = 55
    lens[3::1019] = 64
    if n == 70_001:  # messages past 64 KiB take the eighth-octave classes; one length for many
        lens[5::2003] = rng.integers(65_000, 600_000, size=len(lens[5::2003]))
        lens[6::7] = 777
    gaps = rng.integers(0, 4, size=n).astype(np.uint64)
    off = (np.cumsum(lens.astype(np.uint64) + gaps) - lens).astype(np.uint64)
    total = int(off[-1] + lens[-1])
    blob = rng.integers(0, 256, size=total + 256, dtype=np.uint8)  # SBFT_GV_SHA_BLOB_PAD
    exp = oracle.sha256_batch(blob, off, lens)
    got = gpu.sha256(blob[:total], off, lens)
    assert np.array_equal(got, exp)
    dev = torch.device("cuda:0")
    d_dig = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    gpu.sha256_dev(torch.from_numpy(blob).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                   torch.from_numpy(lens.astype(np.int32)).to(dev), d_dig)
    torch.cuda.synchronize()
    assert np.array_equal(d_dig.cpu().numpy(), exp)


def test_fused_hash_then_verify(gpu):
    rng = np.random.default_rng(9)
    n = 600
    msgs, recs = [], []
    for i in range(n):
        m = rng.bytes(int(rng.integers(0, 400)))
        d = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        k = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        e = hashlib.sha256(m).digest()
        qx, qy = oracle.pubkey(d)
        r, s = oracle.sign(d, k, e)
        if i % 5 == 0:
            m = m + b"x"  # payload tampered after signing
        msgs.append(m)
        recs.append((r, s, qx, qy))
    lens = np.array([len(m) for m in msgs], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    blob = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8)
    cols = [np.frombuffer(b"".join(x[j] for x in recs), dtype=np.uint8).reshape(n, 32) for j in range(4)]
    ok, dig = gpu.sha256_verify(blob, off, lens, *cols, want_digests=True)
    for i in range(n):
        assert dig[i].tobytes() == hashlib.sha256(msgs[i]).digest()
    exp = oracle.verify_batch(dig, *cols)
    assert np.array_equal(ok, exp)
    assert exp.sum() == n - len(range(0, n, 5))


def test_signer_matches_oracle(gpu):
    """GPU key derivation + signing with fixed nonces == the oracle's, byte for byte."""
    rng = np.random.default_rng(21)
    n = 700
    d = [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(n)]
    k = [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(n)]
    d[0], k[0] = 1, 1
    d[1], k[1] = oracle.N - 1, oracle.N - 1
    e = [rng.bytes(32) for _ in range(n)]
    e[2] = b"\xff" * 32
    arr = lambda xs: np.frombuffer(b"".join(x if isinstance(x, bytes) else x.to_bytes(32, "big")
                                            for x in xs), dtype=np.uint8).reshape(-1, 32)
    qx, qy, r, s, st = gpu.sign(arr(d), arr(k), arr(e))
    assert st.all()
    for i in range(n):
        ox, oy = oracle.pubkey(d[i])
        orr, oss = oracle.sign(d[i], k[i], e[i])
        assert (qx[i].tobytes(), qy[i].tobytes()) == (ox, oy), i
        assert (r[i].tobytes(), s[i].tobytes()) == (orr, oss), i
    # out-of-range private keys / nonces are flagged, not signed
    bad = arr([0, oracle.N, oracle.N + 5])
    *_, st2 = gpu.sign(bad, arr([1, 1, 1]), arr([b"\0" * 32] * 3))
    assert not st2.any()
    # batches above the latency-path size (4,096) take the one-lane-per-signature kernel: same
    # outputs, byte for byte, on the same inputs
    m = 5000
    d2 = d + [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(m - n)]
    k2 = k + [int.from_bytes(rng.bytes(32), "big") % oracle.N or 1 for _ in range(m - n)]
    e2 = e + [rng.bytes(32) for _ in range(m - n)]
    big = gpu.sign(arr(d2), arr(k2), arr(e2))
    for got, want in zip(big, (qx, qy, r, s, st)):
        assert np.array_equal(got[:n], want)
    assert big[4].all()
    for i in rng.choice(np.arange(n, m), 100, replace=False):
        assert (big[2][i].tobytes(), big[3][i].tobytes()) == oracle.sign(d2[i], k2[i], e2[i]), i


def test_bench_workload_properties(gpu):
    """The synthetic bench workload: every uncorrupted tuple verifies, every corrupted one
    does not (by construction), and a sample agrees with the oracle."""
    import torch
    from smartbft_amd.workload import make_workload
    wl = make_workload(gpu, 20000, start=12345)
    ok = torch.empty(wl.n, dtype=torch.uint8, device="cuda:0")
    gpu.verify_dev(wl.digest, wl.r, wl.s, wl.qx, wl.qy, ok)
    torch.cuda.synchronize()
    assert torch.equal(ok, (~wl.corrupted).to(torch.uint8))
    frac = float(wl.corrupted.float().mean())
    assert 0.07 < frac < 0.13
    f = wl.host_fields(0, 3000)
    assert np.array_equal(oracle.verify_batch(*f), ok[:3000].cpu().numpy())


@pytest.mark.parametrize("n", [262_145, 786_432, 900_000, 1_000_000])
def test_throughput_grid_shapes(gpu, n):
    """The throughput launch at sizes past one resident round: a partial last round launched
    as is (262,145; 900,000: last round < 80% full), exactly whole rounds (786,432), and a
    mostly full last round, which the launch turns into whole rounds with the tuples spread
    evenly over the workgroups (1,000,000: 3,907 -> 4,096 workgroups of ~244 tuples). Verdicts
    = the workload's construction on every tuple, an oracle sample at workgroup edges."""
    import torch
    from smartbft_amd.workload import make_workload
    wl = make_workload(gpu, n, start=9000 + n % 1000)
    ok = torch.empty(wl.n, dtype=torch.uint8, device="cuda:0")
    gpu.verify_dev(wl.digest, wl.r, wl.s, wl.qx, wl.qy, ok)
    torch.cuda.synchronize()
    assert torch.equal(ok, (~wl.corrupted).to(torch.uint8))
    g = 4096 if n == 1_000_000 else 0  # the spread grid's workgroup edges: b n / 4096
    edges = sorted({e for b in (1, 2, 1000, 4095) for e in ((b * n // g) - 1, b * n // g)} if g else {255, 256, n - 1})
    edges = [e for e in edges if 0 <= e < n]
    f = [x[edges] for x in wl.host_fields()]
    assert np.array_equal(oracle.verify_batch(*f), ok.cpu().numpy()[edges])


# ---- every verify kernel at every size: the one-lane throughput kernel and the small-batch
# latency kernel with two and four lanes per tuple (p256_verify_small_kernel<2|4>, forced on
# for big batches too) and the half-size-scalar kernel (p256_verify_half_kernel)
KERNEL_OPTS = {"lane": dict(pair_max=-1, half_max=-1),
               "pair": dict(pair_max=1 << 30, half_max=-1),
               "half": dict(half_max=1 << 30, halfq_max=-1),
               "halfw": dict(halfq_max=1 << 30)}


@pytest.fixture(scope="module", params=list(KERNEL_OPTS))
def gpu_kernel(request):
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    v = GpuVerifier(**KERNEL_OPTS[request.param])
    yield v
    v.close()


def test_kernels_golden_vectors(gpu_kernel, p256_vectors):
    f, exp, cat, names = p256_vectors
    got = gpu_kernel.verify(*split_fields(f))
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, {names[c]: int((cat[bad] == c).sum()) for c in np.unique(cat[bad])}


# 1023/1024/1025/2049: the edges of the one-lane kernel's 1,024-tuple s^-1 groups
# (p256_verify.hip sinv_prep/sinv_totals)
@pytest.mark.parametrize("n", [1, 2, 31, 32, 33, 255, 256, 257, 1023, 1024, 1025, 2049, 4097])
def test_kernels_ragged_sizes(gpu_kernel, p256_vectors, n):
    f, exp, cat, names = p256_vectors
    idx = np.arange(n) * 5 % len(exp)
    assert np.array_equal(gpu_kernel.verify(*split_fields(f[idx])), exp[idx])


@pytest.fixture(scope="module")
def valid_2100():
    return _rand_tuples(2100, seed=77, corrupt_frac=0.0)


@pytest.mark.parametrize("n", [1024, 1025, 2048, 2049, 2100])
def test_kernels_invalid_s_at_group_edges(gpu_kernel, valid_2100, n):
    """s = 0 and s >= n contribute 1 to the launch-wide batched s^-1 products; placed on both
    sides of every 1,024-tuple group boundary they must neither be accepted nor poison their
    neighbours' inverses (the whole group would then mis-verify)."""
    f = valid_2100[:n].copy()
    N = oracle.N.to_bytes(32, "big")
    specials = {0: bytes(32), 1023: bytes(32), 1024: N, 1022: (oracle.N + 1).to_bytes(32, "big"),
                2047: b"\xff" * 32, 2048: bytes(32), n - 1: N}
    for i, val in specials.items():
        if i < n:
            f[i, 64:96] = np.frombuffer(val, dtype=np.uint8)
    exp = oracle.verify_batch(*split_fields(f))
    assert exp.sum() == n - len([i for i in specials if i < n])
    assert np.array_equal(gpu_kernel.verify(*split_fields(f)), exp)


def test_kernels_random_batch(gpu_kernel):
    f = _rand_tuples(2000, seed=23, corrupt_frac=0.3)
    exp = oracle.verify_batch(*split_fields(f))
    assert np.array_equal(gpu_kernel.verify(*split_fields(f)), exp)


def test_kernels_large_tiled(gpu_kernel, p256_vectors):
    """Many waves per SIMD for both kernels: 64 tiled copies of the fixtures (209k tuples)."""
    f, exp, cat, names = p256_vectors
    reps = 64
    got = gpu_kernel.verify(*split_fields(np.tile(f, (reps, 1))))
    assert np.array_equal(got.reshape(reps, -1), np.tile(exp, (reps, 1)))


@pytest.mark.parametrize("mode", list(KERNEL_OPTS))
def test_framed_hash_then_verify(mode):
    """sbft_gv_sha256_verify_p256_framed: tuples gathered on the device from the blob in the
    signed-request layout (x || y closing the signed body, r || s right after it), both
    kernels; a frame reaching past the blob is rejected, not read."""
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    gv = GpuVerifier(**KERNEL_OPTS[mode])
    rng = np.random.default_rng(31)
    n = 500
    parts, off, lens, exp = [], [], [], []
    pos = 3  # unaligned start
    for i in range(n):
        d = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        k = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        qx, qy = oracle.pubkey(d)
        body = rng.bytes(int(rng.integers(0, 300))) + qx + qy  # the key closes the signed body
        r, s = oracle.sign(d, k, hashlib.sha256(body).digest())
        sig = r + s
        if i % 7 == 3:
            sig = bytes([sig[0] ^ 1]) + sig[1:]
        if i % 11 == 5:
            body = body[:-1] + bytes([body[-1] ^ 0x80])  # key damaged after signing
        cols = (hashlib.sha256(body).digest(), sig[:32], sig[32:], body[-64:-32], body[-32:])
        exp.append(oracle.verify_batch(*[np.frombuffer(x, dtype=np.uint8).reshape(1, 32) for x in cols])[0])
        off.append(pos)
        lens.append(len(body))
        parts.append(body + sig)
        pos += len(body) + 64
    exp = np.array(exp, dtype=np.uint8)
    blob = np.frombuffer(b"\0\0\0" + b"".join(parts), dtype=np.uint8)
    got = gv.sha256_verify_framed(blob, np.array(off), np.array(lens), 0, -64)
    assert np.array_equal(got, exp)
    assert 0 < exp.sum() < n
    with pytest.raises(Exception):
        gv.sha256_verify_framed(blob, np.array(off), np.array(lens), 1, -64)
    gv.close()


@pytest.mark.parametrize("mode", list(KERNEL_OPTS))
def test_framed_exceptional_tuples(mode):
    """Framed tuples whose Shamir sum meets an exceptional addition, through the fused
    hash-and-verify launch (pair, half) and the three-kernel chain (lane): the verify kernel
    writes the flagged tuples' fields out for the fix-up kernel. With u1 = e/s, u2 = r/s:
    Q = -(e/r) G makes R = u1 G + u2 Q infinity (reject); Q = (e/r) G with s = 2e/k and
    r = x(kG) makes u2 Q = u1 G, a doubling, and the signature valid. Verdicts equal the oracle's."""
    import torch
    from smartbft_amd import GpuVerifier
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    gv = GpuVerifier(**KERNEL_OPTS[mode])
    rng = np.random.default_rng(77)
    n, N = 160, oracle.N
    parts, off, lens, exp = [], [], [], []
    pos = 1
    for i in range(n):
        msg = rng.bytes(int(rng.integers(0, 200)))
        e = int.from_bytes(hashlib.sha256(msg).digest(), "big") % N
        k = int.from_bytes(rng.bytes(32), "big") % N or 1
        if i % 4 == 0:  # R = infinity
            r = int.from_bytes(rng.bytes(32), "big") % N or 1
            s = int.from_bytes(rng.bytes(32), "big") % N or 1
            q = oracle.pubkey((-e * pow(r, -1, N)) % N or 1)
        elif i % 4 == 1:  # u2 Q = u1 G: the doubling case, a valid signature
            r = int.from_bytes(oracle.pubkey(k)[0], "big") % N
            s = (2 * e * pow(k, -1, N)) % N or 1
            q = oracle.pubkey((e * pow(r, -1, N)) % N or 1)
        else:  # ordinary signatures
            d = int.from_bytes(rng.bytes(32), "big") % N or 1
            q = oracle.pubkey(d)
            rb, sb = oracle.sign(d, k, hashlib.sha256(msg).digest())
            r, s = int.from_bytes(rb, "big"), int.from_bytes(sb, "big")
        sig = r.to_bytes(32, "big") + s.to_bytes(32, "big")
        cols = (hashlib.sha256(msg).digest(), sig[:32], sig[32:], q[0], q[1])
        exp.append(oracle.verify_batch(*[np.frombuffer(x, dtype=np.uint8).reshape(1, 32) for x in cols])[0])
        off.append(pos)
        lens.append(len(msg))
        parts.append(msg + sig + q[0] + q[1])  # the key follows the signature: Q depends on e
        pos += len(msg) + 128
    exp = np.array(exp, dtype=np.uint8)
    blob = np.frombuffer(b"\0" + b"".join(parts), dtype=np.uint8)
    got = gv.sha256_verify_framed(blob, np.array(off), np.array(lens), 0, 64)
    assert np.array_equal(got, exp)
    assert exp[1::4].all() and not exp[0::4].any()
    gv.close()


def test_pinned_inputs_pipelined_host_verify(gpu):
    """sbft_gv_verify_p256 with all five inputs in sbft_gv_host_alloc memory takes the
    copy/compute pipeline (a 65,536 then 262,144-tuple sub-batches on a copy stream + events,
    verified on two alternating compute streams: gpuverify.cpp enqueue_verify_piped): verdicts
    byte-identical to the pageable call (the same pipeline over page-locked staging) and to the
    workload's construction, including the ragged last sub-batch."""
    import torch
    from smartbft_amd import PinnedArray
    from smartbft_amd.workload import make_workload
    n = 2 * 262144 + 4321
    wl = make_workload(gpu, n, start=777)
    fields = wl.host_fields(0, n)
    pins = [PinnedArray((n, 32)) for _ in range(5)]
    try:
        for p, a in zip(pins, fields):
            p.array[:] = a
        got = gpu.verify(*[p.array for p in pins])
        ref = gpu.verify(*fields)
        assert np.array_equal(got, ref)
        assert np.array_equal(got, (~wl.corrupted).to(torch.uint8).cpu().numpy())
        again = gpu.verify(*[p.array for p in pins])  # reuses the copy stream and events
        assert np.array_equal(again, got)
    finally:
        for p in pins:
            p.close()


def test_pinned_single_allocation_and_mixed_inputs(gpu):
    """INTEGRATION.md's layout: the five arrays at offsets inside ONE sbft_gv_host_alloc
    block (interior pointers must be recognised as pinned), and a call where one input is
    pageable (the pipeline then stages every sub-batch through page-locked memory). Both
    byte-identical to the workload verdicts."""
    import torch
    from smartbft_amd import PinnedArray
    from smartbft_amd.workload import make_workload
    n = 2 * 262144 + 99
    wl = make_workload(gpu, n, start=4242)
    fields = wl.host_fields(0, n)
    want = (~wl.corrupted).to(torch.uint8).cpu().numpy()
    block = PinnedArray((5, n, 32))
    try:
        for k, a in enumerate(fields):
            block.array[k] = a
        views = [block.array[k] for k in range(5)]
        assert np.array_equal(gpu.verify(*views), want)
        mixed = views[:4] + [np.array(fields[4])]
        assert np.array_equal(gpu.verify(*mixed), want)
    finally:
        block.close()


@pytest.mark.parametrize("n", [5000, 70_000])
def test_all_exceptional_batches(gpu_kernel, p256_vectors, n):
    """A batch made only of tuples whose lean Shamir ladder hits an exceptional addition
    (crafted R = infinity, P + P, P + (-P): golden categories r_infinity and shamir_exceptional)
    goes whole to the fix-up kernel, whose grid covers the worst case; every verdict equals
    the fixture's (5,000: latency kernels; 70,000: above their 32,768-tuple limit)."""
    f, exp, cat, names = p256_vectors
    sel = np.isin(cat, [names.index("r_infinity"), names.index("shamir_exceptional")])
    idx = np.resize(np.nonzero(sel)[0], n)
    got = gpu_kernel.verify(*split_fields(f[idx]))
    assert np.array_equal(got, exp[idx])


def test_device_hash_bounds_checked_on_launch_stream(gpu):
    """The device-resident hash entries validate every message against the blob on the launch
    stream before the launch: a message past the end and a uint64 offset >= 2^63 (which would
    wrap negative as int64) are refused; offsets produced on a side stream are read after their
    producer; check=False skips the validation (the caller's responsibility then)."""
    import torch
    dev = torch.device("cuda:0")
    blob = torch.arange(256, dtype=torch.int32, device=dev).to(torch.uint8)
    ln = torch.tensor([10, 20], dtype=torch.int32, device=dev)
    dig = torch.zeros((2, 32), dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        off = torch.tensor([0, 236], dtype=torch.int64, device=dev)
        torch.cuda._sleep(20_000_000)  # the producer is still running when the check is enqueued
        off.add_(1)                    # 1, 237: the second message ends at 257 > 256
    with pytest.raises(ValueError):
        gpu.sha256_dev(blob, off, ln, dig, stream=side)
    with pytest.raises(ValueError):
        gpu.sha256_dev(blob, torch.tensor([0, 1 << 63], dtype=torch.uint64, device=dev), ln, dig)
    with pytest.raises(ValueError):  # off + len would wrap to a small negative int64
        gpu.sha256_dev(blob, torch.tensor([0, (1 << 63) - 1], dtype=torch.int64, device=dev), ln, dig)
    ok_off = torch.tensor([1, 200], dtype=torch.int64, device=dev)
    gpu.sha256_dev(blob, ok_off, ln, dig)
    gpu.sha256_dev(blob, ok_off, ln, dig, check=False)
    torch.cuda.synchronize()
    host = bytes(range(256))
    assert dig[0].cpu().numpy().tobytes() == hashlib.sha256(host[1:11]).digest()
    assert dig[1].cpu().numpy().tobytes() == hashlib.sha256(host[200:220]).digest()
