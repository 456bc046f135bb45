"""Differential parity sweep at scale (round 5; round 6 adds the wide half kernel): N seeded tuples -- GPU-signed, then a seeded mix of
corruptions and edge forms -- through every verify kernel of the engine and the keyed paths,
each compared verdict for verdict with the oracle (oracle/p256_oracle.c, the C restatement of Go's
crypto/ecdsa.Verify: the checker, as in the tests). Prints one JSON line.

  python tools/parity_sweep.py --n 2000000 --threads 16

With --hash / --framed, messages hashed on the GPU as well (config 5's HBM and streamed paths, the
VerifyProposal layout through the fused half kernel): see hash_sweep.

Kinds (a tuple gets one; ~30% stay untouched):
  flip r / s / e bit, r = 0, s = 0, s = n, r = n + small, r = n - 1, s = n - s (high-s form, still
  valid), Qy -> Qy + 1 (off the curve), Q -> -Q (a valid point, the wrong key), Qx / Qy >= p,
  e = 0, e = 2^256 - 1, r = random, s = random, Q = G.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smartbft_amd import gpuverify  # noqa: E402
import oracle  # noqa: E402  (the checker)

N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5
KINDS = ["none", "flip_r", "flip_s", "flip_e", "r0", "s0", "s_n", "r_n_plus", "r_n_minus1", "high_s", "qy_plus1",
         "neg_q", "qx_ge_p", "qy_ge_p", "e0", "e_max", "r_rand", "s_rand", "q_is_g"]


def be(x):
    return np.frombuffer(x.to_bytes(32, "big"), dtype=np.uint8)


def scalars(rng, n):
    """n uniform scalars in [1, n) as (n, 32) big-endian bytes (rejection on the top word)."""
    out = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    out[:, 0] = np.minimum(out[:, 0], 0xFE)  # < 2^255.99: below n for all but a negligible few
    out[:, 31] |= 1  # nonzero
    return out


def build(gv, n, seed):
    rng = np.random.default_rng(seed)
    d, k = scalars(rng, n), scalars(rng, n)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    one = np.zeros((n, 32), dtype=np.uint8)
    one[:, 31] = 1
    qx, qy, _, _, st = gv.sign(d, one, one)  # the public keys
    assert (st == 1).all()
    _, _, r, s, st = gv.sign(d, k, e)
    assert (st == 1).all()
    kind = rng.integers(0, len(KINDS), size=n)
    kind[rng.random(n) < 0.3] = 0
    r, s, e, qx, qy = (np.array(a) for a in (r, s, e, qx, qy))
    byte, bit = rng.integers(0, 32, size=n), rng.integers(0, 8, size=n)
    for i in np.nonzero(kind)[0]:
        kd = KINDS[kind[i]]
        if kd == "flip_r":
            r[i, byte[i]] ^= np.uint8(1 << bit[i])
        elif kd == "flip_s":
            s[i, byte[i]] ^= np.uint8(1 << bit[i])
        elif kd == "flip_e":
            e[i, byte[i]] ^= np.uint8(1 << bit[i])
        elif kd == "r0":
            r[i] = 0
        elif kd == "s0":
            s[i] = 0
        elif kd == "s_n":
            s[i] = be(N)
        elif kd == "r_n_plus":
            r[i] = be(N + int(byte[i]))
        elif kd == "r_n_minus1":
            r[i] = be(N - 1)
        elif kd == "high_s":
            s[i] = be(N - int.from_bytes(s[i].tobytes(), "big"))
        elif kd == "qy_plus1":
            qy[i] = be((int.from_bytes(qy[i].tobytes(), "big") + 1) % (1 << 256))
        elif kd == "neg_q":
            qy[i] = be((P - int.from_bytes(qy[i].tobytes(), "big")) % P)
        elif kd == "qx_ge_p":
            qx[i] = be(int.from_bytes(qx[i].tobytes(), "big") + P if int.from_bytes(qx[i].tobytes(), "big") < (1 << 256) - P else P)
        elif kd == "qy_ge_p":
            qy[i] = be(P + int(byte[i]))
        elif kd == "e0":
            e[i] = 0
        elif kd == "e_max":
            e[i] = 0xFF
        elif kd == "r_rand":
            r[i] = rng.integers(0, 256, size=32, dtype=np.uint8)
        elif kd == "s_rand":
            s[i] = rng.integers(0, 256, size=32, dtype=np.uint8)
        elif kd == "q_is_g":
            qx[i], qy[i] = be(GX), be(GY)
    return e, r, s, qx, qy, kind


def hash_sweep(gv, a, out, record_to):
    """Messages hashed on the GPU, then verified: the HBM path (config 5), the streamed path, and
    the VerifyProposal layout (body ending in qx || qy, r || s after it; the fused half kernel at
    10k per call, the size-selected kernels at 50k). Corruptions: a body byte flipped after
    signing, r or s flipped, the key's last byte flipped (framed: off the curve, and a different
    digest). The oracle gets hashlib's digests."""
    import hashlib
    rng = np.random.default_rng(a.seed + 1)

    def keys_and_sigs(bodies):
        m = len(bodies)
        d, k = scalars(rng, m), scalars(rng, m)
        one = np.zeros((m, 32), dtype=np.uint8)
        one[:, 31] = 1
        qx, qy, _, _, st = gv.sign(d, one, one)
        assert (st == 1).all()
        return d, k, np.array(qx), np.array(qy)

    def sign(d, k, bodies):
        e = np.frombuffer(b"".join(hashlib.sha256(b).digest() for b in bodies), dtype=np.uint8).reshape(-1, 32)
        _, _, r, s, st = gv.sign(d, k, e)
        assert (st == 1).all()
        return np.array(r), np.array(s)

    def check(name, got, bodies, r, s, qx, qy):
        e = np.frombuffer(b"".join(hashlib.sha256(b).digest() for b in bodies), dtype=np.uint8).reshape(-1, 32)
        want = oracle.verify_batch(e, r, s, qx, qy, nthreads=a.threads)
        bad = int((got != want).sum())
        record_to[name] = {"tuples": int(len(got)), "bad": bad, "accepts": int(want.sum())}
        print(name, len(got), "bad", bad, flush=True)

    # config-5 layout: free-standing messages
    m = a.hash
    lens = rng.integers(0, 4097, size=m)
    raw = rng.integers(0, 256, size=int(lens.sum()) + m * 3, dtype=np.uint8).tobytes()
    bodies, pos = [], 0
    for ln in lens:
        pos += int(rng.integers(0, 4))  # unaligned starts
        bodies.append(raw[pos:pos + int(ln)])
        pos += int(ln)
    d, k, qx, qy = keys_and_sigs(bodies)
    r, s = sign(d, k, bodies)
    kind = rng.integers(0, 4, size=m)
    bodies = [bytearray(b) for b in bodies]
    for i in np.nonzero(kind == 1)[0]:
        if len(bodies[i]):
            bodies[i][int(rng.integers(0, len(bodies[i])))] ^= 1
    for i in np.nonzero(kind == 2)[0]:
        r[i, 31] ^= 1
    for i in np.nonzero(kind == 3)[0]:
        s[i, 0] ^= 0x80
    bodies = [bytes(b) for b in bodies]
    off = np.zeros(m, dtype=np.uint64)
    p = 0
    for i, b in enumerate(bodies):
        p += i % 4
        off[i] = p
        p += len(b)
    blob = bytearray(p)
    for i, b in enumerate(bodies):
        blob[int(off[i]):int(off[i]) + len(b)] = b
    blob = np.frombuffer(bytes(blob), dtype=np.uint8)
    ln = np.array([len(b) for b in bodies], dtype=np.uint32)
    check("hash_verify_hbm", gv.sha256_verify(blob, off, ln, r, s, qx, qy), bodies, r, s, qx, qy)
    check("hash_verify_stream", gv.sha256_verify_stream(blob, off, ln, r, s, qx, qy, window_bytes=64 << 20),
          bodies, r, s, qx, qy)

    # VerifyProposal layout: body = payload || qx || qy, then r || s
    f = a.framed
    d, k, qx, qy = keys_and_sigs([b""] * f)
    pay = [rng.integers(0, 256, size=int(rng.integers(0, 400)), dtype=np.uint8).tobytes() for _ in range(f)]
    bodies = [pay[i] + qx[i].tobytes() + qy[i].tobytes() for i in range(f)]
    r, s = sign(d, k, bodies)
    kind = rng.integers(0, 4, size=f)
    bodies = [bytearray(b) for b in bodies]
    for i in np.nonzero(kind == 1)[0]:
        bodies[i][int(rng.integers(0, len(bodies[i])))] ^= 4
    for i in np.nonzero(kind == 2)[0]:
        s[i, 31] ^= 1
    for i in np.nonzero(kind == 3)[0]:
        bodies[i][-1] ^= 1  # the key's last byte: off the curve (and another digest)
    bodies = [bytes(b) for b in bodies]
    qxf = np.frombuffer(b"".join(b[-64:-32] for b in bodies), dtype=np.uint8).reshape(f, 32)
    qyf = np.frombuffer(b"".join(b[-32:] for b in bodies), dtype=np.uint8).reshape(f, 32)
    parts, offs, lns, p = [], [], [], 1
    for i, b in enumerate(bodies):
        offs.append(p)
        lns.append(len(b))
        parts.append(b + r[i].tobytes() + s[i].tobytes())
        p += len(b) + 64
    blob = np.frombuffer(b"\0" + b"".join(parts), dtype=np.uint8)
    offs, lns = np.array(offs, dtype=np.uint64), np.array(lns, dtype=np.uint32)
    got = np.concatenate([gv.sha256_verify_framed(blob, offs[i:i + 10_000], lns[i:i + 10_000], 0, -64)
                          for i in range(0, f, 10_000)])
    check("framed_10k_calls", got, bodies, r, s, qxf, qyf)
    check("framed_one_call", gv.sha256_verify_framed(blob, offs, lns, 0, -64), bodies, r, s, qxf, qyf)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--seed", type=int, default=2605)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--exact", type=int, default=200_000, help="tuples through the exact (8x32) kernel")
    ap.add_argument("--hash", type=int, default=300_000,
                    help="messages (0-4096 B, unaligned, hashed on the GPU) for the hash + verify paths")
    ap.add_argument("--framed", type=int, default=50_000, help="signed requests in the VerifyProposal layout")
    ap.add_argument("--keyed", type=int, default=3000,
                    help="tuples through the keyed paths (a 512 KiB comb table per registered key)")
    a = ap.parse_args()
    gv = gpuverify.GpuVerifier(device_mask=1)
    t0 = time.time()
    e, r, s, qx, qy, kind = build(gv, a.n, a.seed)
    t1 = time.time()
    exp = oracle.verify_batch(e, r, s, qx, qy, nthreads=a.threads)
    t2 = time.time()
    out = {"n": a.n, "seed": a.seed, "accepts": int(exp.sum()), "gen_s": round(t1 - t0, 1), "oracle_s": round(t2 - t1, 1),
           "kinds": {KINDS[j]: int((kind == j).sum()) for j in range(len(KINDS))}, "mismatches": {}}

    def record(name, got, idx=None):
        want = exp if idx is None else exp[idx]
        k = kind if idx is None else kind[idx]
        bad = np.nonzero(got != want)[0]
        out["mismatches"][name] = {"tuples": int(len(got)), "bad": int(len(bad)),
                                   "by_kind": {KINDS[j]: int((k[bad] == j).sum()) for j in np.unique(k[bad])}}
        print(name, len(got), "bad", len(bad), flush=True)

    fields = (e, r, s, qx, qy)
    record("selected", gv.verify(*fields))
    for name, kn in (("throughput", gpuverify.KERNEL_THROUGHPUT), ("pair", gpuverify.KERNEL_PAIR),
                     ("half", gpuverify.KERNEL_HALF), ("half_wide", gpuverify.KERNEL_HALF_WIDE)):
        record(name, gv.verify_kernel(kn, *fields))
    sub = np.arange(min(a.exact, a.n))
    record("exact", gv.verify_kernel(gpuverify.KERNEL_EXACT, *(f[sub] for f in fields)), sub)
    # keyed: register the keys of a subset (valid points only: an invalid key cannot be registered
    # as a consenter; the keyed paths then verify against the registered key ids)
    ks = np.arange(min(a.keyed, a.n))
    ids = gv.register_keys(qx[ks], qy[ks])
    okk = ids > 0
    sel = ks[okk]
    kid = ids[okk]
    for name, step in (("keyed_wave_67", 67), ("keyed_wave_500", 500)):  # host s^-1 / device s^-1
        got = np.concatenate([gv.verify_keyed(*(f[sel[i:i + step]] for f in (e, r, s)), kid[i:i + step])
                              for i in range(0, len(sel), step)])
        record(name, got, sel)
    record("keyed_lanes", gv.verify_keyed(e[sel], r[sel], s[sel], kid), sel)  # >= 1025: four lanes
    out["keyed_registered"] = int(okk.sum())
    if a.hash:
        hash_sweep(gv, a, out, record_to=out["mismatches"])
    out["pass"] = all(v["bad"] == 0 for v in out["mismatches"].values())
    print(json.dumps(out), flush=True)
    gv.close()
    return 0 if out["pass"] else 1


if __name__ == "__main__":
    sys.exit(main())
