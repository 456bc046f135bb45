"""Differential parity sweep at scale (round 5): N seeded tuples -- GPU-signed, then a seeded mix of
corruptions and edge forms -- through every verify kernel of the engine and the keyed paths,
each compared verdict for verdict with the oracle (oracle/p256_oracle.c, the C restatement of Go's
crypto/ecdsa.Verify: the checker, as in the tests). Prints one JSON line.

  python tools/parity_sweep.py --n 2000000 --threads 16

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--seed", type=int, default=2605)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--exact", type=int, default=200_000, help="tuples through the exact (8x32) kernel")
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
                     ("half", gpuverify.KERNEL_HALF)):
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
    out["pass"] = all(v["bad"] == 0 for v in out["mismatches"].values())
    print(json.dumps(out), flush=True)
    gv.close()
    return 0 if out["pass"] else 1


if __name__ == "__main__":
    sys.exit(main())
