#!/usr/bin/env python3
"""Generate tests/golden/p256_crafted.bin: crafted exceptional P-256 tuples (data fixture).

Run from the repo root in the build container:  python tests/golden/gen_crafted.py

Each tuple is a signature whose scalars u1 = e/s, u2 = r/s make a lean point addition of the
engine's verify ladders meet acc == +-addend (p256_f29.hpp add_aff_fix, p256_verify.hip):
  ladder_last : the last addition of the u2 Q ladder (u2 = n - 2|d| or 2|d|: P + P);
  comb_dbl_j  : comb step j (0..K) of u1 G on top of u2 Q meets acc == entry (P + P);
  comb_inf_j  : ... meets acc == -entry (P + (-P)); at j = K that is R = infinity.
(K = ceil(256 / W) windows of W = SBFT_GCOMB_W bits: the engine's comb, 22-bit windows.)
The key is Q = q G with q chosen so that u2 q + (the comb's partial sum) = +-(the entry), which
any client can do for its own request. Verdicts are the oracle's (oracle/p256_oracle.c, Go
crypto/ecdsa.Verify restated), cross-checked with the pure-Python restatement (oracle/pyref.py).
Deterministic: tests/test_golden_crafted.py regenerates the bytes and compares.

Output: p256_crafted.bin (162-byte records: digest|r|s|qx|qy, verdict, tag id) and
p256_crafted.json (tag names).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import pyref  # noqa: E402

N = oracle.N
GW = 22  # the comb's window bits (SBFT_GCOMB_W, p256_verify.hip)
KG = (256 + GW - 1) // GW
TOP = 1 << (GW * KG)  # the comb's constant term 2^(W K) (table[K][0] = 2^(W K) G)


def _b(x: int) -> bytes:
    return (x % (1 << 256)).to_bytes(32, "big")


def craft(u1: int, u2: int, q: int, rng):
    """(digest, r, s, qx, qy) with scalars exactly u1 = e/s, u2 = r/s under Q = q G."""
    qx, qy = oracle.pubkey(q)
    R = oracle.double_mul(u1, u2, qx, qy)
    r = int.from_bytes(R[0], "big") % N if R is not None else int(rng.integers(1, 1 << 62))
    if r == 0:
        return None
    s = r * pow(u2, -1, N) % N
    e = u1 * s % N
    return _b(e), _b(r), _b(s), qx, qy


def comb_digits(u1: int):
    """The comb's recoding of u1 (comb_add_u1g): sign s1 and the odd digits of u1' with
    u1' = sum d_i 2^(W i) + 2^(W K), u1' = u1 (odd) or n - u1 (even u1, negated base)."""
    neg = u1 % 2 == 0
    u = N - u1 if neg else u1
    m = (1 << GW) - 1
    d = [2 * ((u >> (GW * i + 1)) & m) - m for i in range(KG)]
    assert sum(di << (GW * i) for i, di in enumerate(d)) + TOP == u
    return (-1 if neg else 1), d


def comb_collision(u1: int, u2: int, j: int, kind: str):
    """q such that acc == +-entry at comb step j (0..K) for these scalars (None if q = 0)."""
    s1, d = comb_digits(u1)
    partial = sum(d[i] << (GW * i) for i in range(min(j, KG)))
    entry = s1 * (d[j] << (GW * j) if j < KG else TOP)
    target = (entry if kind == "dbl" else -entry) - s1 * partial
    q = target * pow(u2, -1, N) % N
    return q or None


def crafted_set(seed=7):
    rng = np.random.default_rng(seed)
    rows, tags = [], []
    rnd = lambda: int.from_bytes(rng.bytes(32), "big") % (N - 1) + 1
    for k in range(1, 16, 2):
        for u2 in (N - 2 * k, 2 * k):
            t = craft(rnd(), u2, rnd(), rng)
            if t:
                rows.append(t)
                tags.append(f"ladder_last_{'neg' if u2 > N // 2 else 'pos'}{k}")
    for j in range(KG + 1):
        for kind in ("dbl", "inf"):
            for _ in range(3):
                u1, u2 = rnd(), rnd()
                q = comb_collision(u1, u2, j, kind)
                if q is None:
                    continue
                t = craft(u1, u2, q, rng)
                if t:
                    rows.append(t)
                    tags.append(f"comb_{kind}_{j}")
    return rows, tags


def records():
    rows, tags = crafted_set()
    names = sorted(set(tags))
    out = bytearray()
    for row, tag in zip(rows, tags):
        e, r, s, qx, qy = row
        v = oracle.verify(e, r, s, qx, qy)
        w = pyref.verify(e, int.from_bytes(r, "big"), int.from_bytes(s, "big"), int.from_bytes(qx, "big"),
                         int.from_bytes(qy, "big"))
        if bool(v) != bool(w):
            raise SystemExit(f"oracle and pyref disagree on {tag}")
        out += e + r + s + qx + qy + bytes([1 if v else 0, names.index(tag)])
    return bytes(out), names


def main():
    data, names = records()
    out = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(out, "p256_crafted.bin"), "wb") as f:
        f.write(data)
    with open(os.path.join(out, "p256_crafted.json"), "w") as f:
        json.dump({"tags": names, "count": len(data) // 162}, f, indent=1)
    print(f"{len(data) // 162} crafted records, {len(names)} tags")


if __name__ == "__main__":
    main()
