#!/usr/bin/env python3
"""Generate the committed P-256 / SHA-256 golden fixtures.

Run from the repo root in the build container:  python tests/golden/gen_fixtures.py

The reference (pkucode/SmartBFT) holds no cryptographic test vectors (SURVEY.md
8(c): parity unpinned by the reference) and Wycheproof is not available offline,
so this script synthesises the same categories deterministically and pins every
verdict three ways before writing it:
  1. oracle/p256_oracle.c (C restatement of Go crypto/ecdsa.Verify),
  2. oracle/pyref.py (pure-Python affine restatement),
  3. OpenSSL 3.0.2 ECDSA_do_verify (oracle/openssl_xcheck, SEC1 key decoding),
and, for vectors with a known message, 4. Node crypto.verify (oracle/node_xcheck.js).
Any disagreement aborts generation.

Output (tests/golden/):
  p256_vectors.bin   records of 162 bytes: digest|r|s|qx|qy (32 B big-endian each),
                     expected verdict (1 B), category id (1 B)
  p256_messages.bin  for records with a known preimage: u32 index, u32 len, message
  p256_categories.json  category id -> name, count
  sha256_vectors.json   SHA-256 KATs (FIPS 180-4 examples + seeded lengths)
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import pyref  # noqa: E402

N, P = oracle.N, oracle.P
SEED = b"SBFT-GPUV-FIXTURES-1"
OUT = os.path.join(ROOT, "tests", "golden")


def H(*parts) -> bytes:
    h = hashlib.sha256(SEED)
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
    return h.digest()


def Hint(*parts, mod=N) -> int:
    v = int.from_bytes(H(*parts), "big") % mod
    return v if v else 1


def b32(x: int) -> bytes:
    return (x % (1 << 256)).to_bytes(32, "big")


CATS = [
    "valid_random", "flip_r_bit", "flip_s_bit", "flip_e_bit", "r_special", "s_special",
    "q_offcurve", "q_swapped", "qx_ge_p", "q_noncanonical", "rx_ge_n", "r_infinity",
    "shamir_exceptional", "e_special", "high_s", "small_scalars", "valid_crafted",
    "digest_zero_and_max",
]
CID = {c: i for i, c in enumerate(CATS)}

records: list[tuple[bytes, int, int, int, int, int]] = []  # digest, r, s, qx, qy, cat
messages: dict[int, bytes] = {}


def add(digest: bytes, r: int, s: int, qx: int, qy: int, cat: str, msg: bytes | None = None):
    if msg is not None:
        messages[len(records)] = msg
    records.append((digest, r, s, qx, qy, CID[cat]))


def keypair(tag):
    d = Hint("key", tag)
    qx, qy = oracle.pubkey(d)
    return d, int.from_bytes(qx, "big"), int.from_bytes(qy, "big")


def signed(tag):
    d, qx, qy = keypair(tag)
    msg = H("msg", tag) + H("msg2", tag)  # 64-byte message, like the 1M workload
    e = hashlib.sha256(msg).digest()
    r, s = oracle.sign(d, Hint("k", tag), e)
    return e, int.from_bytes(r, "big"), int.from_bytes(s, "big"), qx, qy, msg


def craft(a: int, b: int, qx: int, qy: int):
    """Valid signature with u1 = a, u2 = b for an arbitrary key Q (dlog unknown)."""
    R = oracle.double_mul(a, b, qx, qy)
    if R is None:
        return None
    r = int.from_bytes(R[0], "big") % N
    if r == 0:
        return None
    s = r * pow(b, -1, N) % N
    e = a * s % N
    return b32(e), r, s


def point(k: int):
    x, y = oracle.pubkey(k % N)
    return int.from_bytes(x, "big"), int.from_bytes(y, "big")


def gen_p256():
    for i in range(1000):
        e, r, s, qx, qy, msg = signed(("valid", i))
        add(e, r, s, qx, qy, "valid_random", msg)
    for i in range(200):
        e, r, s, qx, qy, msg = signed(("fr", i))
        add(e, r ^ (1 << (Hint("bit", "fr", i) % 256)), s, qx, qy, "flip_r_bit", msg)
        e, r, s, qx, qy, msg = signed(("fs", i))
        add(e, r, s ^ (1 << (Hint("bit", "fs", i) % 256)), qx, qy, "flip_s_bit", msg)
        e, r, s, qx, qy, _ = signed(("fe", i))
        eb = bytearray(e)
        bit = Hint("bit", "fe", i) % 256
        eb[bit // 8] ^= 1 << (bit % 8)
        add(bytes(eb), r, s, qx, qy, "flip_e_bit")
    specials = [0, 1, N - 1, N, N + 1, (1 << 256) - 1, P - 1, 1 << 255]
    for j, v in enumerate(specials):
        for i in range(4):
            e, r, s, qx, qy, msg = signed(("rsp", j, i))
            add(e, v, s, qx, qy, "r_special", msg)
            e, r, s, qx, qy, msg = signed(("ssp", j, i))
            add(e, r, v, qx, qy, "s_special", msg)
    for i in range(150):
        e, r, s, qx, qy, msg = signed(("offc", i))
        add(e, r, s, qx, (qy + 1) % P, "q_offcurve", msg)
        e, r, s, qx, qy, msg = signed(("offx", i))
        add(e, r, s, (qx + 1 + i) % P, qy, "q_offcurve", msg)
    prev = None
    for i in range(150):
        cur = signed(("swap", i))
        if prev is not None:
            e, r, s, _, _, msg = cur
            add(e, r, s, prev[3], prev[4], "q_swapped", msg)
        prev = cur
    # Qx >= p with Qx - p a real x coordinate: points with x < 2^256 - p.
    found = 0
    i = 0
    while found < 24:
        i += 1
        x = Hint("smallx", i, mod=1 << 223)
        y = oracle.lift_x(x, i & 1)
        if y is None:
            continue
        y = int.from_bytes(y, "big")
        c = craft(Hint("qa", i), Hint("qb", i), x, y)
        if c is None:
            continue
        e, r, s = c
        add(e, r, s, x, y, "valid_crafted")          # accepted with the canonical key
        add(e, r, s, x + P, y, "qx_ge_p")            # the same point, non-canonical x
        add(e, r, s, x, y + P if y + P < (1 << 256) else P + 1, "qx_ge_p")
        found += 1
    for i, (qx, qy) in enumerate([(0, 0), (P, 0), (0, P), (P, P), ((1 << 256) - 1, (1 << 256) - 1),
                                  (oracle.GX, P - oracle.GY + P if P - oracle.GY + P < (1 << 256) else P),
                                  (oracle.GX + P if oracle.GX + P < (1 << 256) else P, oracle.GY)]):
        e, r, s, _, _, msg = signed(("nonc", i))
        add(e, r, s, qx, qy, "q_noncanonical", msg)
    # R.x in [n, p): signatures whose R.x needs the r + n comparison.
    found = 0
    i = 0
    while found < 40:
        i += 1
        x = N + Hint("rxn", i, mod=P - N)
        y = oracle.lift_x(x, i & 1)
        if y is None:
            continue
        y = int.from_bytes(y, "big")
        a, b = Hint("rxa", i), Hint("rxb", i)
        T = oracle.double_mul(N - a, 1, x, y)            # R - aG
        if T is None:
            continue
        Q = oracle.double_mul(0, pow(b, -1, N), T[0], T[1])  # Q = b^-1 (R - aG)
        qx, qy = int.from_bytes(Q[0], "big"), int.from_bytes(Q[1], "big")
        r = x - N
        s = r * pow(b, -1, N) % N
        e = b32(a * s % N)
        add(e, r, s, qx, qy, "rx_ge_n")                  # valid
        add(e, x, s, qx, qy, "rx_ge_n")                  # r >= n: out of range
        add(e, r, (N - s) % N, qx, qy, "rx_ge_n")        # -R has the same x: valid
        eb = bytearray(e)
        eb[31] ^= 1
        add(bytes(eb), r, s, qx, qy, "rx_ge_n")          # wrong digest
        found += 1
    # R = infinity: Q = -(a/b) G, u1 = a, u2 = b.
    for i in range(60):
        a, b = Hint("ia", i), Hint("ib", i)
        if i % 3 == 0:
            a = b  # Q = -G
        qx, qy = point(N - a * pow(b, -1, N) % N)
        s = Hint("is", i)
        r = b * s % N
        add(b32(a * s % N), r, s, qx, qy, "r_infinity")
    # Exceptional additions inside the double-scalar multiplication.
    ks = [1, N - 1, 2, N - 2, 3, 5, 7, 8, 9, 15, 16, 17, 31, 33, 255, 256, 257, 1 << 128]
    for k in ks:
        qx, qy = point(k)
        pats = [(1, 1), (2, 1), (1, 2), (k, 1), (N - 1, 1), (1, N - 1), (Hint("sa", k), Hint("sa", k)),
                (Hint("sb", k), N - Hint("sb", k)), ((1 << 128) + 1, (1 << 128) + 1), (0x10, 0x10),
                (0x80000000, 0x80000000), (Hint("sc", k), 1), (N - 2, 3)]
        for a, b in pats:
            a, b = a % N, b % N
            if a == 0 or b == 0:
                continue
            c = craft(a, b, qx, qy)
            if c is None:
                # aG + bQ = infinity: still a vector (reject) with u1=a, u2=b
                s = Hint("exs", k, a, b)
                add(b32(a * s % N), b * s % N, s, qx, qy, "shamir_exceptional")
                continue
            e, r, s = c
            add(e, r, s, qx, qy, "shamir_exceptional")
            add(e, r, (N - s) % N, qx, qy, "shamir_exceptional")
    # e special: e = 0, e = n (== 0 mod n), e = 2^256 - 1, e = n - 1.
    for i, ev in enumerate([0, N, (1 << 256) - 1, N - 1, N + 1, 1]):
        for j in range(4):
            d, qx, qy = keypair(("esp", i, j))
            r, s = oracle.sign(d, Hint("esk", i, j), b32(ev))
            add(b32(ev), int.from_bytes(r, "big"), int.from_bytes(s, "big"), qx, qy, "e_special")
    for i in range(100):
        e, r, s, qx, qy, msg = signed(("highs", i))
        add(e, r, N - s, qx, qy, "high_s", msg)
    for i in range(60):
        d, qx, qy = keypair(("small", i))
        a = (i % 17) + 1 if i % 2 else Hint("sma", i)
        b = (i % 13) + 1 if i % 3 else Hint("smb", i)
        c = craft(a, b, qx, qy)
        if c:
            e, r, s = c
            add(e, r, s, qx, qy, "small_scalars")
    for i in range(200):
        qx, qy = point(Hint("cq", i))
        c = craft(Hint("ca", i), Hint("cb", i), qx, qy)
        if c:
            e, r, s = c
            add(e, r, s, qx, qy, "valid_crafted")
    for i in range(8):
        d, qx, qy = keypair(("dz", i))
        dig = [b"\x00" * 32, b"\xff" * 32][i & 1]
        r, s = oracle.sign(d, Hint("dzk", i), dig)
        add(dig, int.from_bytes(r, "big"), int.from_bytes(s, "big"), qx, qy, "digest_zero_and_max")


def node_check(idx_msgs, recs):
    """Node crypto.verify on records with a known message (SPKI key, DER signature)."""
    script = os.path.join(ROOT, "oracle", "node_xcheck.js")
    lines = []
    for i, msg in idx_msgs:
        d, r, s, qx, qy, _ = recs[i]
        lines.append(json.dumps({"msg": msg.hex(), "r": b32(r).hex(), "s": b32(s).hex(),
                                 "qx": b32(qx).hex(), "qy": b32(qy).hex()}))
    res = subprocess.run(["node", script], input="\n".join(lines).encode(), capture_output=True,
                         check=True)
    return [int(c) for c in res.stdout.decode().split()]


def main():
    gen_p256()
    n = len(records)
    raw = b"".join(d + b32(r) + b32(s) + b32(qx) + b32(qy) for d, r, s, qx, qy, _ in records)
    # 1. C oracle
    import numpy as np
    arr = np.frombuffer(raw, dtype=np.uint8).reshape(n, 160)
    v_c = oracle.verify_batch(arr[:, 0:32], arr[:, 32:64], arr[:, 64:96], arr[:, 96:128],
                              arr[:, 128:160])
    # 2. pure-Python restatement
    v_py = np.array([pyref.verify(d, r, s, qx, qy) for d, r, s, qx, qy, _ in records], dtype=np.uint8)
    # 3. OpenSSL (records with out-of-range 256-bit r/s fit 32 bytes; oct2point rejects x,y >= p)
    res = subprocess.run([os.path.join(ROOT, "oracle", "openssl_xcheck")], input=raw,
                         capture_output=True, check=True)
    v_ossl = np.frombuffer(res.stdout, dtype=np.uint8)
    assert v_ossl.shape == (n,), v_ossl.shape
    bad = np.nonzero((v_c != v_py) | (v_c != v_ossl))[0]
    if len(bad):
        for i in bad[:20]:
            print("DISAGREE", i, CATS[records[i][5]], v_c[i], v_py[i], v_ossl[i])
        raise SystemExit(1)
    # 4. Node on the message-bearing subset
    idx_msgs = sorted(messages.items())
    v_node = node_check(idx_msgs, records)
    for (i, _), v in zip(idx_msgs, v_node):
        if v != v_c[i]:
            raise SystemExit(f"node disagrees at {i} ({CATS[records[i][5]]}): {v} vs {v_c[i]}")
    with open(os.path.join(OUT, "p256_vectors.bin"), "wb") as f:
        for k in range(n):
            f.write(raw[160 * k:160 * (k + 1)] + bytes([int(v_c[k]), records[k][5]]))
    with open(os.path.join(OUT, "p256_messages.bin"), "wb") as f:
        for i, msg in idx_msgs:
            f.write(struct.pack("<II", i, len(msg)) + msg)
    counts = {}
    for k in range(n):
        c = CATS[records[k][5]]
        counts.setdefault(c, [0, 0])
        counts[c][0] += 1
        counts[c][1] += int(v_c[k])
    with open(os.path.join(OUT, "p256_categories.json"), "w") as f:
        json.dump({"categories": CATS,
                   "counts": {c: {"total": t, "accept": a} for c, (t, a) in counts.items()},
                   "records": n, "node_checked": len(idx_msgs),
                   "checked_by": ["oracle/p256_oracle.c", "oracle/pyref.py",
                                  "OpenSSL 3.0.2 ECDSA_do_verify", "node crypto.verify (subset)"]},
                  f, indent=1)
    gen_sha()
    print(f"wrote {n} P-256 vectors ({int(v_c.sum())} accept), node-checked {len(idx_msgs)}")


def sha_msg(length: int, tag) -> bytes:
    out = bytearray()
    ctr = 0
    while len(out) < length:
        out += hashlib.sha256(SEED + b"shamsg" + str(tag).encode() + ctr.to_bytes(8, "little")).digest()
        ctr += 1
    return bytes(out[:length])


def gen_sha():
    """SHA-256 KATs: FIPS 180-4 examples plus padding-boundary lengths with seeded messages
    (sha_msg above is reproduced in tests/test_oracle.py). Each digest is checked against
    hashlib and the C oracle; `openssl dgst` agrees with hashlib on this image."""
    vecs = [{"msg_hex": b"abc".hex(),
             "sha256": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"},
            {"msg_hex": b"".hex(),
             "sha256": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"},
            {"msg_hex": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq".hex(),
             "sha256": "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"}]
    for v in vecs:
        assert hashlib.sha256(bytes.fromhex(v["msg_hex"])).hexdigest() == v["sha256"]
    lengths = [0, 1, 3, 31, 32, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 1024,
               4095, 4096, 10240, 65535, 65536]
    seeded = []
    for L in lengths:
        m = sha_msg(L, L)
        dg = hashlib.sha256(m).hexdigest()
        assert oracle.sha256(m).hex() == dg
        seeded.append({"len": L, "tag": L, "sha256": dg})
    with open(os.path.join(OUT, "sha256_vectors.json"), "w") as f:
        json.dump({"fips180_4": vecs, "seeded": seeded,
                   "seeded_generator": "concat sha256(SEED+b'shamsg'+str(tag)+ctr_le64), "
                                       "SEED=" + SEED.decode()}, f, indent=1)


if __name__ == "__main__":
    main()
