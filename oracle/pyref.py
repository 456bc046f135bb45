"""Pure-Python big-int restatement of Go 1.24.1 crypto/ecdsa.Verify for P-256.

TEST INFRASTRUCTURE ONLY (third independent check beside oracle/p256_oracle.c
and OpenSSL). Affine arithmetic with Python's pow(x, -1, m); slow (~ms per
verify) so it runs on fixtures and hypothesis samples only.

Restated from the Go standard library (not present in /root/reference):
crypto/ecdsa/ecdsa.go Verify -> crypto/internal/fips140/ecdsa/ecdsa.go
verifyGeneric/hashToNat, crypto/internal/fips140/nistec P256Point.SetBytes.
"""
from __future__ import annotations

P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
G = (0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
     0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)


def on_curve(x: int, y: int) -> bool:
    return 0 <= x < P and 0 <= y < P and (y * y - (x * x * x - 3 * x + B)) % P == 0


def add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 - 3) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def mul(k: int, pt):
    acc = None
    for bit in bin(k)[2:] if k > 0 else "":
        acc = add(acc, acc)
        if bit == "1":
            acc = add(acc, pt)
    return acc


def hash_to_int(h: bytes) -> int:
    """hashToNat: leftmost N.Size() bytes, shorter hashes are smaller integers."""
    return int.from_bytes(h[:32], "big")


def verify(h: bytes, r: int, s: int, qx: int, qy: int) -> bool:
    if r <= 0 or s <= 0 or r >= N or s >= N:
        return False
    if not on_curve(qx, qy):
        return False
    e = hash_to_int(h) % N
    w = pow(s, -1, N)
    R = add(mul(e * w % N, G), mul(r * w % N, (qx, qy)))
    if R is None:
        return False
    return R[0] % N == r
