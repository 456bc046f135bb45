"""ctypes loader for the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker. The product library never calls
into it. See oracle/oracle.h for what is restated (Go 1.24.1 crypto/ecdsa.Verify
for P-256 and crypto/sha256) and how the restatement is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_u8p = ctypes.POINTER(ctypes.c_uint8)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def build() -> None:
    """Compile liboracle.so (and the OpenSSL helpers when libcrypto headers exist)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    if os.path.exists("/usr/include/openssl/ecdsa.h"):
        subprocess.run(["make", "-s", "-C", _HERE, "openssl_xcheck", "openssl_bench"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_verify_p256.restype = ctypes.c_int
        L.oracle_verify_p256_batch.argtypes = [_u8p] * 5 + [ctypes.c_size_t, _u8p, ctypes.c_int]
        L.oracle_sha256_batch.argtypes = [_u8p, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, _u8p,
                                          ctypes.c_int]
        _LIB = L
    return _LIB


def _b32(x) -> bytes:
    if isinstance(x, int):
        return (x % (1 << 256)).to_bytes(32, "big")
    b = bytes(x)
    assert len(b) == 32, len(b)
    return b


def verify(digest, r, s, qx, qy) -> bool:
    return bool(lib().oracle_verify_p256(_b32(digest), _b32(r), _b32(s), _b32(qx), _b32(qy)))


def verify_batch(digest: np.ndarray, r: np.ndarray, s: np.ndarray, qx: np.ndarray, qy: np.ndarray,
                 nthreads: int = 0) -> np.ndarray:
    """SoA uint8 arrays of shape (n, 32). Returns uint8 verdicts (n,)."""
    n = digest.shape[0]
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in (digest, r, s, qx, qy)]
    for a in arrs:
        assert a.shape == (n, 32)
    out = np.zeros(n, dtype=np.uint8)
    nt = nthreads if nthreads > 0 else (os.cpu_count() or 1)
    lib().oracle_verify_p256_batch(*[_ptr(a) for a in arrs], n, _ptr(out), nt)
    return out


def sha256(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_sha256(msg, ctypes.c_size_t(len(msg)), out)
    return out.raw


def sha256_batch(blob: np.ndarray, off: np.ndarray, ln: np.ndarray, nthreads: int = 0) -> np.ndarray:
    n = off.shape[0]
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    out = np.zeros((n, 32), dtype=np.uint8)
    nt = nthreads if nthreads > 0 else (os.cpu_count() or 1)
    lib().oracle_sha256_batch(_ptr(blob), off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                              ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n, _ptr(out), nt)
    return out


def normalize_hash(h: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_normalize_hash(h, ctypes.c_size_t(len(h)), out)
    return out.raw


def pubkey(d) -> tuple[bytes, bytes] | None:
    qx, qy = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    if not lib().oracle_pubkey(_b32(d), qx, qy):
        return None
    return qx.raw, qy.raw


def sign(d, k, digest) -> tuple[bytes, bytes] | None:
    r, s = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    if not lib().oracle_sign(_b32(d), _b32(k), _b32(digest), r, s):
        return None
    return r.raw, s.raw


def double_mul(a, b, qx, qy) -> tuple[bytes, bytes] | None:
    """a*G + b*Q, None for the point at infinity or an invalid Q."""
    ox, oy = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    if not lib().oracle_double_mul(_b32(a), _b32(b), _b32(qx), _b32(qy), ox, oy):
        return None
    return ox.raw, oy.raw


def lift_x(x, odd: int) -> bytes | None:
    y = ctypes.create_string_buffer(32)
    if not lib().oracle_lift_x(_b32(x), int(odd), y):
        return None
    return y.raw


def modn(op: str, a, b=0) -> int:
    out = ctypes.create_string_buffer(32)
    lib().oracle_modn({"add": 0, "sub": 1, "mul": 2, "inv": 3, "neg": 4}[op], _b32(a), _b32(b), out)
    return int.from_bytes(out.raw, "big")


def modp(op: str, a, b=0) -> int:
    out = ctypes.create_string_buffer(32)
    lib().oracle_modp({"add": 0, "sub": 1, "mul": 2, "inv": 3, "neg": 4}[op], _b32(a), _b32(b), out)
    return int.from_bytes(out.raw, "big")


P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5
