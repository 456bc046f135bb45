"""CPU tests: the oracle (test infrastructure) against the committed golden fixtures and
two independent restatements. No GPU."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import oracle
from oracle import pyref
from conftest import GOLDEN, split_fields


def test_oracle_matches_golden_vectors(p256_vectors):
    f, exp, cat, names = p256_vectors
    got = oracle.verify_batch(*split_fields(f))
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), names[cat[i]]) for i in bad[:10]]
    # every category is represented, with both verdicts where the category allows it
    assert set(np.unique(cat)) == set(range(len(names)))
    assert exp.sum() > 1000 and (exp == 0).sum() > 1000


def test_pyref_matches_golden_sample(p256_vectors):
    f, exp, cat, names = p256_vectors
    idx = np.concatenate([np.nonzero(cat == c)[0][:6] for c in range(len(names))])
    for i in idx:
        d, r, s, qx, qy = (bytes(f[i, 32 * k:32 * k + 32]) for k in range(5))
        v = pyref.verify(d, int.from_bytes(r, "big"), int.from_bytes(s, "big"),
                         int.from_bytes(qx, "big"), int.from_bytes(qy, "big"))
        assert v == bool(exp[i]), (int(i), names[cat[i]])


def test_messages_hash_to_digests(p256_vectors):
    f, exp, cat, names = p256_vectors
    raw = open(os.path.join(GOLDEN, "p256_messages.bin"), "rb").read()
    pos, count = 0, 0
    while pos < len(raw):
        i, ln = struct.unpack_from("<II", raw, pos)
        msg = raw[pos + 8:pos + 8 + ln]
        pos += 8 + ln
        assert hashlib.sha256(msg).digest() == bytes(f[i, :32])
        count += 1
    assert count > 1000


def _sha_msg(length, tag, seed=b"SBFT-GPUV-FIXTURES-1"):
    out = bytearray()
    ctr = 0
    while len(out) < length:
        out += hashlib.sha256(seed + b"shamsg" + str(tag).encode() + ctr.to_bytes(8, "little")).digest()
        ctr += 1
    return bytes(out[:length])


def test_sha256_kats():
    d = json.load(open(os.path.join(GOLDEN, "sha256_vectors.json")))
    for v in d["fips180_4"]:
        assert oracle.sha256(bytes.fromhex(v["msg_hex"])).hex() == v["sha256"]
    for v in d["seeded"]:
        assert oracle.sha256(_sha_msg(v["len"], v["tag"])).hex() == v["sha256"]


def test_sha256_batch_matches_hashlib():
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 300, size=200).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    blob = rng.integers(0, 256, size=int(lens.sum()) + 1, dtype=np.uint8)
    got = oracle.sha256_batch(blob, off, lens)
    for i in range(len(lens)):
        m = blob[int(off[i]):int(off[i]) + int(lens[i])].tobytes()
        assert got[i].tobytes() == hashlib.sha256(m).digest()


def test_normalize_hash_go_semantics():
    assert oracle.normalize_hash(b"") == b"\0" * 32
    assert oracle.normalize_hash(b"\x01\x02") == b"\0" * 30 + b"\x01\x02"
    h = bytes(range(64))
    assert oracle.normalize_hash(h) == h[:32]


@settings(max_examples=25, deadline=None)
@given(st.integers(1, oracle.N - 1), st.integers(1, oracle.N - 1), st.binary(min_size=0, max_size=80))
def test_sign_verify_roundtrip_property(d, k, msg):
    e = oracle.normalize_hash(hashlib.sha256(msg).digest())
    qx, qy = oracle.pubkey(d)
    sig = oracle.sign(d, k, e)
    if sig is None:
        return
    r, s = sig
    assert oracle.verify(e, r, s, qx, qy)
    assert oracle.verify(e, r, (oracle.N - int.from_bytes(s, "big")), qx, qy)  # high-s accepted
    bad = (int.from_bytes(s, "big") ^ 2) % oracle.N
    assert oracle.verify(e, r, bad, qx, qy) == pyref.verify(
        e, int.from_bytes(r, "big"), bad, int.from_bytes(qx, "big"), int.from_bytes(qy, "big"))


def test_scalar_helpers():
    a, b = 12345678901234567890, 98765432109876543210
    assert oracle.modn("mul", a, b) == a * b % oracle.N
    assert oracle.modn("inv", a) == pow(a, -1, oracle.N)
    assert oracle.modp("mul", a, b) == a * b % oracle.P
    assert oracle.modp("sub", a, b) == (a - b) % oracle.P
