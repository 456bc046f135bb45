"""CPU tests that pin the oracle and the committed fixtures to third-party verifiers on every
run, not only at fixture-generation time (tests/golden/gen_fixtures.py):

- OpenSSL 3.0.2 libcrypto ECDSA_do_verify (oracle/openssl_xcheck, SEC1 key decoding) over
  every record of tests/golden/p256_vectors.bin and tests/golden/p256_crafted.bin;
- Node crypto.verify (oracle/node_xcheck.js, OpenSSL-backed, hashes the message itself) over
  every vector whose message is committed (tests/golden/p256_messages.bin).

The reference has no vectors for this path and Go (whose crypto/ecdsa.Verify the plugin would
call) is absent here; these independent implementations are what pin the
oracle. A drift in the oracle, the fixtures or the checkers fails here. No GPU."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, ROOT, split_fields

XCHECK = os.path.join(ROOT, "oracle", "openssl_xcheck")
NODE_XCHECK = os.path.join(ROOT, "oracle", "node_xcheck.js")


def _openssl_xcheck():
    if not os.path.exists(XCHECK):
        if not os.path.exists("/usr/include/openssl/ecdsa.h"):
            pytest.skip("OpenSSL headers absent: cannot build oracle/openssl_xcheck")
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "openssl_xcheck"], check=True)
    return XCHECK


def test_openssl_agrees_with_every_fixture_verdict(p256_vectors):
    f, exp, cat, names = p256_vectors
    out = subprocess.run([_openssl_xcheck()], input=np.ascontiguousarray(f).tobytes(), capture_output=True,
                         check=True, timeout=300).stdout
    got = np.frombuffer(out, dtype=np.uint8)
    assert got.shape == exp.shape
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, [(int(i), names[cat[i]]) for i in bad[:10]]
    # and the C oracle on the same records (the restatement the GPU tests compare against)
    assert np.array_equal(oracle.verify_batch(*split_fields(f)), got)


def test_openssl_agrees_with_crafted_exceptional_fixture():
    """tests/golden/p256_crafted.bin (keys crafted so the engine's lean additions meet
    P + P or P + (-P) at a chosen step): OpenSSL's verdicts equal the fixture's."""
    raw = np.fromfile(os.path.join(GOLDEN, "p256_crafted.bin"), dtype=np.uint8).reshape(-1, 162)
    out = subprocess.run([_openssl_xcheck()], input=np.ascontiguousarray(raw[:, :160]).tobytes(),
                         capture_output=True, check=True, timeout=300).stdout
    assert np.array_equal(np.frombuffer(out, dtype=np.uint8), raw[:, 160])


def test_openssl_agrees_with_oracle_on_random_corruptions():
    """Fresh seeded tuples (not in the fixtures): oracle-signed, then corrupted bytewise; the
    oracle and OpenSSL must agree on every one."""
    import hashlib
    rng = np.random.default_rng(2024)
    n = 400
    recs = np.zeros((n, 160), dtype=np.uint8)
    for i in range(n):
        d = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        k = int.from_bytes(rng.bytes(32), "big") % oracle.N or 1
        e = hashlib.sha256(rng.bytes(40)).digest()
        qx, qy = oracle.pubkey(d)
        r, s = oracle.sign(d, k, e)
        rec = bytearray(e + r + s + qx + qy)
        if i % 2:
            rec[int(rng.integers(0, 160))] ^= 1 << int(rng.integers(0, 8))
        recs[i] = np.frombuffer(bytes(rec), dtype=np.uint8)
    out = subprocess.run([_openssl_xcheck()], input=recs.tobytes(), capture_output=True, check=True,
                         timeout=120).stdout
    got = np.frombuffer(out, dtype=np.uint8)
    want = oracle.verify_batch(*split_fields(recs))
    assert np.array_equal(got, want)
    assert 0 < want.sum() < n


def test_node_agrees_with_fixture_verdicts_for_known_messages(p256_vectors):
    node = shutil.which("node")
    if not node:
        pytest.skip("node absent")
    f, exp, cat, names = p256_vectors
    raw = open(os.path.join(GOLDEN, "p256_messages.bin"), "rb").read()
    lines, idx = [], []
    pos = 0
    while pos < len(raw):
        i, ln = struct.unpack_from("<II", raw, pos)
        msg = raw[pos + 8:pos + 8 + ln]
        pos += 8 + ln
        rec = bytes(f[i])
        lines.append('{"msg":"%s","r":"%s","s":"%s","qx":"%s","qy":"%s"}' % (
            msg.hex(), rec[32:64].hex(), rec[64:96].hex(), rec[96:128].hex(), rec[128:160].hex()))
        idx.append(i)
    res = subprocess.run([node, NODE_XCHECK], input="\n".join(lines).encode(), capture_output=True,
                         check=True, timeout=300)
    got = np.array([int(x) for x in res.stdout.decode().split()], dtype=np.uint8)
    assert len(got) == len(idx) > 1000
    idx = np.array(idx)
    bad = np.nonzero(got != exp[idx])[0]
    assert len(bad) == 0, [(int(idx[i]), names[cat[idx[i]]]) for i in bad[:10]]
