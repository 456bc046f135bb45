"""Quick latency probe of the registered-key path: 67 signatures (n=100 commit quorum) and
other batch sizes through sbft_gv_verify_p256_keyed / sbft_gv_sha256_verify_p256_keyed."""
import hashlib
import json
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (test infrastructure: signs the probe's inputs)
from smartbft_amd import GpuVerifier  # noqa: E402

N = oracle.N
gv = GpuVerifier(device_mask=1)
rng = random.Random(1)
keys = [rng.randrange(1, N) for _ in range(100)]
pubs = [oracle.pubkey(d) for d in keys]
t0 = time.perf_counter()
kid = [gv.register_key(*p) for p in pubs]
reg_ms = (time.perf_counter() - t0) * 1e3 / len(pubs)
out = {"register_ms_per_key": round(reg_ms, 3)}
for n in (1, 67, 256, 1024, 4096):
    rows, msgs, ids = [], [], []
    for i in range(n):
        j = i % 100
        m = rng.randbytes(128)
        e = hashlib.sha256(m).digest()
        r, s = oracle.sign(keys[j], rng.randrange(1, N), e)
        rows.append(e + r + s)
        msgs.append(m)
        ids.append(kid[j])
    f = np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(n, 96)
    d, r, s = f[:, :32], f[:, 32:64], f[:, 64:96]
    ids = np.array(ids, dtype=np.uint32)
    assert gv.verify_keyed(d, r, s, ids).all()
    ts = []
    for _ in range(100):
        t0 = time.perf_counter()
        gv.verify_keyed(d, r, s, ids)
        ts.append(time.perf_counter() - t0)
    ln = np.full(n, 128, dtype=np.uint32)
    off = (np.arange(n, dtype=np.uint64) * 128)
    blob = np.frombuffer(b"".join(msgs), dtype=np.uint8)
    assert gv.sha256_verify_keyed(blob, off, ln, r, s, ids).all()
    th = []
    for _ in range(100):
        t0 = time.perf_counter()
        gv.sha256_verify_keyed(blob, off, ln, r, s, ids)
        th.append(time.perf_counter() - t0)
    out[f"n{n}"] = {"digest_p50_us": round(float(np.median(ts)) * 1e6, 1),
                    "hash_p50_us": round(float(np.median(th)) * 1e6, 1),
                    "verifies_per_s": round(n / float(np.median(ts)))}
print(json.dumps(out))
