"""SHA-256 kernel A/B on BASELINE config 5's payloads (1-64 KiB, 2M messages, ~70 GB in HBM):
kernel-time GB/s of the variant selected by SBFT_SHA_VARIANT (0 per-lane loads, 1 / 2 the
LDS-staged kernel with C = 1 / 2 blocks per step), digests checked against hashlib on a sample
and against variant-independent properties (index order == permuted order)."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import GpuVerifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_097_152
gv = GpuVerifier(device_mask=1)
dev = torch.device("cuda:0")
rng = np.random.default_rng(5)
ln = rng.integers(1024, 65537, size=n).astype(np.uint32)
off = np.concatenate([[0], np.cumsum(ln.astype(np.uint64))[:-1]]).astype(np.uint64)
total = int(ln.astype(np.uint64).sum())
g = torch.Generator(device=dev)
g.manual_seed(5)
blob = torch.randint(0, 256, (total + 256,), dtype=torch.uint8, device=dev, generator=g)
d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
dig = torch.empty((n, 32), dtype=torch.uint8, device=dev)
gv.sha256_dev(blob, d_off, d_len, dig)
torch.cuda.synchronize()
for i in list(range(0, n, max(1, n // 50))) + [n - 1]:
    m = blob[int(off[i]):int(off[i]) + int(ln[i])].cpu().numpy().tobytes()
    assert dig[i].cpu().numpy().tobytes() == hashlib.sha256(m).digest(), i
order = torch.from_numpy(np.random.default_rng(1).permutation(n).astype(np.int32)).to(dev)
dig2 = torch.empty_like(dig)
gv.sha256_dev(blob, d_off, d_len, dig2, d_order=order)
torch.cuda.synchronize()
assert torch.equal(dig, dig2)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
e0.record()
for _ in range(reps):
    gv.sha256_dev(blob, d_off, d_len, dig, check=False)
e1.record()
torch.cuda.synchronize()
sec = e0.elapsed_time(e1) / 1e3 / reps
print(json.dumps({"variant": os.environ.get("SBFT_SHA_VARIANT", "1"), "messages": n, "bytes": total,
                  "ms": round(sec * 1e3, 3), "GBs": round((total + 32 * n) / sec / 1e9, 1)}))
