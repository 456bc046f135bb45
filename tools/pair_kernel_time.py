"""The pair kernel (p256_verify_small_kernel<2>) on 20,000 tiled golden vectors, 6 calls, checked against
the fixtures (for rocprofv3 --kernel-trace --stats A/Bs of the pair kernel)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smartbft_amd import gpuverify  # noqa: E402

raw = np.fromfile(os.path.join(ROOT, "tests", "golden", "p256_vectors.bin"), dtype=np.uint8).reshape(-1, 162)
idx = np.arange(20_000) % len(raw)
cols = [np.ascontiguousarray(raw[idx, 32 * k:32 * k + 32]) for k in range(5)]
gv = gpuverify.GpuVerifier(device_mask=1)
for _ in range(6):
    got = gv.verify_kernel(gpuverify.KERNEL_PAIR, *cols)
    assert np.array_equal(got, raw[idx, 160]), int((got != raw[idx, 160]).sum())
gv.close()
print("ok")
