"""Streamed config-5 hash+verify (sbft_gv_sha256_verify_p256_stream) from pageable and pinned
host memory at several window sizes: GB/s per setting (diagnostics for DESIGN.md)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from smartbft_amd import GpuVerifier, PinnedArray  # noqa: E402
from smartbft_amd.workload import make_config5  # noqa: E402

gv = GpuVerifier(device_mask=1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
c5 = make_config5(gv, n)
span = int(c5.off[-1]) + int(c5.ln[-1])
hb = c5.blob[:span].cpu().numpy()
cols = [t.cpu().numpy() for t in (c5.r, c5.s, c5.qx, c5.qy)]
want = (~c5.corrupted).to(torch.uint8).cpu().numpy()
pin = PinnedArray(hb.shape)
pin.array[:] = hb
out = {}
for name, b in (("pageable", hb), ("pinned", pin.array)):
    for wmb in (16, 64, 256, 1024):
        gv.sha256_verify_stream(b, c5.off, c5.ln, *cols, window_bytes=wmb << 20)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ok = gv.sha256_verify_stream(b, c5.off, c5.ln, *cols, window_bytes=wmb << 20)
            ts.append(time.perf_counter() - t0)
        assert np.array_equal(ok, want)
        out[f"{name}_{wmb}MiB"] = round(span / min(ts) / 1e9, 1)
t0 = time.perf_counter()
d = torch.from_numpy(pin.array).to("cuda:0", non_blocking=False)
torch.cuda.synchronize()
out["plain_pinned_h2d_GBs"] = round(span / (time.perf_counter() - t0) / 1e9, 1)
pin.close()
print(json.dumps(out))
