"""Verify-pipeline latency by batch size for the two kernels (development aid, not the bench):
the one-lane throughput kernel (pair_max = -1) vs the two-lanes-per-tuple latency kernel.
Device-resident bench-workload tuples; p50 over 20 calls of wall time around verify_dev +
synchronize."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from smartbft_amd import GpuVerifier
from smartbft_amd.workload import make_workload

check = "--no-check" not in sys.argv
sizes = [int(x) for x in sys.argv[1:] if not x.startswith("--")] or [64, 1000, 4096, 10000, 20000, 32768, 49152, 65536, 131072]
g = {"lane": GpuVerifier(device_mask=1, pair_max=-1, half_max=-1),
     "pair": GpuVerifier(device_mask=1, pair_max=1 << 30, half_max=-1),
     "half": GpuVerifier(device_mask=1, half_max=1 << 30)}
wl = make_workload(g["lane"], max(sizes))
dev = torch.device("cuda:0")
for n in sizes:
    f = [x[:n] for x in (wl.digest, wl.r, wl.s, wl.qx, wl.qy)]
    row = {"n": n}
    ref = None
    for k, gv in g.items():
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        gv.verify_dev(*f, ok)
        torch.cuda.synchronize()
        got = ok.cpu().numpy()
        if ref is None:
            ref = got
        assert not check or np.array_equal(got, ref), f"kernels disagree at n={n}"
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            gv.verify_dev(*f, ok)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        row[k + "_ms"] = round(sorted(ts)[10] * 1e3, 3)
    row["accepts"] = int(ref.sum())
    print(row, flush=True)
