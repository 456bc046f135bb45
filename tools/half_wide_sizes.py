"""The half-size-scalar kernel at per-device share sizes: four lanes per tuple (pairs, p256_verify_half_kernel<
false, false>) against its wide form (a quad per ladder, <false, true>), VERDICT r05 #1.

Usage: python tools/half_wide_sizes.py N [REPS] -- one size per process (run it under rocprofv3
--kernel-trace --stats for the committed per-kernel averages). Config-2-style tuples (distinct keys,
~10% corrupted by the bench's seeded kinds), device-resident; HIP events around the verify kernel
(sbft_gv_kernel_timing), the two kernels interleaved call by call; verdicts of both checked against
the oracle (the checker only). Prints one JSON line."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from smartbft_amd import GpuVerifier  # noqa: E402
from smartbft_amd.workload import make_workload  # noqa: E402


def main():
    n = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    gvs = {"half4": GpuVerifier(device_mask=1, halfq_max=-1), "wide": GpuVerifier(device_mask=1, halfq_max=1 << 30)}
    w = make_workload(gvs["half4"], n)
    want = oracle.verify_batch(*w.host_fields())
    dev = w.digest.device
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    out = {"n": n, "accepts": int(want.sum())}
    times = {k: [] for k in gvs}
    for gv in gvs.values():
        for _ in range(3):
            gv.verify_dev(w.digest, w.r, w.s, w.qx, w.qy, ok)
        torch.cuda.synchronize(dev)
        gv.kernel_timing(True)
        gv.kernel_time()
    for _ in range(reps):
        for name, gv in gvs.items():
            ok.zero_()
            gv.verify_dev(w.digest, w.r, w.s, w.qx, w.qy, ok)
            torch.cuda.synchronize(dev)
            cnt, ms = gv.kernel_time()
            assert cnt == 1, cnt
            times[name].append(ms * 1e3)
            got = ok.cpu().numpy()
            if not np.array_equal(got, want):
                raise SystemExit(f"{name} n={n}: {int((got != want).sum())} verdicts differ from the oracle")
    for name, t in times.items():
        out[f"{name}_us_median"] = round(statistics.median(t), 1)
        out[f"{name}_us_min"] = round(min(t), 1)
    out["wide_vs_half4"] = round(out["wide_us_median"] / out["half4_us_median"], 4)
    print(json.dumps(out), flush=True)
    for gv in gvs.values():
        gv.close()


if __name__ == "__main__":
    main()
