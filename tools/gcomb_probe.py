"""Comb-width A/B helper: time the generic comb table's first-use build and a 10k-tuple latency
call (pair kernel), and check both against the oracle-derived fixture verdicts.
Run with SBFT_GV_LIB pointing at a tools/variants build (tools/gpu_gcomb_ab.sh)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import gpuverify  # noqa: E402
from tests.conftest import load_p256_vectors, split_fields  # noqa: E402


def main():
    eng = gpuverify.GpuVerifier()
    fields, expect, _, _ = load_p256_vectors()
    d, r, s, qx, qy = split_fields(fields)
    v = {"digest": d, "r": r, "s": s, "qx": qx, "qy": qy, "ok": expect}
    t0 = time.perf_counter()
    ok = eng.verify(v["digest"][:1], v["r"][:1], v["s"][:1], v["qx"][:1], v["qy"][:1])
    build_s = time.perf_counter() - t0
    ok = eng.verify(v["digest"], v["r"], v["s"], v["qx"], v["qy"])
    bad = int(np.count_nonzero(ok != v["ok"]))
    reps = np.tile(np.arange(len(v["ok"])), 10000 // len(v["ok"]) + 1)[:10000]
    args = [v[k][reps] for k in ("digest", "r", "s", "qx", "qy")]
    ts = []
    for _ in range(30):
        t = time.perf_counter()
        ok = eng.verify(*args)
        ts.append(time.perf_counter() - t)
    bad += int(np.count_nonzero(ok != v["ok"][reps]))
    print(json.dumps({"lib": os.path.basename(gpuverify.LIB_PATH), "first_call_s": round(build_s, 3),
                      "verify_10k_p50_ms": round(1e3 * float(np.median(ts)), 3), "mismatches": bad}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
