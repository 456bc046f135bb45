"""A split VerifyProposal's host-side cost on one GPU: a proposal of N requests through a context
with K slots (the multi-device split path with min_split = 1, a share of N / K per slot, each slot
standing in for a GPU; shares small enough that the K kernels do not contend for CUs) against a
proposal of N / K requests on a one-slot context -- what one device of a K-GPU split would do
alone. p50 / p99 of the C-ABI call, interleaved. Usage: python tools/split_probe.py N K CALLS"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from smartbft_amd import GpuVerifier, plugin  # noqa: E402
from smartbft_amd.workload import make_signed_requests  # noqa: E402


def main():
    n, k, calls = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    gvs = {"one_slot_share": GpuVerifier(device_mask=1),
           f"{k}_slots_split": GpuVerifier(device_mask=1, slots_per_device=k, min_split=1)}
    reqs = make_signed_requests(gvs["one_slot_share"], n, start=777)
    props = {"one_slot_share": plugin.Proposal(plugin.encode_payload(reqs[:n // k]), b"h", b"m", 1),
             f"{k}_slots_split": plugin.Proposal(plugin.encode_payload(reqs), b"h", b"m", 1)}
    keep = []
    cprops = {name: plugin._prop(p, keep) for name, p in props.items()}
    cap = 64 + len(props[f"{k}_slots_split"].Payload)
    infos = ctypes.create_string_buffer(cap)
    count, bad = ctypes.c_size_t(), ctypes.c_int64()
    err = ctypes.create_string_buffer(512)
    vs = {name: plugin.Verifier(g, 1) for name, g in gvs.items()}
    sizes = {"one_slot_share": n // k, f"{k}_slots_split": n}
    ts = {name: [] for name in vs}
    for name, v in vs.items():
        assert len(v.VerifyProposal(props[name])) == sizes[name]
        for _ in range(5):
            v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cprops[name]), infos, cap, ctypes.byref(count),
                                              ctypes.byref(bad), err, 512)
    for _ in range(calls):
        for name, v in vs.items():
            t0 = time.perf_counter()
            rc = v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cprops[name]), infos, cap, ctypes.byref(count),
                                                   ctypes.byref(bad), err, 512)
            ts[name].append((time.perf_counter() - t0) * 1e3)
            assert rc == 0 and count.value == sizes[name], (name, rc, err.value)
    out = {"n": n, "slots": k}
    for name, t in ts.items():
        out[name] = {"p50_ms": round(float(np.percentile(t, 50)), 4), "p99_ms": round(float(np.percentile(t, 99)), 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
