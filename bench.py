#!/usr/bin/env python3
"""bench.py — P-256 ECDSA verifies/s on MI355X (BASELINE.json metric, config 2).

A "step" is one launch of the verify hot path over one batch of device-resident
synthetic tuples: 1,000,000 per GPU (32-byte SHA-256 digests, distinct key per tuple,
~10% corrupted; smartbft_amd/workload.py). Multi-GPU (weak scaling): one process per GPU,
rank r owns tuples [r*N, (r+1)*N) — no data-path collective (there is nothing to reduce;
SURVEY.md 8(e)); a barrier brackets the timed region and the time is the max over ranks.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--n TUPLES]
  N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
Prints ONE JSON line on rank 0 (fields: see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Roofline accounting: algorithmic work per verify = 4,096 F_p-multiplication
# equivalents x 64 32x32->64 products; peak = measured rate of the product
# instruction the kernel issues, v_mad_i64_i32, on MI355X (tools/valu_peak.hip: 38.0 T
# lane-ops/s; profiles/r01g_valu_peak.txt).
PRODUCTS_PER_VERIFY = 262_144
MAD_PEAK_T = 38.0
VALU_ISSUE_PEAK_T = 39.3  # 1,024 SIMDs x 64 lanes / 4 cycles x 2.4 GHz (64-bit ops and mads)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5,
                    help="untimed steps: the first full-size dispatches after start-up run ~15%% slower")
    ap.add_argument("--n", type=int, default=1_000_000, help="tuples per GPU")
    ap.add_argument("--cpu-sample", type=int, default=131072)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the CPU baselines (0 = every core this job may use: "
                         "sched_getaffinity capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip configs 3/4 latency")
    ap.add_argument("--latency-calls", type=int, default=200)
    ap.add_argument("--no-sha", action="store_true", help="skip the config-5 hashing measurement")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-buffer rate")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the multi-stream sustained rate (its concurrent launches would mix into a profile)")
    ap.add_argument("--sha-messages", type=int, default=2_097_152,
                    help="config 5: 16M requests over 8 GPUs = 2M per GPU (~68 GB of payload in HBM)")
    ap.add_argument("--dist-backend", default="gloo", choices=["gloo", "nccl"],
                    help="process group for the barrier and the max-time reduction, the only "
                         "cross-rank traffic (no data-path collective: SURVEY.md 8(e)). gloo (host "
                         "TCP, default) keeps RCCL out of the process entirely, as north_star has "
                         "it; nccl (= RCCL) is kept for A/B only")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "pmc_verify_latest.json"))
    ap.add_argument("--logical-slots", type=int, default=1,
                    help="rehearsal of the multi-device path on one GPU: K engine slots on the device "
                         "(sbft_gv_opts.slots_per_device), each with its own N-tuple workload and stream, "
                         "standing in for K GPUs (the step launches all K; the host-buffer rate splits "
                         "one call over the K slots). Not a scaling measurement: K slots share one GPU")
    ap.add_argument("--split", type=int, default=1,
                    help="A/B tool: cut each device's step into S equal sub-batches (contiguous slices)")
    ap.add_argument("--split-streams", type=int, default=1,
                    help="A/B tool: run the sub-batches over this many streams, forked from and joined "
                         "back into the step's stream every step")
    return ap.parse_args()


def host_cores() -> dict:
    """The host cores this job may use: the affinity mask, capped by the cgroup CPU quota
    (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us) when one is set."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    used = aff if quota is None else max(1, min(aff, int(quota)))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"affinity": aff, "cgroup_quota_cores": quota, "cores_available": used, "cpu": model}


def _openssl_rate(tuples: np.ndarray, threads: int, seconds: float, runs: int = 5):
    exe = os.path.join(ROOT, "oracle", "openssl_bench")
    if not os.path.exists(exe):
        return None
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as tf:
        tf.write(tuples.tobytes())
        path = tf.name
    try:
        out = subprocess.run([exe, path, str(threads), str(seconds), str(runs)], capture_output=True, text=True,
                             timeout=300)
        if out.returncode != 0:
            return None
        return json.loads(out.stdout.strip().splitlines()[-1])
    finally:
        os.unlink(path)


def _mapped(pattern: str) -> list:
    """Files of this process's mappings whose path contains `pattern`."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if pattern in ln and "/" in ln})
    except OSError:
        return []


def _harness(*args, timeout=600, tool="latency_harness"):
    """tools/latency_harness (per-call latency of configs 3 and 4, GPU and CPU), or another tools/
    measurement binary; None if absent."""
    exe = os.path.join(ROOT, "tools", tool)
    if not os.path.exists(exe):
        return None
    out = subprocess.run([exe, *[str(a) for a in args]], capture_output=True, text=True, timeout=timeout)
    if out.returncode != 0:
        raise RuntimeError(f"{tool} {args}: rc={out.returncode} {out.stderr[-500:]}")
    return json.loads(out.stdout.strip().splitlines()[-1])


def cpu_baseline(wl, sample: int, threads: int):
    """The CPU baselines, timed on host cores over a bounded sample of the same workload.
      - baseline: OpenSSL ECDSA_do_verify (ecp_nistz256 assembly) on every core this job may
        use, and on one core: the stand-in for Go's assembly-optimised P-256 that north_star
        names (Go is absent on both machines, so it is labelled a fallback, as SURVEY 8(d)
        prescribes). openssl_bench times only tuples whose key decodes: a Go plugin rejects an
        undecodable key before any arithmetic.
      - oracle: oracle/p256_oracle.c, the deliberately plain C restatement the tests check
        against, on the same threads (a checker, not a competitor); its verdicts of the sample
        are a free parity check of the bench run.
    Returns (baseline or None, oracle, oracle verdicts)."""
    import oracle  # test infrastructure: the cpu_baseline leg is one of its allowed users
    sample = min(sample, wl.n)
    f = wl.host_fields(0, sample)
    oracle.lib()
    t0 = time.perf_counter()
    ok_cpu = oracle.verify_batch(*f, nthreads=threads)
    dt = time.perf_counter() - t0
    hc = host_cores()
    port = {"value": round(sample / dt, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
            "sample": f"first {sample} tuples of the bench workload, oracle/p256_oracle.c "
                      f"(C restatement of Go crypto/ecdsa.Verify), {threads} pthreads, {dt:.2f} s",
            "cpu": hc["cpu"], "cores_available": hc["cores_available"]}
    base = None
    tuples = np.concatenate(f, axis=1)
    # 1 warm-up + 5 timed runs of >= 2 s each, the median reported
    one = _openssl_rate(tuples, 1, 2.0, 5)
    allc = _openssl_rate(tuples, threads, 2.0, 5)
    if allc:
        base = {"value": allc["verifies_per_s"], "unit": "verifies/s", "cores": threads,
                "kind": "port (fallback: OpenSSL 3.0.2 ECDSA_do_verify, ecp_nistz256 assembly; not Go, "
                        "which is absent here)",
                "sample": f"first {sample} tuples of the bench workload, cycled: 1 warm-up + "
                          f"{allc.get('runs', 1)} timed runs of >= 2 s on {threads} threads, median "
                          f"(runs: {allc.get('runs_per_s')})",
                "single_core": one["verifies_per_s"] if one else None,
                "single_core_runs": one.get("runs_per_s") if one else None,
                "cpu": hc["cpu"], "cores_available": hc["cores_available"], "host": hc}
    return base, port, ok_cpu


def pipelined(gv, wl, dev, steps: int, streams: int = 4):
    """Sustained rate with several batches in flight: the same 1M device-resident tuples cut into
    `streams` contiguous sub-batches, each verified over and over on a stream of its own with no
    join between passes (a serving loop with that many launches in flight). A single launch ends
    with a tail (the last resident round's waves finish at different times, then the fix-up and
    s^-1 kernels run on an idle GPU); here other streams' work fills it. Reported beside
    `value` (one launch per step, steps serialised on one stream), never as it."""
    n = wl.n
    sts = [torch.cuda.Stream(device=dev) for _ in range(streams)]
    oks = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(streams)]

    def run(k):
        for i, st in enumerate(sts):
            lo, hi = n * i // streams, n * (i + 1) // streams
            for _ in range(k):
                gv.verify_dev(wl.digest[lo:hi], wl.r[lo:hi], wl.s[lo:hi], wl.qx[lo:hi], wl.qy[lo:hi], oks[i][lo:hi], st)

    run(2)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    want = (~wl.corrupted).to(torch.uint8)
    mism = 0
    for i in range(streams):
        lo, hi = n * i // streams, n * (i + 1) // streams
        mism += int((oks[i][lo:hi] != want[lo:hi]).sum())
    return {"value": round(n * steps / dt, 1), "unit": "verifies/s", "streams": streams, "passes": steps,
            "ms_per_pass": round(dt / steps * 1e3, 4), "mismatches": mism,
            "path": f"sbft_gv_verify_p256_dev, {streams} streams x {n // streams} tuples, no join between passes"}


def host_path(gv, wls, dev, reps: int = 3):
    """PCIe-inclusive rate of the host-buffer C ABI (sbft_gv_verify_p256: the call a cgo
    plugin makes with Go-heap tuples): H2D of 160 B/tuple + verify pipeline + D2H of verdicts,
    on the same tuples (every device's; one call, split over the context's devices, each
    device's share on a host thread of its own). Reported beside `value`, never as it."""
    f = [np.ascontiguousarray(np.concatenate(parts)) for parts in zip(*[w.host_fields(0, w.n) for w in wls])]
    n = len(f[0])
    ok = gv.verify(*f)  # warm-up (workspace growth)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ok = gv.verify(*f)
        ts.append(time.perf_counter() - t0)
    want = np.concatenate([(~w.corrupted).to(torch.uint8).cpu().numpy() for w in wls])
    best = min(ts)
    out = {"value": round(n / best, 1), "unit": "verifies/s", "ms": round(best * 1e3, 3),
           "mismatches": int((ok != want).sum()), "devices": gv.device_count,
           "path": "sbft_gv_verify_p256, pageable host buffers, H2D + kernels + D2H"}
    # the same call with the inputs in sbft_gv_host_alloc memory: H2D of later sub-batches
    # overlaps the kernels of earlier ones (gpuverify.cpp enqueue_verify_piped)
    from smartbft_amd import PinnedArray
    pins = [PinnedArray(a.shape) for a in f]
    try:
        for p, a in zip(pins, f):
            p.array[:] = a
        pa = [p.array for p in pins]
        okp = gv.verify(*pa)
        tp = []
        for _ in range(reps):
            t0 = time.perf_counter()
            okp = gv.verify(*pa)
            tp.append(time.perf_counter() - t0)
        bp = min(tp)
        out["pinned"] = {"value": round(n / bp, 1), "unit": "verifies/s", "ms": round(bp * 1e3, 3),
                         "mismatches": int((okp != want).sum()),
                         "path": "sbft_gv_verify_p256, inputs in sbft_gv_host_alloc memory, "
                                 "copy stream overlapped with sub-batch verify launches on two compute streams"}
    finally:
        for p in pins:
            p.close()
    return out


def _pcts(ts):
    ts = np.array(ts) * 1e3
    return round(float(np.percentile(ts, 50)), 3), round(float(np.percentile(ts, 99)), 3)


def split_latency(nd: int, calls: int):
    """BASELINE config 3 as north_star splits it: VerifyProposal over a 10k-request proposal with
    the engine's context over the node's first nd GPUs (host batch split, a share and a stream per
    device, no collective; each share of 10k / nd <= halfq_max runs the wide half kernel), against
    a context on GPU 0 alone, interleaved call by call in the same run. Driven from rank 0 while
    the other ranks wait on a CPU-side barrier, so nothing else runs on their GPUs."""
    import ctypes
    from smartbft_amd import GpuVerifier, plugin
    from smartbft_amd.workload import make_signed_requests
    gvs = {"one_gpu": GpuVerifier(device_mask=1), "split": GpuVerifier(device_mask=(1 << nd) - 1)}
    reqs = make_signed_requests(gvs["one_gpu"], 10_000)
    prop = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
    keep = []
    cprop = plugin._prop(prop, keep)
    cap = 64 + len(prop.Payload)
    infos = ctypes.create_string_buffer(cap)
    count, bad = ctypes.c_size_t(), ctypes.c_int64()
    err = ctypes.create_string_buffer(512)
    vs = {k: plugin.Verifier(g, 1) for k, g in gvs.items()}
    want = vs["one_gpu"].VerifyProposal(prop)
    assert len(want) == 10_000
    ts = {k: [] for k in vs}
    for k, v in vs.items():  # warm-up (staging, mapped buffers, both kernels' first launches)
        assert v.VerifyProposal(prop) == want
        for _ in range(5):
            v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cprop), infos, cap, ctypes.byref(count),
                                              ctypes.byref(bad), err, 512)
    for _ in range(calls):
        for k, v in vs.items():
            t0 = time.perf_counter()
            rc = v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cprop), infos, cap, ctypes.byref(count),
                                                   ctypes.byref(bad), err, 512)
            ts[k].append(time.perf_counter() - t0)
            assert rc == 0 and count.value == 10_000, (k, rc, err.value)
    out = {"devices": nd, "requests": 10_000, "calls": calls, "share": 10_000 // nd,
           "devices_seen": gvs["split"].device_count}
    for k in vs:
        p50, p99 = _pcts(ts[k])
        out[k] = {"p50_ms": p50, "p99_ms": p99}
    out["p50_speedup_vs_one_gpu"] = round(out["one_gpu"]["p50_ms"] / out["split"]["p50_ms"], 3)
    out["path"] = ("sbft_verifier_verify_proposal (C ABI), host buffers; split: one context over GPUs "
                   "0..nd-1, contiguous shares, one stream per device (sbft_gv_plan_split)")
    for v in vs.values():
        v.close()
    for g in gvs.values():
        g.close()
    return out


def _call_kernel_times(v, cprop, infos, cap, count, bad, err, calls: int,
                       kernel: str = "p256_verify_half_kernel<true> (hash on the helper wavefront)"):
    """The VerifyProposal kernel's own time: HIP events around the call's one launch
    (sbft_gv_kernel_timing), over a separate set of calls (the events' cost stays out of the
    timed p50 / p99 above), with the roofline on the throughput kernel's accounting (262,144
    32x32-bit products per verify against the measured v_mad_i64_i32 peak)."""
    import ctypes
    gv = v.gv
    gv.kernel_timing(True)
    gv.kernel_time()
    ks = []
    for _ in range(max(50, calls // 4)):
        rc = v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cprop), infos, cap, ctypes.byref(count),
                                               ctypes.byref(bad), err, 512)
        assert rc == 0, (rc, err.value)
        nl, ms = gv.kernel_time()
        if nl == 1:
            ks.append(ms * 1e3)
    gv.kernel_timing(False)
    if not ks:
        return None
    p50 = float(np.percentile(ks, 50))
    ach = 10_000 * PRODUCTS_PER_VERIFY / (p50 * 1e-6) / 1e12
    return {"name": kernel, "us_p50": round(p50, 1), "us_p99": round(float(np.percentile(ks, 99)), 1),
            "launches": len(ks), "timing": "HIP events around the launch (sbft_gv_kernel_timing)",
            "roofline": {"achieved": round(ach, 3), "peak": MAD_PEAK_T, "frac": round(ach / MAD_PEAK_T, 4),
                         "unit": "T 32x32->64 products/s, 262,144 per verify"}}


def latency_configs(gv, calls: int):
    """BASELINE configs 3 and 4 through the plugin mirror (host buffers, PCIe included):
    VerifyProposal on 10k-request proposals (view.go:555) and a 67-signature commit quorum at
    n = 100 (view.go:631). p50/p99 wall latency per call, timed around the C-ABI call the cgo
    plugin makes (include/sbft_verifier.h) with its arguments prepared once, as
    Go holds them already; the Python wrapper's latency (ctypes marshalling + building Python
    RequestInfo objects) is reported beside it."""
    import ctypes
    from smartbft_amd import plugin
    from smartbft_amd.workload import make_signed_requests
    out = {}
    reqs = make_signed_requests(gv, 10_000)
    prop = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
    v = plugin.Verifier(gv, 1)
    assert len(v.VerifyProposal(prop)) == 10_000
    keep = []
    cprop = plugin._prop(prop, keep)
    cap = 64 + len(prop.Payload)
    infos = ctypes.create_string_buffer(cap)
    count, bad = ctypes.c_size_t(), ctypes.c_int64()
    err = ctypes.create_string_buffer(512)

    def warm(ver):  # the C-ABI call's first uses (mapped buffers, per-thread scratch) stay untimed
        for _ in range(5):
            assert ver.L.sbft_verifier_verify_proposal(ver.h, ctypes.byref(cprop), infos, cap, ctypes.byref(count),
                                                       ctypes.byref(bad), err, 512) == 0

    warm(v)
    ts, tp = [], []
    for _ in range(calls):
        t0 = time.perf_counter()
        rc = v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cprop), infos, cap, ctypes.byref(count),
                                               ctypes.byref(bad), err, 512)
        ts.append(time.perf_counter() - t0)
        assert rc == 0 and count.value == 10_000, (rc, err.value)
    for _ in range(max(10, calls // 10)):
        t0 = time.perf_counter()
        v.VerifyProposal(prop)
        tp.append(time.perf_counter() - t0)
    p50, p99 = _pcts(ts)
    out["verify_proposal_10k"] = {"p50_ms": p50, "p99_ms": p99, "calls": calls, "requests": 10_000,
                                  "verifies_per_s": round(10_000 / (p50 / 1e3)),
                                  "python_wrapper_p50_ms": _pcts(tp)[0],
                                  "path": "sbft_verifier_verify_proposal (C ABI), host buffers, PCIe incl.",
                                  "kernel": _call_kernel_times(v, cprop, infos, cap, count, bad, err, calls)}
    # the same proposals with the 10k client keys registered (sbft_verifier_add_clients): every
    # request takes the keyed comb-table launch (no doublings, one wavefront per signature)
    vr = plugin.Verifier(gv, 1)
    t0 = time.perf_counter()
    vr.add_clients([q[-129:-64] for q in reqs])
    reg_s = time.perf_counter() - t0
    assert vr.VerifyProposal(prop) == v.VerifyProposal(prop)
    warm(vr)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        rc = vr.L.sbft_verifier_verify_proposal(vr.h, ctypes.byref(cprop), infos, cap, ctypes.byref(count),
                                                ctypes.byref(bad), err, 512)
        ts.append(time.perf_counter() - t0)
        assert rc == 0 and count.value == 10_000, (rc, err.value)
    p50, p99 = _pcts(ts)
    out["verify_proposal_10k_registered_clients"] = {
        "p50_ms": p50, "p99_ms": p99, "calls": calls, "requests": 10_000,
        "registration_s": round(reg_s, 2), "client_tables_GB": round(10_000 * 512 * 1024 / 1e9, 2),
        "path": "sbft_verifier_verify_proposal with the clients' keys registered (keyed launch), host buffers",
        "kernel": _call_kernel_times(vr, cprop, infos, cap, count, bad, err, calls,
                                     "p256_verify_keyed_lanes_kernel<true> (hash on a fifth wavefront)")}
    vr.close()
    # where a call's time goes, over all calls and over the calls above p95 (the tail): the
    # engine's SBFT_VP_TRACE split (parse, copy wait, staging, launch, kernel + verdicts) and the
    # kernel's HIP-event time per call (tools/latency_harness proposal-phases, C, no ctypes)
    for reg, key in ((0, "verify_proposal_10k"), (1, "verify_proposal_10k_registered_clients")):
        try:
            ph = _harness("proposal-phases", 10_000, max(200, calls), reg)
        except Exception as e:
            ph = {"error": repr(e)[:300]}
        if ph:
            out[key]["phases"] = ph
    # n = 100 replicas: q = 67 signatures per decision
    import hashlib
    q, f = plugin.compute_quorum(100)
    signers = [plugin.Signer(gv, i, (int.from_bytes(hashlib.sha256(b"n100-%d" % i).digest(), "big") %
                                     0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551).to_bytes(32, "big"))
               for i in range(1, q + 1)]
    for sg in signers:
        v.add_consenter(sg.id, sg.public_key())
    block = plugin.Proposal(b"block-payload" * 100, b"h", b"m", 1)
    sigs = [sg.SignProposal(block, b"") for sg in signers]
    assert v.VerifyConsenterSigs(sigs, block) == [0] * q
    arr = (plugin._Signature * q)(*[plugin._sig(sg, keep) for sg in sigs])
    st = (ctypes.c_int32 * q)()
    cblock = plugin._prop(block, keep)
    # warm-up: small keyed batches rotate over the engine's four zero-copy lanes, and a lane's
    # first call allocates its mapped buffer (~0.3-0.6 ms): three first calls inside 200 timed
    # ones were the 0.34-0.65 ms p99 of rounds 2-3 (the C harness warms up, hence its 0.065)
    for _ in range(8):
        assert v.L.sbft_verifier_verify_consenter_sigs(v.h, arr, q, ctypes.byref(cblock), st) == 0
    ts, tp = [], []
    for _ in range(calls):
        t0 = time.perf_counter()
        rc = v.L.sbft_verifier_verify_consenter_sigs(v.h, arr, q, ctypes.byref(cblock), st)
        ts.append(time.perf_counter() - t0)
        assert rc == 0 and list(st) == [0] * q
    for _ in range(max(10, calls // 10)):
        t0 = time.perf_counter()
        v.VerifyConsenterSigs(sigs, block)
        tp.append(time.perf_counter() - t0)
    p50, p99 = _pcts(ts)
    out["commit_quorum_n100"] = {"p50_ms": p50, "p99_ms": p99, "calls": calls, "signatures": q,
                                 "python_wrapper_p50_ms": _pcts(tp)[0],
                                 "path": "sbft_verifier_verify_consenter_sigs (C ABI), host buffers"}
    # the same hook timed in C (no ctypes), 8 proposals in rotation (the digest memo misses)
    qb = _harness("quorum-batch", q, calls)
    if qb:
        assert qb["wrong_verdicts"] == 0
        out["commit_quorum_n100"]["c_harness"] = qb
    # SignProposal's signing (view.go:481), one message at a time: the GPU signer against
    # OpenSSL ECDSA_do_sign on one core
    sg = _harness("sign", calls)
    if sg:
        assert sg["failures"] == 0
        out["sign_one"] = sg
    # the unmodified library: 66 goroutines (view.go:537-541), one VerifyConsenterSig each
    # (:834), released together per decision (tools/latency_harness quorum-gpu); stock = one
    # launch per call, coalesced = sbft_verifier_coalesce_consenter_sigs(66, 50 us)
    # the patched processCommits (go/patches/internal_bft_commits.patch): 67 votes arrive per
    # decision, the collector hands them to one call once 66 can complete the quorum, and votes
    # arriving while it is in flight to a second, overlapped one (a decision with a bad vote);
    # latency = release -> 66 valid votes
    hook = _harness("quorum-hook", 67, 66, calls, 2)
    if hook:
        assert hook["wrong_verdicts"] == 0
        out["commit_quorum_n100_hook"] = dict(hook, path="sbft_verifier_verify_consenter_sigs from the collector "
                                                         "as votes arrive (processCommits batch hook, 2 in flight)")
    # pipelined decisions (config 4): 2 consensus instances deciding back to back on the node
    # (prev-commit batch of 67, then 66 arriving votes each); GPU (patched library) against
    # OpenSSL (stock library: serial prev-commit loop, a goroutine per vote) on the same cores.
    # Votes are delivered (and, on the CPU side, verified) by host_cores / 2 threads per channel,
    # as the Go runtime runs goroutines on GOMAXPROCS threads; the View blocks while it waits
    # (round 5; round 4 ran a thread per vote and spinning waits: its CPU per decision was the
    # harness's, profiles/r05c_config4_ab.txt). engine_call_cpu_ms_per_decision is the CPU time
    # spent inside the engine's calls alone.
    # Two CPU legs: "cpu_openssl_batched" runs the same patched call sequence as
    # the GPU leg (the prev-commit hook's VerifyConsenterSigs spreads the 67 signatures over the
    # channel's share of the cores), the fair comparison; "cpu_openssl_stock" is the unmodified
    # library, whose prev-commit loop verifies serially on the View goroutine.
    pipe = {b: _harness("quorum-pipe", 2, max(100, calls), b) for b in ("gpu", "cpu-batched", "cpu")}
    if pipe["gpu"] and pipe["cpu"] and pipe["cpu-batched"]:
        assert all(pipe[b]["wrong_verdicts"] == 0 for b in pipe)
        out["commit_quorum_n100_pipelined"] = {
            "gpu": pipe["gpu"],
            "cpu_openssl_batched": dict(pipe["cpu-batched"], label="patched library, CPU VerifyConsenterSigs "
                                        "over the cores (the GPU leg's call sequence)"),
            "cpu_openssl_stock": dict(pipe["cpu"], label="stock library (serial prev-commit loop)"),
            "decisions_per_s_vs_cpu": round(pipe["gpu"]["decisions_per_s"] / pipe["cpu-batched"]["decisions_per_s"], 2),
            "decisions_per_s_vs_cpu_stock": round(pipe["gpu"]["decisions_per_s"] / pipe["cpu"]["decisions_per_s"], 2),
            "path": "tools/latency_harness quorum-pipe: 2 channels x back-to-back decisions, each = "
                    "verifyPrevCommitSignatures (67) + processCommits (66 of 67 arriving votes); votes "
                    "delivered by host_cores/2 threads per channel, blocking waits; decisions_per_s_vs_cpu "
                    "is against cpu_openssl_batched"}
    stock = _harness("quorum-gpu", 66, calls, 0, 0)
    coal = _harness("quorum-gpu", 66, calls, 66, 50)
    if stock and coal:
        assert stock["wrong_verdicts"] == 0 and coal["wrong_verdicts"] == 0
        out["commit_quorum_n100_concurrent_singles"] = {
            "stock": stock, "coalesced": coal,
            "path": "66 threads, one sbft_verifier_verify_consenter_sig each per decision; every 10th "
                    "decision has one bad vote, whose caller must get its own EVERIFY"}
    return out


def sha_roofline(gbs: float) -> dict:
    """The hash kernel against HBM and against its compute ceiling. SHA-256 on gfx950 is VALU
    bound: its rotates (v_alignbit_b32) and 3-input adds (v_add3_u32) issue at half rate
    (tools/valu_rates), ~1,430 VALU instructions per 64-B block; the ceiling is measured live
    by tools/sha_ceiling (the same compression on register-resident blocks, no memory
    traffic), the best of one and two messages per lane."""
    out = {"bound": "valu", "hbm_peak_GBs": 8000, "frac_of_hbm": round(gbs / 8000, 4)}
    exe = os.path.join(ROOT, "tools", "sha_ceiling")
    if os.path.exists(exe):
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        vals = [float(line.split(" GB/s")[0].split()[-1]) for line in r.stdout.splitlines() if "GB/s" in line]
        if vals:
            ceil = max(vals)
            out.update({"valu_ceiling_GBs": round(ceil, 1), "frac_of_valu_ceiling": round(gbs / ceil, 4),
                        "ceiling_source": "tools/sha_ceiling, this run (register-resident compression)"})
    return out


def sha_config5(gv, dev, n_msgs: int, e2e_msgs: int = 262144):
    """BASELINE config 5 on one GPU: requests with payload lengths uniform in [1 KiB, 64 KiB]
    (seeded; 2M per GPU = the 16M of config 5 over 8 GPUs), each signed under its own key,
    ~10% corrupted (smartbft_amd/workload.py make_config5).
      - hash only: the SHA-256 kernel on the HBM-resident payloads (kernel time);
      - hash + verify: sbft_gv_sha256_verify_p256_dev, digests never leave the GPU (kernel
        time of the SHA + verify launches); parity: verdict == not corrupted, every request;
      - streamed end to end from host memory: sbft_gv_sha256_verify_p256_stream on the first
        e2e_msgs requests (~8.7 GB: the pipeline's fixed ramp -- the first window's copy, the
        last window's serial hashing -- is ~15% of a 2 GB sample and ~4% of this one; config 5's
        530 GB amortises it fully), from pageable and from page-locked memory (PCIe included);
        verdicts equal the device-resident ones."""
    import hashlib
    from smartbft_amd import PinnedArray
    from smartbft_amd.workload import make_config5
    c5 = make_config5(gv, n_msgs, device=dev.index)
    n = c5.n
    stream = torch.cuda.current_stream(dev)
    dig = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    gv.sha256_dev(c5.blob, c5.d_off, c5.d_len, dig, stream)
    torch.cuda.synchronize(dev)
    for i in (0, n // 2, n - 1):
        m = c5.blob[int(c5.off[i]):int(c5.off[i]) + int(c5.ln[i])].cpu().numpy().tobytes()
        assert dig[i].cpu().numpy().tobytes() == hashlib.sha256(m).digest(), i
    # the d_order path (messages taken in a permuted sequence) must give the same digests
    order = torch.flip(torch.arange(n, device=dev, dtype=torch.int32), [0])
    dig2 = torch.empty_like(dig)
    gv.sha256_dev(c5.blob, c5.d_off, c5.d_len, dig2, stream, d_order=order)
    torch.cuda.synchronize(dev)
    assert torch.equal(dig, dig2), "permuted-order SHA-256 differs from index order"
    del dig2, order

    def timed(fn, reps=3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / 1e3 / reps

    nbytes = c5.total + 32 * n
    # offsets validated by the untimed calls above: the timed ones skip the (stream-synchronising)
    # bounds check so that only the kernels are in the event window
    sec_h = timed(lambda: gv.sha256_dev(c5.blob, c5.d_off, c5.d_len, dig, stream, check=False))
    hv = lambda: gv.sha256_verify_dev(c5.blob, c5.d_off, c5.d_len, c5.r, c5.s, c5.qx, c5.qy, ok, dig, stream,
                                      check=False)
    sec_hv = timed(hv)
    want = (~c5.corrupted).to(torch.uint8)
    mism = int((ok != want).sum())
    # streamed from host memory, bounded sample of the same requests
    k = min(n, e2e_msgs)
    span = int(c5.off[k - 1]) + int(c5.ln[k - 1])
    hb = c5.blob[:span].cpu().numpy()
    cols = [t[:k].cpu().numpy() for t in (c5.r, c5.s, c5.qx, c5.qy)]
    want_k = ok[:k].cpu().numpy()
    gv.sha256_verify_stream(hb, c5.off[:k], c5.ln[:k], *cols)  # warm-up (staging growth)
    t0 = time.perf_counter()
    ok_e = gv.sha256_verify_stream(hb, c5.off[:k], c5.ln[:k], *cols)
    e2e = time.perf_counter() - t0
    pin = PinnedArray(hb.shape)
    try:
        pin.array[:] = hb
        gv.sha256_verify_stream(pin.array, c5.off[:k], c5.ln[:k], *cols)
        t0 = time.perf_counter()
        ok_p = gv.sha256_verify_stream(pin.array, c5.off[:k], c5.ln[:k], *cols)
        e2e_p = time.perf_counter() - t0
    finally:
        pin.close()
    e2e_bytes = span + 32 * k
    del hb
    gbs_h, gbs_hv = nbytes / sec_h / 1e9, nbytes / sec_hv / 1e9
    return {"value": round(gbs_h, 1), "unit": "GB/s (payload + digest bytes, kernel time)",
            "messages": n, "payload_bytes": c5.total, "avg_kernel_ms": round(sec_h * 1e3, 3),
            "roofline": sha_roofline(gbs_h),
            "hash_verify": {"value": round(gbs_hv, 1), "unit": "GB/s (payload + digest bytes, kernel time)",
                            "verifies_per_s": round(n / sec_hv, 1), "ms": round(sec_hv * 1e3, 3),
                            "mismatches": mism, "expected_accepts": int(want.sum()),
                            "path": "sbft_gv_sha256_verify_p256_dev: SHA-256 -> verify, digests stay in HBM"},
            "streamed": {"pageable": {"value": round(e2e_bytes / e2e / 1e9, 1), "unit": "GB/s",
                                      "mismatches": int((ok_e != want_k).sum())},
                         "pinned": {"value": round(e2e_bytes / e2e_p / 1e9, 1), "unit": "GB/s",
                                    "mismatches": int((ok_p != want_k).sum())},
                         "messages": k, "bytes": e2e_bytes,
                         "path": "sbft_gv_sha256_verify_p256_stream: 256 MiB windows, 6 in flight per device "
                                 "(H2D of one window || SHA -> verify of earlier ones), PCIe included"}}


def adversarial(gv, dev):
    """Worst case a client can force: every tuple of a batch exceptional inside the lean Shamir
    ladder (crafted R = infinity, P + P / P + (-P) additions; the request format lets the client
    choose Q), so the whole batch is re-verified by the case-split fix-up kernel. Tiled from
    the golden categories r_infinity and shamir_exceptional (tests/golden, data only); verdicts
    checked against the fixtures. A bad proposal triggers complain + sync in the library
    (view.go:386-393), so the cost of rejecting one matters."""
    import json as _json
    raw = np.fromfile(os.path.join(ROOT, "tests", "golden", "p256_vectors.bin"), dtype=np.uint8).reshape(-1, 162)
    cats = _json.load(open(os.path.join(ROOT, "tests", "golden", "p256_categories.json")))["categories"]
    sel = np.isin(raw[:, 161], [cats.index("r_infinity"), cats.index("shamir_exceptional")])
    base = raw[sel]
    # crafted tuples (tests/golden/p256_crafted.bin, data): keys chosen so that the comb or the
    # ladder's last addition meets acc == +-addend at a chosen step -- what a client controlling
    # its own Q, r, s can aim at
    crafted = np.fromfile(os.path.join(ROOT, "tests", "golden", "p256_crafted.bin"), dtype=np.uint8).reshape(-1, 162)
    out = {"base_vectors": int(len(base)), "base_accepts": int(base[:, 160].sum()),
           "crafted_vectors": int(len(crafted))}
    stream = torch.cuda.current_stream(dev)
    for name, src, n in (("all_exceptional", base, 10_000), ("all_exceptional", base, 1_000_000),
                         ("crafted_collisions", crafted, 10_000), ("crafted_collisions", crafted, 1_000_000)):
        t = np.resize(src, (n, 162))
        f = [torch.from_numpy(np.ascontiguousarray(t[:, 32 * k:32 * k + 32])).to(dev) for k in range(5)]
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        run = lambda: gv.verify_dev(*f, ok, stream)
        run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        out[f"{name}_{n}"] = {"ms": round(ms, 3), "verifies_per_s": round(n / ms * 1e3, 1),
                                       "mismatches": int((ok.cpu().numpy() != t[:, 160]).sum())}
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank on the node; a box with fewer devices than ranks (a gloo rehearsal)
        # maps ranks onto its devices round-robin
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    from smartbft_amd import GpuVerifier
    from smartbft_amd.workload import make_workload

    from smartbft_amd.dist import reduce_timing, shard_range

    # devices this process drives: one under torchrun (one process per GPU), or all --gpus of
    # them in one process (the library's in-process multi-device path: one context over N
    # devices, each device's launch enqueued on its own stream, no collective)
    slots = max(1, args.logical_slots)
    if world > 1:
        assert world == args.gpus, f"WORLD_SIZE={world} but --gpus {args.gpus}"
        assert slots == 1, "--logical-slots rehearses the in-process path only"
        devs = [local]
    else:
        avail = torch.cuda.device_count()
        assert args.gpus <= avail, f"--gpus {args.gpus} but {avail} visible devices"
        assert slots == 1 or args.gpus == 1, "--logical-slots needs --gpus 1"
        devs = list(range(args.gpus))
    gv = GpuVerifier(device_mask=sum(1 << d for d in devs), slots_per_device=slots)
    assert gv.device_count == len(devs) * slots
    # the workloads the step launches: one per device, or one per logical slot of the one
    # device, each on a stream of its own
    lanes = devs if slots == 1 else devs * slots
    n = args.n
    wls, oks, streams = [], [], []
    for j, d in enumerate(lanes):
        lo, _ = shard_range(rank * len(lanes) + j, world * len(lanes), n)
        wls.append(make_workload(gv, n, start=lo, device=d))
        oks.append(torch.empty(n, dtype=torch.uint8, device=f"cuda:{d}"))
        streams.append(torch.cuda.current_stream(torch.device(f"cuda:{d}")) if slots == 1
                       else torch.cuda.Stream(device=torch.device(f"cuda:{d}")))
    wl, ok, stream = wls[0], oks[0], streams[0]
    rehearsal = slots > 1

    S, SS = max(1, args.split), max(1, args.split_streams)
    subs = [[torch.cuda.Stream(device=torch.device(f"cuda:{d}")) for _ in range(SS - 1)] for d in lanes]

    def step():
        for j, (w, o, st, d) in enumerate(zip(wls, oks, streams, lanes)):  # asynchronous: every device runs concurrently
            if S == 1:
                gv.verify_dev(w.digest, w.r, w.s, w.qx, w.qy, o, st)
                continue
            # A/B: S sub-batches over SS streams, forked from st and joined back into it
            fork = torch.cuda.Event()
            fork.record(st)
            pool = [st] + subs[j]
            for x in subs[j]:
                x.wait_event(fork)
            for i in range(S):
                lo, hi = n * i // S, n * (i + 1) // S
                gv.verify_dev(w.digest[lo:hi], w.r[lo:hi], w.s[lo:hi], w.qx[lo:hi], w.qy[lo:hi], o[lo:hi],
                              pool[i % SS])
            for x in subs[j]:
                ev = torch.cuda.Event()
                ev.record(x)
                st.wait_event(ev)

    def sync_all():
        for d in devs:
            torch.cuda.synchronize(d)

    for _ in range(args.warmup):
        step()
    sync_all()
    # parity property at full size: verdict == not corrupted, for every tuple
    expect = (~wl.corrupted).to(torch.uint8)
    mismatches = sum(int((o != (~w.corrupted).to(torch.uint8)).sum()) for w, o in zip(wls, oks))

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    # HIP events around the main p256_verify_kernel itself, recorded by the library on the
    # launch stream (roofline.achieved); the torch events above bracket the whole step
    gv.kernel_timing(True)
    gv.kernel_time()
    if world > 1:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    sync_all()
    for st in streams:
        st.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        elapsed, mismatches = reduce_timing(elapsed, mismatches,
                                            device=dev if args.dist_backend == "nccl" else None)
    step_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    avg_step_gpu_ms = sum(step_ms) / len(step_ms)
    launches, kern_total_ms = gv.kernel_time()
    gv.kernel_timing(False)
    assert launches == args.steps * len(lanes) * S, (launches, args.steps)
    avg_kern_s = kern_total_ms / launches / 1e3
    n_gpus = world * len(devs)
    # a CPU-side group for the final wait: ranks other than 0 must not sit in a collective kernel
    # on their GPUs while rank 0 runs config 3 across all of them (split_latency)
    gloo = dist.new_group(backend="gloo") if world > 1 else None

    if rank == 0:
        total = n * world * len(lanes) * args.steps
        value = total / elapsed
        achieved_t = n / S * PRODUCTS_PER_VERIFY / avg_kern_s / 1e12
        traffic = None
        instr_per_verify = None
        if os.path.exists(args.traffic_file):
            try:
                tj = json.load(open(args.traffic_file))
                if tj.get("n") == n:
                    traffic = tj.get("hbm_bytes_per_launch")
                    instr_per_verify = tj.get("valu_instructions_per_verify")
            except (OSError, ValueError):
                traffic = None
        rec = {
            "metric": "P-256 ECDSA verifies/sec",
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32 limbs, int64 accumulators (256-bit field elements as 9 signed 29-bit limbs)",
            "data": "synthetic (on-GPU seeded keys/signatures, ~10% corrupted; smartbft_amd/workload.py)",
            "config": {"workload": "BASELINE config 2: synthetic P-256 verifies, 32-byte SHA-256 digests, "
                                   "distinct key per tuple, 10% corrupted, device-resident",
                       "tuples_per_gpu": n * slots,
                       "parallelism": (f"one process per GPU x{world}" if world > 1 else
                                       f"in-process multi-device x{len(devs)}") + " (no collective)"},
            "roofline": {"bound": "valu", "achieved": round(achieved_t, 3), "peak": MAD_PEAK_T,
                         "unit": "T 32x32->64 products/s (v_mad_i64_i32 issue rate)",
                         "frac": round(achieved_t / MAD_PEAK_T, 4), "traffic": traffic,
                         # rocprofv3 cannot run inside this process: traffic (FETCH_SIZE +
                         # WRITE_SIZE per launch) and valu_issue come from the committed PMC passes
                         # of the same kernel (tools/pmc_summary.py -> --traffic-file), not this run
                         "traffic_source": (os.path.relpath(args.traffic_file, ROOT) +
                                            " (committed rocprofv3 --pmc passes, not this run)") if traffic else None,
                         "kernel": "p256_verify_kernel", "avg_kernel_ms": round(avg_kern_s * 1e3, 4),
                         "kernel_timing": "HIP events around p256_verify_kernel on its launch stream",
                         "step_gpu_ms": round(avg_step_gpu_ms, 4),
                         "step_kernels": "sinv_prep + sinv_totals + verify + fixup",
                         "products_per_verify": PRODUCTS_PER_VERIFY},
            # issued-instruction view of the same kernel: VALU instructions per verify from the
            # committed PMC pass (SQ_INSTS_VALU x 64 / n, profiles/pmc_verify_latest.json) at this
            # run's rate, against the chip's issue capacity (1,024 SIMDs x 64 lanes / 4 cycles at
            # the 2.4 GHz peak clock; the kernel runs at ~2.05 GHz, GRBM_GUI_ACTIVE)
            # wave-instruction slots (SQ_INSTS_VALU x 64 lanes) per tuple, idle lanes of the
            # spread grid's partly filled waves included, against 4 cycles per instruction at the
            # 2.4 GHz peak clock (the chip holds ~2.1-2.2 GHz under this kernel)
            "valu_issue": None if not instr_per_verify else {
                "instr_slots_per_verify": round(instr_per_verify),
                "achieved_T": round(instr_per_verify * n / avg_kern_s / 1e12, 2),
                "peak_T": VALU_ISSUE_PEAK_T, "frac": round(instr_per_verify * n / avg_kern_s / 1e12 / VALU_ISSUE_PEAK_T, 3)},
            "parity": {"full_size_mismatches": mismatches,
                       "expected_accepts": sum(int((~w.corrupted).sum()) for w in wls) * world},
            # the HIP runtime this process's engine ran on: torch (imported first for device
            # memory) brings its own libamdhip64 with the engine's SONAME, so here the engine
            # binds to torch's copy; a deployment (cgo) loads /opt/rocm's. The parity suite on
            # the shipped runtime is tests/test_gpu_runtime.py (a torch-free child process).
            "hip_runtime": _mapped("libamdhip64"),
        }
        if rehearsal:
            # the K slots' launches run concurrently, so a launch's own duration says nothing
            # about the kernel: the roofline of a rehearsal is taken over the whole step
            ach = value * PRODUCTS_PER_VERIFY / 1e12
            rec["roofline"].update({"achieved": round(ach, 3), "frac": round(ach / MAD_PEAK_T, 4),
                                    "kernel_timing": "whole step (K concurrent launches), not one launch"})
            rec["valu_issue"] = None
            # K logical slots on one GPU stand in for K devices: the in-process multi-device
            # code path (per-slot workloads and streams here; the library's host-side split,
            # share offsets and verdict placement in host_buffer_path) runs, but the K slots
            # share one GPU's CUs, so `value` is the one GPU's rate, not a K-GPU one
            rec["metric"] = "P-256 ECDSA verifies/sec (multi-device rehearsal on one GPU)"
            rec["config"]["logical_slots"] = slots
            rec["config"]["parallelism"] = f"in-process, {slots} engine slots on 1 GPU (rehearsal, no scaling claim)"
        if n_gpus == 1 and not rehearsal and not args.no_cpu_baseline:
            cpu_threads = args.cpu_threads or host_cores()["cores_available"]
            base, port, ok_cpu = cpu_baseline(wl, args.cpu_sample, cpu_threads)
            if base:
                rec["cpu_baseline"] = base
                rec["speedup_vs_cpu_baseline"] = round(value / base["value"], 1)
            rec["cpu_oracle"] = port
            rec["parity"]["oracle_sample_mismatches"] = int(
                (ok[:len(ok_cpu)].cpu().numpy() != ok_cpu).sum())
        if n_gpus == 1 and not rehearsal and S == 1 and not args.no_pipelined:
            rec["pipelined"] = pipelined(gv, wl, dev, args.steps)
        if n_gpus == 1 and not rehearsal and S == 1:
            # the same config-2 measurement without torch, on the HIP runtime the engine ships with
            # (tools/config2_harness: engine-generated workload staged once in HBM, the C ABI's
            # device-resident verify on one stream); value above runs on torch's libamdhip64
            try:
                tf = _harness(n, args.steps, args.warmup, tool="config2_harness", timeout=900)
            except Exception as e:  # a side leg must not lose the headline line
                tf = {"error": repr(e)[:300]}
            if tf:
                if "verifies_per_s" in tf:
                    tf["vs_torch_process_value"] = round(tf["verifies_per_s"] / value, 4)
                rec["torch_free_config2"] = tf
        if world == 1 and not args.no_host_path:
            rec["host_buffer_path"] = host_path(gv, wls, dev)
        if n_gpus == 1 and not rehearsal and not args.no_sha:
            rec["sha256_config5"] = sha_config5(gv, dev, args.sha_messages)
        if n_gpus == 1 and not rehearsal and not args.no_latency:
            rec["adversarial"] = adversarial(gv, dev)
            lat = latency_configs(gv, args.latency_calls)
            if not args.no_cpu_baseline:
                # measured CPU latencies of the same calls (tools/latency_harness, OpenSSL):
                # VerifyProposal's 10k verifies over every core this job may use, and the
                # commit quorum's 66 votes with one thread per vote (view.go:537-541), capped
                # at the cores available
                cores = args.cpu_threads or host_cores()["cores_available"]
                pc = _harness("proposal-cpu", 10_000, 20, cores)
                qc = _harness("quorum-cpu", 66, 200, min(66, cores))
                if pc:
                    lat["verify_proposal_10k"]["cpu_openssl"] = pc
                    lat["verify_proposal_10k"]["speedup_p50_vs_cpu"] = round(
                        pc["p50_ms"] / lat["verify_proposal_10k"]["p50_ms"], 1)
                if qc and "commit_quorum_n100_concurrent_singles" in lat:
                    lat["commit_quorum_n100_concurrent_singles"]["cpu_openssl"] = qc
                    lat["commit_quorum_n100_concurrent_singles"]["speedup_p50_vs_cpu"] = round(
                        qc["p50_ms"] / lat["commit_quorum_n100_concurrent_singles"]["coalesced"]["p50_ms"], 1)
                if "commit_quorum_n100_hook" in lat:
                    # the hook's own scenario on the CPU (tools/latency_harness quorum-vote-cpu):
                    # the same 67 votes released per decision, each verified as it arrives, 66
                    # valid close it, every 10th decision with a bad vote -- on the job's cores,
                    # and with one thread per vote as the stock library's goroutines would run:
                    # Go sizes GOMAXPROCS by the affinity mask, not the cgroup quota, so on a box
                    # whose mask is wider than its quota the 67 verifies run on 67 CPUs at once
                    # (bursting past the quota, which a 16-core machine could not do)
                    h = lat["commit_quorum_n100_hook"]
                    calls = h.get("decisions", 200)
                    qv = _harness("quorum-vote-cpu", 67, 66, calls, cores)
                    if qv:
                        h["cpu_openssl"] = qv
                        h["speedup_p50_vs_cpu"] = round(qv["p50_ms"] / h["p50_ms"], 2)
                        h["speedup_p99_vs_cpu"] = round(qv["p99_ms"] / h["p99_ms"], 2)
                    if cores < 67 and host_cores().get("affinity", 0) >= 67:
                        q67 = _harness("quorum-vote-cpu", 67, 66, calls, 67)
                        if q67:
                            q67["note"] = ("67 threads on a %d-CPU affinity mask, %s-core quota"
                                           % (host_cores()["affinity"], host_cores().get("cgroup_quota_cores")))
                            h["cpu_openssl_thread_per_vote"] = q67
                            h["speedup_p50_vs_cpu_thread_per_vote"] = round(q67["p50_ms"] / h["p50_ms"], 2)
                            h["speedup_p99_vs_cpu_thread_per_vote"] = round(q67["p99_ms"] / h["p99_ms"], 2)
            rec["latency"] = lat
        if (world > 1 or len(devs) > 1) and not rehearsal and not args.no_latency:
            # config 3 split over the node's GPUs, measured on the hardware (no
            # multi-GPU run of it existed)
            try:
                rec["latency_split"] = split_latency(max(world, len(devs)), args.latency_calls)
            except Exception as e:  # a measurement leg must not lose the headline line
                rec["latency_split"] = {"error": repr(e)[:300]}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier(group=gloo)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
