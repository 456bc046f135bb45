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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000, help="tuples per GPU")
    ap.add_argument("--cpu-sample", type=int, default=131072)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip configs 3/4 latency")
    ap.add_argument("--latency-calls", type=int, default=200)
    ap.add_argument("--no-sha", action="store_true", help="skip the config-5 hashing measurement")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-buffer rate")
    ap.add_argument("--sha-messages", type=int, default=2_097_152,
                    help="config 5: 16M requests over 8 GPUs = 2M per GPU (~68 GB of payload in HBM)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "pmc_verify_latest.json"))
    return ap.parse_args()


def cpu_baseline(wl, sample: int, threads: int):
    """Oracle ('port') and OpenSSL timed on host cores over a bounded sample of the same
    workload; also returns the oracle verdicts of the sample (a free parity check)."""
    import oracle  # test infrastructure: the cpu_baseline leg is one of its allowed users
    sample = min(sample, wl.n)
    f = wl.host_fields(0, sample)
    oracle.lib()
    t0 = time.perf_counter()
    ok_cpu = oracle.verify_batch(*f, nthreads=threads)
    dt = time.perf_counter() - t0
    port = {"value": round(sample / dt, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
            "sample": f"first {sample} tuples of the bench workload, oracle/p256_oracle.c "
                      f"(C restatement of Go crypto/ecdsa.Verify), {threads} pthreads, {dt:.2f} s"}
    go_proxy = None
    exe = os.path.join(ROOT, "oracle", "openssl_bench")
    if os.path.exists(exe):
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as tf:
            tf.write(np.concatenate(f, axis=1).tobytes())
            path = tf.name
        try:
            out = subprocess.run([exe, path, str(threads), "10"], capture_output=True, text=True,
                                 timeout=120)
            if out.returncode == 0:
                j = json.loads(out.stdout.strip().splitlines()[-1])
                go_proxy = {"value": j["verifies_per_s"], "unit": "verifies/s", "cores": threads,
                            "kind": "fallback: OpenSSL 3.0.2 ECDSA_do_verify, not Go (Go absent)",
                            "sample": f"{sample} workload tuples cycled for {j['seconds']:.1f} s"}
        finally:
            os.unlink(path)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    port["cpu"] = cpu_model
    if go_proxy:
        go_proxy["cpu"] = cpu_model
    return port, go_proxy, ok_cpu


def host_path(gv, wl, dev, reps: int = 3):
    """PCIe-inclusive rate of the host-buffer C ABI (sbft_gv_verify_p256: the call a cgo
    plugin makes with Go-heap tuples): H2D of 160 B/tuple + verify pipeline + D2H of verdicts,
    on the same 1M tuples. Reported beside `value`, never as it."""
    f = [np.ascontiguousarray(a) for a in wl.host_fields(0, wl.n)]
    ok = gv.verify(*f)  # warm-up (workspace growth)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ok = gv.verify(*f)
        ts.append(time.perf_counter() - t0)
    want = (~wl.corrupted).to(torch.uint8).cpu().numpy()
    best = min(ts)
    out = {"value": round(wl.n / best, 1), "unit": "verifies/s", "ms": round(best * 1e3, 3),
           "mismatches": int((ok != want).sum()),
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
        out["pinned"] = {"value": round(wl.n / bp, 1), "unit": "verifies/s", "ms": round(bp * 1e3, 3),
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
                                  "path": "sbft_verifier_verify_proposal (C ABI), host buffers, PCIe incl."}
    # the same proposals with the 10k client keys registered (sbft_verifier_add_clients): every
    # request takes the keyed comb-table launch (no doublings, one wavefront per signature)
    vr = plugin.Verifier(gv, 1)
    t0 = time.perf_counter()
    vr.add_clients([q[-129:-64] for q in reqs])
    reg_s = time.perf_counter() - t0
    assert vr.VerifyProposal(prop) == v.VerifyProposal(prop)
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
        "path": "sbft_verifier_verify_proposal with the clients' keys registered (keyed launch), host buffers"}
    vr.close()
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
    return out


def sha_config5(gv, dev, n_msgs: int, uniform_len: int = 0):
    """BASELINE config 5's hashing stage on one GPU: payload lengths uniform in [1 KiB, 64 KiB]
    (seeded), device-resident, SHA-256 kernel only (kernel-time GB/s of payload bytes). A sample of
    digests is checked against hashlib."""
    import hashlib
    rng = np.random.default_rng(5)
    ln = rng.integers(1024, 65537, size=n_msgs).astype(np.uint32)
    if uniform_len:  # diagnostics: every message the same length
        ln[:] = uniform_len
    off = np.concatenate([[0], np.cumsum(ln.astype(np.uint64))[:-1]]).astype(np.uint64)
    total = int(ln.astype(np.uint64).sum())
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    blob = torch.randint(0, 256, (total + 128,), dtype=torch.uint8, device=dev, generator=g)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
    dig = torch.empty((n_msgs, 32), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    gv.sha256_dev(blob, d_off, d_len, dig, stream)
    torch.cuda.synchronize(dev)
    for i in (0, n_msgs // 2, n_msgs - 1):
        m = blob[int(off[i]):int(off[i]) + int(ln[i])].cpu().numpy().tobytes()
        assert dig[i].cpu().numpy().tobytes() == hashlib.sha256(m).digest(), i
    # the d_order path (messages taken in a permuted sequence) must give the same digests
    order = torch.flip(torch.arange(n_msgs, device=dev, dtype=torch.int32), [0])
    dig2 = torch.empty_like(dig)
    gv.sha256_dev(blob, d_off, d_len, dig2, stream, d_order=order)
    torch.cuda.synchronize(dev)
    assert torch.equal(dig, dig2), "permuted-order SHA-256 differs from index order"

    def timed(o):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record(stream)
        for _ in range(reps):
            gv.sha256_dev(blob, d_off, d_len, dig, stream, d_order=o)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / 1e3 / reps

    sec = timed(None)  # index order: the load-balanced kernel needs no length sort
    gbs = (total + 32 * n_msgs) / sec / 1e9
    # end to end from host memory (the host-buffer C ABI: pageable H2D + kernel + D2H) on a
    # bounded sample of the same messages: 65,536 messages, ~2.1 GB
    k = min(n_msgs, 65536)
    hb = blob[:int(off[k - 1]) + int(ln[k - 1])].cpu().numpy()
    gv.sha256(hb, off[:k], ln[:k])  # warm-up (staging growth)
    t0 = time.perf_counter()
    hd = gv.sha256(hb, off[:k], ln[:k])
    e2e = time.perf_counter() - t0
    assert hd[k - 1].tobytes() == dig[k - 1].cpu().numpy().tobytes()
    e2e_gbs = (hb.size + 32 * k) / e2e / 1e9
    del blob, hb
    return {"value": round(gbs, 1), "unit": "GB/s (payload + digest bytes, kernel time)",
            "messages": n_msgs, "payload_bytes": total, "avg_kernel_ms": round(sec * 1e3, 3),
            "end_to_end": {"value": round(e2e_gbs, 1), "unit": "GB/s", "messages": k,
                           "path": "sbft_gv_sha256 from pageable host memory (H2D + kernel + D2H)"},
            "roofline": {"bound": "valu", "hbm_peak_GBs": 8000, "frac_of_hbm": round(gbs / 8000, 4),
                         "valu_ceiling_GBs": 1840,
                         "frac_of_valu_ceiling": round(gbs / 1840, 4),
                         "note": "one lane per message; 1,421 VALU instructions per 64-B block (22.2/B) "
                                 "cap SHA-256 at ~1.84 TB/s on MI355X (tools/sha_ceiling.hip, "
                                 "register-resident blocks), below HBM"}}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    from smartbft_amd import GpuVerifier
    from smartbft_amd.workload import make_workload

    from smartbft_amd.dist import reduce_timing, shard_range

    gv = GpuVerifier(device_mask=1 << local)
    n = args.n
    lo, _ = shard_range(rank, world, n)
    wl = make_workload(gv, n, start=lo, device=local)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        gv.verify_dev(wl.digest, wl.r, wl.s, wl.qx, wl.qy, ok, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # parity property at full size: verdict == not corrupted, for every tuple
    expect = (~wl.corrupted).to(torch.uint8)
    mismatches = int((ok != expect).sum())

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    # HIP events around the main p256_verify_kernel itself, recorded by the library on the
    # launch stream (roofline.achieved); the torch events above bracket the whole step
    gv.kernel_timing(True)
    gv.kernel_time()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        elapsed, mismatches = reduce_timing(elapsed, mismatches, device=dev)
    step_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    avg_step_gpu_ms = sum(step_ms) / len(step_ms)
    launches, kern_total_ms = gv.kernel_time()
    gv.kernel_timing(False)
    assert launches == args.steps, (launches, args.steps)
    avg_kern_s = kern_total_ms / launches / 1e3

    if rank == 0:
        total = n * world * args.steps
        value = total / elapsed
        achieved_t = n * PRODUCTS_PER_VERIFY / avg_kern_s / 1e12
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
            "n_gpus": world,
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
                       "tuples_per_gpu": n, "parallelism": f"batch split x{world} (no collective)"},
            "roofline": {"bound": "valu", "achieved": round(achieved_t, 3), "peak": MAD_PEAK_T,
                         "unit": "T 32x32->64 products/s (v_mad_i64_i32 issue rate)",
                         "frac": round(achieved_t / MAD_PEAK_T, 4), "traffic": traffic,
                         "kernel": "p256_verify_kernel", "avg_kernel_ms": round(avg_kern_s * 1e3, 4),
                         "kernel_timing": "HIP events around p256_verify_kernel on its launch stream",
                         "step_gpu_ms": round(avg_step_gpu_ms, 4),
                         "step_kernels": "sinv_prep + sinv_totals + verify + fixup",
                         "products_per_verify": PRODUCTS_PER_VERIFY},
            # issued-instruction view of the same kernel: VALU instructions per verify from the
            # committed PMC pass (SQ_INSTS_VALU x 64 / n, profiles/pmc_verify_latest.json) at this
            # run's rate, against the chip's issue capacity (1,024 SIMDs x 64 lanes / 4 cycles at
            # the 2.4 GHz peak clock; the kernel runs at ~2.05 GHz, GRBM_GUI_ACTIVE)
            "valu_issue": None if not instr_per_verify else {
                "instr_per_verify": round(instr_per_verify), "achieved_T": round(instr_per_verify * n / avg_kern_s / 1e12, 2),
                "peak_T": VALU_ISSUE_PEAK_T, "frac": round(instr_per_verify * n / avg_kern_s / 1e12 / VALU_ISSUE_PEAK_T, 3),
                "frac_at_2_05GHz": round(instr_per_verify * n / avg_kern_s / 1e12 / (VALU_ISSUE_PEAK_T * 2.05 / 2.4), 3)},
            "parity": {"full_size_mismatches": mismatches,
                       "expected_accepts": int(expect.sum()) * world},
        }
        if world == 1 and not args.no_cpu_baseline:
            port, go_proxy, ok_cpu = cpu_baseline(wl, args.cpu_sample, args.cpu_threads)
            rec["cpu_baseline"] = port
            if go_proxy:
                rec["cpu_baseline_go_proxy"] = go_proxy
            rec["parity"]["oracle_sample_mismatches"] = int(
                (ok[:len(ok_cpu)].cpu().numpy() != ok_cpu).sum())
            rec["speedup_vs_cpu_baseline"] = round(value / port["value"], 1)
            if go_proxy:
                rec["speedup_vs_go_proxy"] = round(value / go_proxy["value"], 1)
        if world == 1 and not args.no_host_path:
            rec["host_buffer_path"] = host_path(gv, wl, dev)
        if world == 1 and not args.no_sha:
            rec["sha256_config5"] = sha_config5(gv, dev, args.sha_messages)
        if world == 1 and not args.no_latency:
            lat = latency_configs(gv, args.latency_calls)
            if "cpu_baseline_go_proxy" in rec:
                thr = rec["cpu_baseline_go_proxy"]["value"]
                lat["verify_proposal_10k"]["cpu_go_proxy_ms_estimate"] = round(10_000 / thr * 1e3, 3)
                lat["commit_quorum_n100"]["cpu_go_proxy_ms_estimate"] = round(67 / thr * 1e3, 3)
            rec["latency"] = lat
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
