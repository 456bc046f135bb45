"""Child process of tests/test_gpu_runtime.py: the engine on the HIP runtime it ships with.

Every other GPU test runs in the pytest process, where torch (imported first, tests/conftest.py)
has already loaded its own bundled libamdhip64 (ROCm 7.0); the engine's NEEDED libamdhip64.so.7
then binds to torch's copy, and the tests verify on that runtime. A deployment (the Go plugin over
cgo, tools/latency_harness) loads no torch: the engine binds to /opt/rocm's runtime through its
RUNPATH. This script is that configuration: no torch, only ctypes and numpy, through the
host-buffer C ABI. It checks, against the golden fixtures and the oracle (the checker):
  - the 3,263 golden vectors and the crafted collisions on every kernel (throughput, pair, half,
    the exact fixup net);
  - a 10,000-request VerifyProposal, honest and with bad requests (first, middle, last index);
  - a 67-signature consenter batch (VerifyConsenterSigs), honest and with 3 bad signatures;
and prints one JSON line: the mapped HIP runtime paths and the results. Exit 0 iff all pass."""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from smartbft_amd import gpuverify, plugin  # noqa: E402


def mapped(pattern):
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if pattern in ln and "/" in ln})


def golden():
    raw = np.fromfile(os.path.join(HERE, "golden", "p256_vectors.bin"), dtype=np.uint8).reshape(-1, 162)
    cr = np.fromfile(os.path.join(HERE, "golden", "p256_crafted.bin"), dtype=np.uint8).reshape(-1, 162)
    return raw, cr


def cols(raw):
    return [np.ascontiguousarray(raw[:, 32 * k:32 * k + 32]) for k in range(5)]


def signed_requests(gv, n, start):
    """Config-3 requests (include/sbft_verifier.h format) signed with the host-buffer signer:
    distinct key per request, 64-256 B payloads."""
    def h(tag, i):
        return hashlib.sha256(b"SBFT-RT" + tag + i.to_bytes(8, "little")).digest()
    nn = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    def scalar(tag, i):
        return (int.from_bytes(h(tag, i), "big") % (nn - 1) + 1).to_bytes(32, "big")
    d = np.frombuffer(b"".join(scalar(b"d", start + i) for i in range(n)), dtype=np.uint8).reshape(n, 32)
    k = np.frombuffer(b"".join(scalar(b"k", start + i) for i in range(n)), dtype=np.uint8).reshape(n, 32)
    one = np.zeros((n, 32), dtype=np.uint8)
    one[:, 31] = 1
    qx, qy, _, _, st = gv.sign(d, one, one)  # pass 1: the public keys
    assert (st == 1).all()
    rng = np.random.default_rng(start)
    bodies = []
    for i in range(n):
        cid, rid = f"client{start + i}".encode(), f"tx{start + i}".encode()
        pl = (h(b"pl", start + i) * 9)[:int(rng.integers(64, 257))]
        bodies.append(b"SBR1" + len(cid).to_bytes(2, "little") + cid + len(rid).to_bytes(2, "little") + rid +
                      len(pl).to_bytes(4, "little") + pl + b"\x04" + qx[i].tobytes() + qy[i].tobytes())
    e = np.frombuffer(b"".join(hashlib.sha256(b).digest() for b in bodies), dtype=np.uint8).reshape(n, 32)
    _, _, r, s, st = gv.sign(d, k, e)
    assert (st == 1).all()
    return [b + r[i].tobytes() + s[i].tobytes() for i, b in enumerate(bodies)]


def main():
    out = {"torch_loaded": "torch" in sys.modules}
    gv = gpuverify.GpuVerifier(device_mask=1)
    out["hip_runtime"] = mapped("libamdhip64")
    out["hsa_runtime"] = mapped("libhsa-runtime64")
    raw, cr = golden()
    kernels = {"exact": gpuverify.KERNEL_EXACT, "throughput": gpuverify.KERNEL_THROUGHPUT,
               "pair": gpuverify.KERNEL_PAIR, "half": gpuverify.KERNEL_HALF}
    out["golden_mismatches"] = {}
    for name, k in kernels.items():
        got = gv.verify_kernel(k, *cols(raw))
        got_c = gv.verify_kernel(k, *cols(cr))
        out["golden_mismatches"][name] = int((got != raw[:, 160]).sum()) + int((got_c != cr[:, 160]).sum())
    out["golden_mismatches"]["selected"] = int((gv.verify(*cols(raw)) != raw[:, 160]).sum())

    # config 3: a 10k-request proposal, honest, then with bad requests
    reqs = signed_requests(gv, 10_000, 4242)
    v = plugin.Verifier(gv, 1)
    p = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
    infos = v.VerifyProposal(p)
    res = {"honest_ok": [(i.ClientID, i.ID) for i in infos] ==
           [(f"client{4242 + i}", f"tx{4242 + i}") for i in range(10_000)]}
    for where in ([0], [5000], [9999], [9999, 5000, 17]):
        bad = list(reqs)
        for i in where:
            q = bytearray(bad[i])
            q[-40] ^= 0x10  # a bit of s
            bad[i] = bytes(q)
        try:
            v.VerifyProposal(plugin.Proposal(plugin.encode_payload(bad), b"header", b"metadata", 1))
            res[str(where)] = "accepted"
        except plugin.VerifyError as e:
            res[str(where)] = "ok" if (e.code == plugin.EVERIFY and e.index == min(where)) else f"index {e.index}"
    out["verify_proposal_10k"] = res

    # config 4: 67 consenter signatures over one proposal, in one batch call
    signers = []
    for node in range(1, 68):
        priv = (int.from_bytes(hashlib.sha256(b"SBFT-RT-node" + bytes([node])).digest(), "big") % (2 ** 255) + 1)
        sg = plugin.Signer(gv, node, priv.to_bytes(32, "big"))
        v.add_consenter(node, sg.public_key())
        signers.append(sg)
    sigs = [sg.SignProposal(p, b"aux%d" % i) for i, sg in enumerate(signers)]
    st = v.VerifyConsenterSigs(sigs, p)
    bad_sigs = list(sigs)
    for i in (0, 33, 66):
        val = bytearray(bad_sigs[i].Value)
        val[5] ^= 1
        bad_sigs[i] = plugin.Signature(bad_sigs[i].ID, bytes(val), bad_sigs[i].Msg)
    st_bad = v.VerifyConsenterSigs(bad_sigs, p)
    out["consenter_67"] = {"honest_all_ok": all(x == 0 for x in st),
                           "bad_flagged": [i for i, x in enumerate(st_bad) if x != 0]}
    for sg in signers:
        sg.close()
    v.close()
    gv.close()
    out["torch_loaded_at_end"] = "torch" in sys.modules
    ok = (not out["torch_loaded_at_end"] and all(x == 0 for x in out["golden_mismatches"].values()) and
          all(x in (True, "ok") for x in res.values()) and out["consenter_67"]["honest_all_ok"] and
          out["consenter_67"]["bad_flagged"] == [0, 33, 66] and len(out["hip_runtime"]) == 1 and
          out["hip_runtime"][0].startswith("/opt/rocm"))
    out["pass"] = bool(ok)
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
