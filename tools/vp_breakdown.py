"""Where the config-3 VerifyProposal latency goes: the whole C-ABI call vs its engine call
(sbft_gv_sha256_verify_p256 on prepared SoA arrays) vs the parse-only path."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from smartbft_amd import GpuVerifier, plugin  # noqa: E402
from smartbft_amd.workload import make_signed_requests  # noqa: E402

gv = GpuVerifier(device_mask=1)
reqs = make_signed_requests(gv, 10_000)
prop = plugin.Proposal(plugin.encode_payload(reqs), b"header", b"metadata", 1)
v = plugin.Verifier(gv, 1)
keep = []
cp = plugin._prop(prop, keep)
cap = 64 + len(prop.Payload)
infos = ctypes.create_string_buffer(cap)
cnt, bad = ctypes.c_size_t(), ctypes.c_int64()
err = ctypes.create_string_buffer(512)


def p50(f, reps=100):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[reps // 2] * 1e3


full = p50(lambda: v.L.sbft_verifier_verify_proposal(v.h, ctypes.byref(cp), infos, cap, ctypes.byref(cnt),
                                                      ctypes.byref(bad), err, 512))
parse = p50(lambda: v.L.sbft_verifier_requests_from_proposal(v.h, ctypes.byref(cp), infos, cap, ctypes.byref(cnt)))
# engine call alone on SoA arrays (offsets of each request body inside the payload)
pl = prop.Payload
off, ln, r, s, qx, qy = [], [], [], [], [], []
pos = 4
for q in reqs:
    pos += 4
    body = len(q) - 64
    off.append(pos); ln.append(body)
    sig = q[-64:]; pub = q[-129:-64]
    r.append(sig[:32]); s.append(sig[32:]); qx.append(pub[1:33]); qy.append(pub[33:])
    pos += len(q)
blob = np.frombuffer(pl, dtype=np.uint8)
arrs = [np.frombuffer(b"".join(x), dtype=np.uint8).reshape(-1, 32) for x in (r, s, qx, qy)]
o64, l32 = np.array(off, dtype=np.uint64), np.array(ln, dtype=np.uint32)
eng = p50(lambda: gv.sha256_verify(blob, o64, l32, *arrs))
okv = gv.sha256_verify(blob, o64, l32, *arrs)
print({"verify_proposal_ms": round(full, 3), "parse_only_ms": round(parse, 3), "engine_call_ms": round(eng, 3),
       "engine_ok": int(okv.sum()), "payload_bytes": len(pl)})
