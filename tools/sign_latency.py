import sys, time, os
sys.path.insert(0, '.')
from smartbft_amd import GpuVerifier, plugin
import hashlib
gv = GpuVerifier(device_mask=1)
s = plugin.Signer(gv, 1, hashlib.sha256(b"k").digest())
s.Sign(b"warm")
ts = []
for i in range(100):
    t0 = time.perf_counter(); s.Sign(b"msg%d" % i); ts.append(time.perf_counter() - t0)
ts.sort()
print("Signer.Sign p50 %.3f ms p99 %.3f ms" % (ts[50] * 1e3, ts[98] * 1e3))
