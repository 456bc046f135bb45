"""Quick kernel timing on tiled golden vectors (development aid, not the bench)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from smartbft_amd import GpuVerifier
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_p256_vectors, split_fields
f, exp, cat, names = load_p256_vectors()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
reps = (n + len(f) - 1) // len(f)
big = np.tile(f, (reps, 1))[:n]
g = GpuVerifier()
dev = torch.device("cuda:0")
t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in split_fields(big)]
ok = torch.zeros(n, dtype=torch.uint8, device=dev)
g.verify_dev(*t, ok); torch.cuda.synchronize()
assert np.array_equal(ok.cpu().numpy(), np.tile(exp, reps)[:n])
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(3):
    e0.record(); g.verify_dev(*t, ok); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"n={n} kernel {ms:.2f} ms  {n / ms * 1e3 / 1e6:.3f} M verifies/s", flush=True)
