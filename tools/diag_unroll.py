import sys, random
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from test_gpu_field import _mul, _run, GX, GY, N
from smartbft_amd import GpuVerifier
import os
gpu = GpuVerifier()
rng = random.Random(5)
pts = [(GX, GY)] + [_mul(rng.randrange(1, N), (GX, GY)) for _ in range(20)]
want = [_mul(32, p)[0] for p in pts]
for op in (14, 15, 20, 21, 22):
    got = _run(gpu, op, pts)
    print(op, sum(g == w for g, w in zip(got, want)), "/", len(pts))
