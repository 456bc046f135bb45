"""Diagnostic: host-API verify of tiled golden vectors at increasing sizes (one size per call
of this script, so a device fault ends only this process)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from conftest import load_p256_vectors, split_fields
from smartbft_amd import GpuVerifier
n = int(sys.argv[1])
f, exp, cat, names = load_p256_vectors()
reps = (n + len(f) - 1) // len(f)
big = np.tile(f, (reps, 1))[:n]
want = np.tile(exp, reps)[:n]
g = GpuVerifier()
got = g.verify(*split_fields(big))
print(f"n={n} mismatches={int((got != want).sum())}", flush=True)
