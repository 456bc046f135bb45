"""Latency configs 3/4 alone (bench.latency_configs), for profiling the small-batch path:
  rocprofv3 --kernel-trace --stats -d gpurun_out/lat -- python3 tools/latency_probe.py --calls 50"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from smartbft_amd import GpuVerifier  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=50)
a = ap.parse_args()
print(json.dumps(bench.latency_configs(GpuVerifier(device_mask=1), a.calls)))
