"""Config-5 hashing stage alone (bench.sha_config5) at a given message count."""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from smartbft_amd import GpuVerifier  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--messages", type=int, default=2_097_152)
ap.add_argument("--uniform-len", type=int, default=0)
a = ap.parse_args()
print(json.dumps(bench.sha_config5(GpuVerifier(device_mask=1), torch.device("cuda:0"), a.messages, a.uniform_len)))
