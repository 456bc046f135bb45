"""bench.adversarial alone (worst-case batches: every tuple exceptional or a crafted collision), for
same-box A/B of library variants: SBFT_GV_LIB=tools/variants/lib_X.so python tools/adv_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from smartbft_amd import GpuVerifier  # noqa: E402

print(json.dumps(bench.adversarial(GpuVerifier(device_mask=1), torch.device("cuda:0"))))
