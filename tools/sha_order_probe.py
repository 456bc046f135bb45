"""Config-5 hash kernel, 2M random 1-64 KiB messages: the engine's own order (no d_order: at
>= 65,536 messages it sorts them longest first itself), an exact host-computed longest-first
order, and a random permutation (sbft_gv_sha256_dev's d_order). Each lane streams whole
messages from its wave's queue, so long messages drawn last set a tail."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import GpuVerifier  # noqa: E402
from smartbft_amd.workload import make_config5  # noqa: E402

gv = GpuVerifier(device_mask=1)
dev = torch.device("cuda:0")
c5 = make_config5(gv, 2_097_152, device=0)
n = c5.n
dig = torch.empty(32 * n, dtype=torch.uint8, device=dev)
dig2 = torch.empty_like(dig)
stream = torch.cuda.current_stream(dev)
lpt = torch.argsort(c5.d_len.to(torch.int64), descending=True).to(torch.int32)
rnd = torch.randperm(n, device=dev).to(torch.int32)


def timed(f, reps=5):
    f()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = []
    for _ in range(reps):
        ev[0].record(stream)
        f()
        ev[1].record(stream)
        torch.cuda.synchronize()
        best.append(ev[0].elapsed_time(ev[1]))
    best.sort()
    return best[len(best) // 2]


out = {}
for rep in range(2):
    out[f"engine_ms_{rep}"] = timed(lambda: gv.sha256_dev(c5.blob, c5.d_off, c5.d_len, dig, stream, check=False))
    out[f"lpt_ms_{rep}"] = timed(lambda: gv.sha256_dev(c5.blob, c5.d_off, c5.d_len, dig2, stream, d_order=lpt, check=False))
    out[f"random_ms_{rep}"] = timed(lambda: gv.sha256_dev(c5.blob, c5.d_off, c5.d_len, dig2, stream, d_order=rnd, check=False))
assert torch.equal(dig, dig2)
out["payload_bytes"] = int(c5.total)
out["GBs_engine"] = out["payload_bytes"] / out["engine_ms_1"] / 1e6
out["GBs_lpt"] = out["payload_bytes"] / out["lpt_ms_1"] / 1e6
print(json.dumps(out))
