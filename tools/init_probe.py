"""Context start-up cost (sbft_gv_init): with and without the power-on self-test, and with 8 engine
slots on the one device (the in-process stand-in for an 8-GPU node: eight self-tests, which run
concurrently, one host thread per slot; the slots of one device share its G comb, so the 8-GPU
node's eight comb builds are not reproduced here -- they run concurrently the same way)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import gpuverify  # noqa: E402

out = {}
for label, env, slots in (("with_selftest_s", None, 1), ("without_selftest_s", "0", 1),
                          ("with_selftest_again_s", None, 1), ("with_selftest_8_slots_s", None, 8),
                          ("without_selftest_8_slots_s", "0", 8)):
    if env is None:
        os.environ.pop("SBFT_GV_SELFTEST", None)
    else:
        os.environ["SBFT_GV_SELFTEST"] = env
    t = time.perf_counter()
    g = gpuverify.GpuVerifier(device_mask=1, slots_per_device=slots)
    out[label] = round(time.perf_counter() - t, 4)
    g.close()
print(json.dumps(out))
