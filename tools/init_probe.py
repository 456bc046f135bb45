"""Context start-up cost with and without the power-on self-test (sbft_gv_init)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import gpuverify  # noqa: E402

out = {}
for label, env in (("with_selftest_s", None), ("without_selftest_s", "0"), ("with_selftest_again_s", None)):
    if env is None:
        os.environ.pop("SBFT_GV_SELFTEST", None)
    else:
        os.environ["SBFT_GV_SELFTEST"] = env
    t = time.perf_counter()
    g = gpuverify.GpuVerifier()
    out[label] = round(time.perf_counter() - t, 4)
    g.close()
print(json.dumps(out))
