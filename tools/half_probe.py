"""Phase times of p256_verify_half_kernel (library built with -DSBFT_HALF_PROBE: workgroup 0's
verify lane 0 and helper lane 0 print 100 MHz real-time ticks since the kernel's start) on a
config-3 VerifyProposal of 10k requests. Usage: SBFT_GV_LIB=tools/variants/lib_probe.so python tools/half_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import GpuVerifier, plugin  # noqa: E402
from smartbft_amd.workload import make_signed_requests  # noqa: E402

# HALF_PROBE_N requests (default 10k: the four-lane kernel on one device); HALF_PROBE_WIDE=1 with
# N <= 6144 runs the wide form (a quad per ladder), =0 the four-lane one at the same N
n = int(os.environ.get("HALF_PROBE_N", "10000"))
gv = GpuVerifier(device_mask=1, halfq_max=0 if os.environ.get("HALF_PROBE_WIDE", "1") == "1" else -1)
reqs = make_signed_requests(gv, n, start=4242)
v = plugin.Verifier(gv, 0)
p = plugin.Proposal(plugin.encode_payload(reqs), b"h", b"m", 0)
# HALF_PROBE_NOCHECK=1: a timing-only build with wrong verdicts (run it with SBFT_GV_SELFTEST=0)
nocheck = os.environ.get("HALF_PROBE_NOCHECK") == "1"
for _ in range(int(os.environ.get("HALF_PROBE_CALLS", "4"))):  # more for a rocprofv3 average
    try:
        assert len(v.VerifyProposal(p)) == len(reqs)
    except Exception:
        if not nocheck:
            raise
sys.stdout.flush()
