"""Phase times of p256_verify_half_kernel (library built with -DSBFT_HALF_PROBE: workgroup 0's
verify lane 0 and helper lane 0 print 100 MHz real-time ticks since the kernel's start) on a
config-3 VerifyProposal of 10k requests. Usage: SBFT_GV_LIB=tools/variants/lib_probe.so python tools/half_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import GpuVerifier, plugin  # noqa: E402
from smartbft_amd.workload import make_signed_requests  # noqa: E402

gv = GpuVerifier(device_mask=1)
reqs = make_signed_requests(gv, 10_000, start=4242)
v = plugin.Verifier(gv, 0)
p = plugin.Proposal(plugin.encode_payload(reqs), b"h", b"m", 0)
for _ in range(int(os.environ.get("HALF_PROBE_CALLS", "4"))):  # more for a rocprofv3 average
    assert len(v.VerifyProposal(p)) == len(reqs)
sys.stdout.flush()
