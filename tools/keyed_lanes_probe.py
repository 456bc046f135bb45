"""Phase times of p256_verify_keyed_lanes_kernel<true> (library built with -DSBFT_KEYED_PROBE:
workgroup 0's wavefronts print 100 MHz real-time ticks since the kernel's start) on a config-3
VerifyProposal of 10k requests whose clients are registered.
Verify wavefronts: [s^-1, digest barrier, u, comb, quad combines, final check];
hash wavefront: [hashed, barrier]. Usage: SBFT_GV_LIB=tools/variants/lib_kprobe.so python tools/keyed_lanes_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smartbft_amd import GpuVerifier, plugin  # noqa: E402
from smartbft_amd.workload import make_signed_requests  # noqa: E402

gv = GpuVerifier(device_mask=1)
reqs = make_signed_requests(gv, 10_000, start=4242)
v = plugin.Verifier(gv, 1)
v.add_clients([q[-129:-64] for q in reqs])
p = plugin.Proposal(plugin.encode_payload(reqs), b"h", b"m", 0)
check = not os.environ.get("KEYED_PROBE_NOCHECK")  # set for timing-only builds (wrong verdicts)
for _ in range(int(os.environ.get("KEYED_PROBE_CALLS", "4"))):  # more for a rocprofv3 average
    if check:
        assert len(v.VerifyProposal(p)) == len(reqs)
    else:
        try:
            v.VerifyProposal(p)
        except plugin.VerifyError:
            pass
sys.stdout.flush()
