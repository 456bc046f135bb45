"""The parity suite on the HIP runtime the engine ships with.

The other GPU tests share a process with torch, whose bundled ROCm 7.0 libamdhip64 the engine then
binds to (same SONAME). This test starts a fresh, torch-free child (tests/gpu_child_runtime.py:
ctypes + numpy over the host-buffer C ABI, as the Go plugin over cgo would load the engine) and
requires that the child maps only /opt/rocm's libamdhip64 (the engine's RUNPATH, ROCm 7.2) and that
it gets every verdict right: golden vectors and crafted collisions on every kernel, a 10k-request
VerifyProposal with bad requests, a 67-signature consenter batch."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_parity_on_the_shipped_hip_runtime():
    env = {k: v for k, v in os.environ.items() if k not in ("LD_LIBRARY_PATH", "SBFT_GV_LIB")}
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "gpu_child_runtime.py")],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    out = json.loads(lines[-1])
    print(json.dumps(out))
    assert not out["torch_loaded_at_end"]
    assert len(out["hip_runtime"]) == 1 and out["hip_runtime"][0].startswith("/opt/rocm"), out["hip_runtime"]
    assert "torch" not in " ".join(out["hip_runtime"] + out["hsa_runtime"])
    assert out["golden_mismatches"] == {"exact": 0, "throughput": 0, "pair": 0, "half": 0, "selected": 0}
    assert all(v in (True, "ok") for v in out["verify_proposal_10k"].values()), out["verify_proposal_10k"]
    assert out["consenter_67"] == {"honest_all_ok": True, "bad_flagged": [0, 33, 66]}
    assert out["pass"] and p.returncode == 0
