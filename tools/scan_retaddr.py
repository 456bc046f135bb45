"""Scan the gfx950 code objects in a HIP shared library for device functions that overwrite
their own return address (round-5 finding, DESIGN.md §4 "The fix-up kernel's fault").

A non-kernel device function is entered with its return address in s[30:31] and returns with
`s_setpc_b64 s[30:31]`. ROCm 7.2's branch relaxation, expanding the conditional branches of a
function too large for a 16-bit branch offset, picked s[30:31] itself as the scratch pair of its
long branches (`s_getpc_b64 s[30:31]; s_add_u32 s30 ...; s_setpc_b64 s[30:31]`) in
`verify_general`, the fix-up kernel's callee: the function's return then jumped to its last
long-branch target and the kernel faulted. A leaf function has no reason to write s30 or s31 at
all, so any such write is reported.

Usage: python tools/scan_retaddr.py [lib.so] -> prints the offending functions; exit 1 if any.
Also imported by tests/test_abi.py (CPU only: llvm-objdump from /opt/rocm)."""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WRITE_S30 = re.compile(r"^\s*(s_\w+)\s+(s\[30:31\]|s30|s31)\b")


def code_objects(lib):
    """Extract the gfx950 code objects of lib (llvm-objdump --offloading writes them beside its
    input, so it runs on a copy in a temporary directory)."""
    tmp = tempfile.mkdtemp(prefix="sbft_scan_")
    cp = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, cp)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", cp], check=True, capture_output=True)
    return tmp, sorted(os.path.join(tmp, f) for f in os.listdir(tmp) if f.endswith("gfx950"))


def functions(co):
    """{name: [instruction lines]} of every code symbol, and the set of kernel names (.kd)."""
    syms = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", co], check=True, capture_output=True, text=True).stdout
    kernels = {m.group(1) for m in re.finditer(r"\s(\S+)\.kd\s*$", syms, re.M)}
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                         text=True).stdout
    out, cur = {}, None
    for ln in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur is not None and ln.strip():
            out[cur].append(ln.split("//")[0].strip())
    return out, kernels


def offenders(lib):
    """[(function, count of s30/s31 writes, first offending instruction)] over lib's device code."""
    tmp, cos = code_objects(lib)
    bad = []
    try:
        for co in cos:
            funcs, kernels = functions(co)
            for name, ins in funcs.items():
                if name in kernels or name.startswith(".L"):
                    continue
                if any(i.startswith("s_swappc_b64") for i in ins):
                    continue  # makes calls: saves and restores its return address itself
                writes = [i for i in ins if WRITE_S30.match(i) and not i.startswith("s_setpc_b64")]
                if writes:
                    bad.append((name, len(writes), writes[0]))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return bad


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "smartbft_amd", "libsbft_gpuverify.so")
    found = offenders(lib)
    for name, n, first in found:
        print(f"{name}: {n} writes of its return address, e.g. `{first}`")
    print(f"{len(found)} function(s) overwrite their return address")
    sys.exit(1 if found else 0)
