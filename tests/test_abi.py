"""CPU tests of the C-ABI library: it loads, exports every symbol include/*.h declares, and
its host-only helpers follow Go semantics. No compute call is made without a GPU."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        syms |= set(re.findall(r"\b(sbft_\w+)\s*\(", text))
    return syms


def test_library_exports_every_declared_symbol():
    from smartbft_amd import gpuverify
    lib = gpuverify.load_library()
    syms = _declared_symbols()
    assert len(syms) >= len(gpuverify.EXPORTS)
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from smartbft_amd import gpuverify
    hdr = set()
    text = open(os.path.join(ROOT, "include", "sbft_gpuverify.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    hdr |= set(re.findall(r"\b(sbft_gv_\w+)\s*\(", text))
    assert hdr == set(gpuverify.EXPORTS)


def test_normalize_helpers_go_semantics():
    from smartbft_amd import gpuverify
    import oracle
    for h in [b"", b"\x05", bytes(range(20)), bytes(range(32)), bytes(range(48)), bytes(range(64))]:
        assert gpuverify.normalize_hash(h) == oracle.normalize_hash(h)
    assert gpuverify.normalize_scalar(b"\x01\x02") == b"\0" * 30 + b"\x01\x02"
    assert gpuverify.normalize_scalar(b"\0" * 5 + b"\xff" * 32) == b"\xff" * 32
    assert gpuverify.normalize_scalar(b"\x01" + b"\0" * 32) is None  # 257 bits: reject


def test_strerror_and_no_gpu_failure_is_loud():
    from smartbft_amd import gpuverify
    lib = gpuverify.load_library()
    assert lib.sbft_gv_strerror(-2) == b"no usable GPU"
    assert lib.sbft_gv_strerror(-6) == b"device failed the known-answer self-test"
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: the no-GPU error path is not reachable")
    with pytest.raises(gpuverify.GpuVerifyError):
        gpuverify.GpuVerifier()


def test_verify_workspace_layout():
    """The verify pipeline's device workspace: fixup counter + list (4(n+1) B, 256-aligned),
    then pre | suf (32 B per tuple) and tot | kb (32 B per 256-tuple workgroup), then (256-aligned)
    the per-lane Q tables (640 B per tuple). An undersized workspace is a device fault, so pin
    the formula on the CPU."""
    from smartbft_amd import gpuverify
    lib = gpuverify.load_library()
    for n in [1, 255, 256, 257, 65280, 65536, 1_000_000]:
        blocks = (n + 255) // 256
        want = ((((4 * (n + 1) + 255) // 256) * 256 + 64 * n + 64 * blocks + 255) // 256) * 256 + 640 * n
        assert lib.sbft_gv_verify_workspace_bytes(n) == want, n


def test_host_alloc_argument_handling():
    """sbft_gv_host_alloc: a NULL out pointer is EINVAL, a zero-byte request succeeds with
    *out = NULL (neither touches the device); sbft_gv_host_free(NULL) is a no-op."""
    from smartbft_amd import gpuverify
    lib = gpuverify.load_library()
    assert lib.sbft_gv_host_alloc(16, None) == -1  # SBFT_GV_EINVAL
    p = ctypes.c_void_p(1)
    assert lib.sbft_gv_host_alloc(0, ctypes.byref(p)) == 0
    assert p.value is None
    lib.sbft_gv_host_free(None)


def test_go_binding_uses_only_declared_symbols():
    """go/gpuverify is uncompiled here (no Go toolchain): at least every C function and macro it
    names must exist in include/*.h, and every api.Verifier / api.Signer method
    (pkg/api/dependencies.go:46-71) must be defined."""
    declared = _declared_symbols()
    text = ""
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text += open(h).read()
    macros = set(re.findall(r"#define\s+(SBFT_\w+)", text))
    go = ""
    for f in glob.glob(os.path.join(ROOT, "go", "gpuverify", "*.go")):
        go += open(f).read()
    used = set(re.findall(r"\bC\.(sbft_\w+)\s*\(", go))
    assert used and not (used - declared), sorted(used - declared)
    used_macros = set(re.findall(r"\bC\.(SBFT_\w+)", go))
    assert not (used_macros - macros), sorted(used_macros - macros)
    for m in ["VerifyProposal", "VerifyRequest", "VerifyConsenterSig", "VerifySignature", "VerificationSequence",
              "RequestsFromProposal", "AuxiliaryData", "Sign", "SignProposal", "VerifyConsenterSigs"]:
        assert re.search(r"func \(\w+ \*(Verifier|Signer)\) %s\(" % m, go), m
    assert "elided" not in go


def test_power_on_selftest_vectors_match_fixtures():
    """The engine's init-time known-answer records (smartbft_amd/csrc/p256_post_vectors.inc,
    tools/gen_post_vectors.py) are fixture records with the fixtures' verdicts, and its SHA-256
    answers are hashlib's: a stale or hand-edited table would make every context refuse to start."""
    import hashlib
    import re
    text = open(os.path.join(ROOT, "smartbft_amd", "csrc", "p256_post_vectors.inc")).read()
    body = text[text.index("kPostVectors"):text.index("};")]
    recs = [bytes(int(x, 16) for x in m.split(",")) for m in re.findall(r"\{([0-9a-fx,]+)\}", body)]
    raw = np.fromfile(os.path.join(ROOT, "tests", "golden", "p256_vectors.bin"), dtype=np.uint8).reshape(-1, 162)
    fixtures = {bytes(r[:160]): int(r[160]) for r in raw}
    assert len(recs) == int(re.search(r"SBFT_POST_N (\d+)", text).group(1)) >= 64
    for r in recs:
        assert len(r) == 161 and fixtures[r[:160]] == r[160]
    cats = set(int(r[161]) for r in raw if bytes(r[:160]) in {x[:160] for x in recs})
    assert len(cats) == 18  # every category, the exceptional ones included
    blob = bytes(int(x, 16) for x in re.findall(r"0x([0-9a-f]{2})", text[text.index("kPostShaBlob"):text.index("kPostShaOff")]))
    off = [int(x) for x in re.search(r"kPostShaOff\[SBFT_POST_SHA_N\] = \{([^}]*)\}", text).group(1).split(",")]
    ln = [int(x) for x in re.search(r"kPostShaLen\[SBFT_POST_SHA_N\] = \{([^}]*)\}", text).group(1).split(",")]
    dig = text[text.index("kPostShaDigest"):]
    digs = [bytes(int(x, 16) for x in m.split(",")) for m in re.findall(r"\{([0-9a-fx,]+)\}", dig)]
    assert [hashlib.sha256(blob[o:o + n]).digest() for o, n in zip(off, ln)] == digs


def test_half_kernel_constants():
    """The constants p256_verify_half_kernel carries in its source: b 2^261 mod p in radix 2^29
    (the curve's b in the ladder's Montgomery domain), p - n (the bound below which x(R) = r + n
    is a second candidate), and the group order of p256_halfgcd.hpp."""
    import re
    P = 2**256 - 2**224 + 2**192 + 2**96 - 1
    N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
    src = open(os.path.join(ROOT, "smartbft_amd", "csrc", "p256_verify.hip")).read()

    def words(name, radix):
        m = re.search(name + r"\[\d+\] = \{([^}]*)\}", src)
        return sum(int(w.strip().rstrip("u"), 16) << (radix * i) for i, w in enumerate(m.group(1).split(",")))
    assert words("C29_B", 29) == B * 2**261 % P
    assert words("P256_PMN", 32) == P - N
    hg = open(os.path.join(ROOT, "smartbft_amd", "csrc", "p256_halfgcd.hpp")).read()
    m = re.search(r"#define SBFT_HGCD_N \{([^}]*)\}", hg)
    assert sum(int(w.strip().rstrip("u"), 16) << (32 * i) for i, w in enumerate(m.group(1).split(","))) == N


def test_blob_bounds_predicate_does_not_wrap():
    """_blob_bounds_bad (the device-resident hash entries' offset check) compares without forming
    off + len, so offsets near 2^63 are refused instead of wrapping into range."""
    import torch
    from smartbft_amd.gpuverify import GpuVerifier
    off = torch.tensor([0, 246, 247, (1 << 63) - 1, (1 << 63) - 5, -1, 0], dtype=torch.int64)
    ln = torch.tensor([256, 10, 10, 10, 4, 1, 257], dtype=torch.int32)
    got = GpuVerifier._blob_bounds_bad(off, ln, 256).tolist()
    assert got == [False, False, True, True, True, True, True]
    u = torch.tensor([0, 1 << 63, (1 << 64) - 1], dtype=torch.uint64)  # >= 2^63 reads negative
    assert GpuVerifier._blob_bounds_bad(u, torch.tensor([1, 1, 1], dtype=torch.int32), 256).tolist() == \
        [False, True, True]
    big = torch.tensor([0], dtype=torch.int32) - 1  # length 2^32 - 1 as uint32
    assert GpuVerifier._blob_bounds_bad(torch.tensor([0]), big, 256).tolist() == [True]


def test_no_device_function_overwrites_its_return_address():
    """The built library holds no non-kernel device function that writes s[30:31], its return
    address (tools/scan_retaddr.py). ROCm 7.2's branch relaxation did this in the >128 KiB
    verify_general (the fixup kernel's callee) from round 4 on, and the fixup kernel faulted on its
    first flagged tuple."""
    import shutil
    if not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump") or not shutil.which("python3"):
        pytest.skip("no ROCm llvm-objdump")
    sys_path = os.path.join(ROOT, "tools")
    import importlib.util
    spec = importlib.util.spec_from_file_location("scan_retaddr", os.path.join(sys_path, "scan_retaddr.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from smartbft_amd import gpuverify
    assert mod.offenders(gpuverify.LIB_PATH) == []
