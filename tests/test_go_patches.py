"""The internal/bft batch-hook patches (go/patches/*.patch) against the reference
tree: each applies cleanly, in order, to the reference's own files (`git apply`, the way a
maintainer would apply them at the SmartBFT module root), and the hooks they add are present.
Go is absent, so the patched files are not compiled; this catches drift between the patches and
the reference. Skipped where the reference tree is absent (the GPU box)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCHES = ["internal_bft_prev_commits.patch", "internal_bft_commits.patch"]  # application order

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "internal", "bft")),
                                reason="reference tree absent")


def _touched(patch: str) -> list[str]:
    txt = open(os.path.join(ROOT, "go", "patches", patch)).read()
    return sorted(set(re.findall(r"^\+\+\+ b/(\S+)", txt, flags=re.M)))


def test_patches_apply_in_order(tmp_path):
    files = sorted({f for p in PATCHES for f in _touched(p)})
    assert "internal/bft/view.go" in files and "internal/bft/support.go" in files
    for f in files:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    for p in PATCHES:
        r = subprocess.run(["git", "apply", "--verbose", os.path.join(ROOT, "go", "patches", p)],
                           cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 0, f"{p}: {r.stderr}"
    view = (tmp_path / "internal/bft/view.go").read_text()
    support = (tmp_path / "internal/bft/support.go").read_text()
    assert "type batchConsenterSigVerifier interface" in support
    # hook 1: verifyPrevCommitSignatures keeps both error texts of the serial loop
    assert view.count('"failed verifying consenter signature of %d: %w"') == 2
    assert view.count('"failed unmarshaling auxiliary input from %d: %w"') == 2
    # hook 2: processCommits batches the votes and keeps the per-vote warnings
    assert "bv, batched := v.Verifier.(batchConsenterSigVerifier)" in view
    assert view.count('"Couldn\'t verify %d\'s signature: %v"') == 2
    assert view.count('"Got wrong digest at processCommits for seq %d"') == 2
    assert "case <-v.abortChan:" in view


def test_patch_lines_are_gofmt_indented():
    """Added Go lines indent with tabs, as gofmt writes them."""
    for p in PATCHES:
        for line in open(os.path.join(ROOT, "go", "patches", p)):
            if line.startswith("+") and not line.startswith("+++"):
                body = line[1:].rstrip("\n")
                assert not re.match(r"^ +\S", body), f"{p}: space-indented line {body!r}"
