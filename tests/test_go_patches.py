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


def test_commit_hook_overlaps_and_guards_result_counts(tmp_path):
    """The processCommits hook keeps up to two VerifyConsenterSigs calls in flight (a decision
    with a bad vote overlaps its follow-up batch instead of serialising it), its result channel
    holds every in-flight batch (an aborted View leaves no goroutine blocked), and both hooks
    survive a batch verifier that returns the wrong number of results (no index panic)."""
    files = sorted({f for p in PATCHES for f in _touched(p)})
    for f in files:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    for p in PATCHES:
        subprocess.run(["git", "apply", os.path.join(ROOT, "go", "patches", p)], cwd=tmp_path, check=True)
    view = (tmp_path / "internal/bft/view.go").read_text()
    support = (tmp_path / "internal/bft/support.go").read_text()
    assert "const maxCommitBatches = 2" in view
    assert "batchDone := make(chan commitBatch, maxCommitBatches)" in view
    assert "inFlight < maxCommitBatches" in view
    assert "if len(res.errs) != len(res.sigs)" in view
    assert "batch verifier returned %d results for %d signatures" in view
    assert "len(auxes) == len(errs) ==" in support


def test_go_binding_fails_stop_on_engine_errors():
    """pkg/gpuverify never returns an engine failure (negative SBFT_GV_E* code) as a verification
    error: every entry point that can see one hands it to failStop."""
    src = open(os.path.join(ROOT, "go", "gpuverify", "verifier.go")).read()
    bat = open(os.path.join(ROOT, "go", "gpuverify", "batcher.go")).read()
    # engine codes only (ENODEV .. ESELFTEST); EINVAL and verdicts come back as VerifyError
    assert "func engineFailure(rc C.int) bool { return rc <= C.SBFT_GV_ENODEV && rc >= C.SBFT_GV_ESELFTEST }" in src
    for op in ("VerifyProposal", "VerifyRequest", "VerifyConsenterSig", "VerifyConsenterSigs", "VerifySignature",
               "PruneSet"):
        assert f'v.failStop("{op}", rc)' in src, op
    assert 'rv.failStop("VerifyRequest", rc)' in bat
    # every failStop is behind engineFailure: bad input (EINVAL, EFORMAT) never stops a replica
    assert src.count("if engineFailure(rc) {") == 6, src.count("if engineFailure(rc) {")
    assert bat.count("if engineFailure(rc) {") == 1
    test = open(os.path.join(ROOT, "go", "gpuverify", "verifier_test.go")).read()
    assert "func TestVerifyRequestEmptyIsMalformed" in test and "[][]byte{nil, {}}" in test
    assert "log.Fatalf" in src
