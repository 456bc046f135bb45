#!/bin/bash
# Host-code AddressSanitizer on the GPU box: the library's host objects (gpuverify.cpp,
# verifier.cpp) and tools/latency_harness built with ASan for the host only (device code is the
# regular gfx950 build; no GPU sanitizer), then the harness's thread-heavy GPU modes: the
# consenter coalescer (66 concurrent callers), the uncoalesced zero-copy lanes, the batch hook,
# the processCommits collector, the signer and VerifyProposal (generic, bad signature, truncated,
# registered clients). Any ASan report aborts the step (halt_on_error).
# tools/asan_build (the ASan builds) is gpurun-ignored: drop that line from
# .gpurunignore to run this again.
mkdir -p gpurun_out
out=gpurun_out/r03asan.txt
: > $out
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0
H=tools/asan_build/latency_harness
run() {
  echo "== $*" >> $out
  timeout -k 10 180 $H "$@" >> $out 2>&1
  local rc=$?
  echo "rc=$rc" >> $out
  return $rc
}
run quorum-batch 67 200 && run quorum-gpu 66 200 66 50 && run quorum-gpu 66 100 0 0 && \
  run quorum-hook 67 66 200 && run sign 100 && run proposal-gpu 3000 20 && run proposal-gpu 10000 5
rc=$?
grep -c "AddressSanitizer" $out || true
cat $out | grep -v "^W2026\|^E2026\|amdgpu.ids" | tail -30
exit $rc
