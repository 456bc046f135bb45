#!/bin/bash
# Host-code ThreadSanitizer on the GPU box: the library's host objects and tools/latency_harness
# built with -fsanitize=thread for the host only (device code the regular gfx950 build), through
# the multi-threaded GPU paths: the consenter coalescer, the processCommits collector, and
# VerifyProposal (its payload-copy helper thread). Reports inside the uninstrumented HIP runtime
# are suppressed; anything in our code is printed. tools/tsan_build is gpurun-ignored: drop that
# line from .gpurunignore to run this again.
mkdir -p gpurun_out
out=gpurun_out/r03tsan.txt
: > $out
printf 'called_from_lib:libamdhip64.so\ncalled_from_lib:libhsa-runtime64.so\n' > /tmp/tsan.supp
export TSAN_OPTIONS="suppressions=/tmp/tsan.supp halt_on_error=0 report_signal_unsafe=0"
H=tools/tsan_build/latency_harness
run() {
  echo "== $*" >> $out
  timeout -k 10 240 $H "$@" >> $out 2>&1
  local rc=$?
  echo "rc=$rc" >> $out
  return $rc
}
run parse-cpu 6000 20 && run quorum-gpu 66 50 66 50 && run quorum-hook 67 66 50 && run proposal-gpu 3000 10
rc=$?
echo "tsan warnings: $(grep -c 'WARNING: ThreadSanitizer' $out)"
grep -v "^W2026\|^E2026\|amdgpu.ids" $out | grep -E "^==|^\{|rc=|WARNING|#0|#1|#2|#3" | head -60
exit $rc
