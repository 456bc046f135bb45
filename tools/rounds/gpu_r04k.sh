#!/bin/bash
# Half kernel without the square root on its critical path (pair B on E_c with W = c Z^2, the
# helper's Lehmer reduction, hash and square test after barrier 1): the half-kernel tests first,
# then the whole GPU suite, the phase probe, and interleaved A/B against HEAD's library (the
# round-4 half kernel; lib_pipe0 = the same without the pipelined safegcd).
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/r04k.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/r04k_$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/r04k_$name.log" | tail -4 | tee -a gpurun_out/r04k.log
    echo "rc=$rc" | tee -a gpurun_out/r04k.log
    return $rc
}
step half 400 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py -x -v --timeout 120 --timeout-method thread || exit $?
step tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
SBFT_GV_LIB=$V/lib_probe.so step probe 120 python tools/half_probe.py || exit $?
mkdir -p /tmp/headlib /tmp/pipe0lib && ln -sf $V/lib_head.so /tmp/headlib/libsbft_gpuverify.so && ln -sf $V/lib_pipe0.so /tmp/pipe0lib/libsbft_gpuverify.so
Q="--no-sha --no-host-path --no-cpu-baseline --no-pipelined --steps 10 --warmup 3"
out=gpurun_out/r04k_ab.txt
: > $out
for rep in 1 2; do
  for v in cur head pipe0; do
    case $v in cur) unset SBFT_GV_LIB; LP=;; head) export SBFT_GV_LIB=$V/lib_head.so; LP=/tmp/headlib;; pipe0) export SBFT_GV_LIB=$V/lib_pipe0.so; LP=/tmp/pipe0lib;; esac
    timeout -k 10 300 python bench.py $Q > gpurun_out/r04k_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r04k_${v}_$rep.log; exit 1; }
    python - gpurun_out/r04k_${v}_$rep.log $v $rep >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
L = d["latency"]
print(sys.argv[2], "rep", sys.argv[3], "value", round(d["value"] / 1e6, 2), "M/s kernel_ms", d["roofline"]["avg_kernel_ms"],
      "| vp10k p50/p99", L["verify_proposal_10k"]["p50_ms"], L["verify_proposal_10k"]["p99_ms"],
      "| registered p50/p99", L["verify_proposal_10k_registered_clients"]["p50_ms"], L["verify_proposal_10k_registered_clients"]["p99_ms"])
PY
    echo "$v rep $rep harness quorum-batch: $(LD_LIBRARY_PATH=$LP timeout -k 10 60 tools/latency_harness quorum-batch 67 400)" >> $out || exit 1
  done
done
unset SBFT_GV_LIB
cat $out
