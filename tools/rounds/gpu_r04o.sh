#!/bin/bash
# Half kernel: table loops unrolled (entries and ratios in VGPRs, no scratch), verify-side input checks
# dropped (valid from the helper); then the co-Z entries staged in their LDS table slots (cur) against
# the all-register unrolled form (unroll) and the r04m build.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/r04o.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/r04o_$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/r04o_$name.log" | tail -4 | tee -a gpurun_out/r04o.log
    echo "rc=$rc" | tee -a gpurun_out/r04o.log
    return $rc
}
step half 500 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py tests/test_gpu_configs.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread || exit $?
SBFT_GV_LIB=$V/lib_probe.so step probe 120 python tools/half_probe.py || exit $?
out=gpurun_out/r04o_ab.txt
: > $out
for rep in 1 2 3; do
  for v in cur unroll r04m; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -k 10 180 python tools/latency_probe.py --calls 200 > gpurun_out/r04o_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r04o_${v}_$rep.log; exit 1; }
    python - gpurun_out/r04o_${v}_$rep.log $v $rep >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
L = d["verify_proposal_10k"]
print(sys.argv[2], "rep", sys.argv[3], "vp10k p50/p99", L["p50_ms"], L["p99_ms"])
PY
  done
done
unset SBFT_GV_LIB
cat $out
