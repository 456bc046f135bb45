#!/bin/bash
# Round 5: the half kernel's table inversion split over the pair (inv::inv_mod_pair) against
# the one-lane inversion on both lanes (tools/variants/lib_inv1.so, -DSBFT_HALF_INV_PAIR=0): GPU tests, config-3 A/B,
# PMC VALU count and kernel stats of both.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
L=gpurun_out/r05i.log; : > $L
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a $L
    timeout -k 10 "$secs" "$@" > "gpurun_out/r05i_$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/r05i_$name.log" | tail -4 | tee -a $L
    echo "rc=$rc" | tee -a $L
    return $rc
}
step tests 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py tests/test_gpu_configs.py tests/test_gpu_split.py tests/test_gpu_fixup.py -x -q --timeout 240 --timeout-method thread || exit $?
SBFT_GV_LIB=$V/lib_probe.so step probe 120 python tools/half_probe.py || exit $?
out=gpurun_out/r05i_ab.txt; : > $out
for rep in 1 2 3; do
  for v in cur inv1; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_inv1.so;; esac
    timeout -k 10 180 python tools/latency_probe.py --calls 200 > gpurun_out/r05i_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05i_${v}_$rep.log; exit 1; }
    python - gpurun_out/r05i_${v}_$rep.log $v $rep >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
L = d["verify_proposal_10k"]
print(sys.argv[2], "rep", sys.argv[3], "vp10k p50/p99", L["p50_ms"], L["p99_ms"])
PY
  done
done
unset SBFT_GV_LIB
cat $out
R=--kernel-include-regex=p256_verify_half_kernel
for v in cur inv1; do
  case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_inv1.so;; esac
  timeout -s KILL 120 rocprofv3 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -d gpurun_out/r05i_pmc_$v -o pmc --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05i_pmc_$v.log 2>&1 || { tail -5 gpurun_out/r05i_pmc_$v.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05i_stats_$v -o st --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05i_stats_$v.log 2>&1 || { tail -5 gpurun_out/r05i_stats_$v.log; exit 1; }
done
unset SBFT_GV_LIB
find gpurun_out/r05i_pmc_* gpurun_out/r05i_stats_* -name "*.csv" | sort
