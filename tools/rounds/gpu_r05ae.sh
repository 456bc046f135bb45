#!/bin/bash
# Round 5: the half kernel's ladder digits by selects (q_digit_sel: k stays in registers instead of
# an alloca LLVM promoted to 8 KB of LDS) against the runtime-indexed q_digit (lib_dig0,
# -DSBFT_HALF_DIGIT_SEL=0), one box: GPU tests, phases (probe build), kernel stats, config-3 p50.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py tests/test_gpu_fixup.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ae_tests.log 2>&1 || { tail -15 gpurun_out/r05ae_tests.log; exit 1; }
out=gpurun_out/r05ae_ab.txt; : > $out
tail -1 gpurun_out/r05ae_tests.log >> $out
SBFT_GV_LIB=$V/lib_probe.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05ae_probe.log 2>&1 || { tail -5 gpurun_out/r05ae_probe.log; exit 1; }
grep "half-probe" gpurun_out/r05ae_probe.log | grep -v clk | tail -4 >> $out
for rep in 1 2 3; do
  for v in cur dig0; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ae_st_${v}_$rep -o st --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05ae_st_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05ae_st_${v}_$rep.log; exit 1; }
    timeout -k 10 180 python tools/latency_probe.py --calls 200 > gpurun_out/r05ae_lat_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05ae_lat_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05ae_st_${v}_$rep/st_kernel_stats.csv gpurun_out/r05ae_lat_${v}_$rep.log $v $rep >> $out <<'PY'
import csv, json, sys
h = [r for r in csv.DictReader(open(sys.argv[1])) if "half_kernel<true>" in r["Name"]][0]
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
L = d["verify_proposal_10k"]
print(sys.argv[3], "rep", sys.argv[4], "half<true> avg_us", round(float(h["AverageNs"]) / 1e3, 1), "min_us", round(float(h["MinNs"]) / 1e3, 1), "| vp10k p50/p99", L["p50_ms"], L["p99_ms"])
PY
  done
done
unset SBFT_GV_LIB
cat $out
