#!/bin/bash
# Round 5: the half kernel's ladder reads a digit's table entry before its four doublings (pinned
# there, the sign applied after them; SBFT_HALF_ENTRY_EARLY=1) against reading it after them
# (lib_early0): GPU tests on the new build, then rocprofv3 averages over 40 config-3 proposals
# each, interleaved on one box.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py tests/test_gpu_fixup.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ao_tests.log 2>&1 || { tail -15 gpurun_out/r05ao_tests.log; exit 1; }
out=gpurun_out/r05ao_ab.txt; : > $out
tail -1 gpurun_out/r05ao_tests.log >> $out
for rep in 1 2 3; do
  for v in cur early0; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    HALF_PROBE_CALLS=40 timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ao_st_${v}_$rep -o st --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05ao_st_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05ao_st_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05ao_st_${v}_$rep/st_kernel_stats.csv $v $rep >> $out <<'PY'
import csv, sys
h = [r for r in csv.DictReader(open(sys.argv[1])) if "half_kernel<true>" in r["Name"]][0]
print(sys.argv[2], "rep", sys.argv[3], "half<true> calls", h["Calls"], "avg_us", round(float(h["AverageNs"]) / 1e3, 1), "min_us", round(float(h["MinNs"]) / 1e3, 1))
PY
  done
done
unset SBFT_GV_LIB
cat $out
