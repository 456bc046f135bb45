#!/bin/bash
# Round 5: the pair kernel's digits by selects (q_digit_sel) against the runtime-indexed q_digit
# (lib_pdig0, -DSBFT_PAIR_DIGIT_SEL=0): pair-kernel stats over golden-vector batches of 20k
# (tools/pair_kernel_time.py), one box, interleaved; then the GPU verify tests.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
out=gpurun_out/r05af_ab.txt; : > $out
for rep in 1 2 3; do
  for v in cur pdig0; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05af_st_${v}_$rep -o st --output-format csv -- python3 tools/pair_kernel_time.py > gpurun_out/r05af_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05af_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05af_st_${v}_$rep/st_kernel_stats.csv $v $rep >> $out <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "small_kernel<2" in r["Name"]:
        print(sys.argv[2], "rep", sys.argv[3], r["Name"].split("(")[0], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
  done
done
unset SBFT_GV_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py tests/test_gpu_fixup.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05af_tests.log 2>&1 || { tail -15 gpurun_out/r05af_tests.log; exit 1; }
tail -1 gpurun_out/r05af_tests.log >> $out
cat $out
