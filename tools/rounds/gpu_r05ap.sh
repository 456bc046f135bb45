#!/bin/bash
# Round 5: the registered-client keyed kernel's comb with the next accumulator's Z^2, Z^3 formed
# inside the current addition (SBFT_KEYED_LANES_ZPRE=1, the new default) against forming them at
# the start of the next (lib_zpre0): rocprofv3 averages over 40 proposals each, interleaved on
# one box; then the keyed / config / plugin / fault GPU tests on the default build.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
out=gpurun_out/r05ap_ab.txt; : > $out
for rep in 1 2 3; do
  for v in cur zpre0; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    KEYED_PROBE_CALLS=40 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ap_st_${v}_$rep -o st --output-format csv -- python3 tools/keyed_lanes_probe.py > gpurun_out/r05ap_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05ap_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05ap_st_${v}_$rep/st_kernel_stats.csv $v $rep >> $out <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "keyed_lanes" in r["Name"]:
        print(sys.argv[2], "rep", sys.argv[3], r["Name"].split("(")[0], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1), "min_us", round(float(r["MinNs"]) / 1e3, 1))
PY
  done
done
unset SBFT_GV_LIB
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_configs.py tests/test_gpu_plugin.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ap_tests.log 2>&1 || { tail -15 gpurun_out/r05ap_tests.log; exit 1; }
tail -1 gpurun_out/r05ap_tests.log >> $out
cat $out
