#!/bin/bash
# Round 5: the registered-client keyed kernel (p256_verify_keyed_lanes_kernel<true>, config 3 with
# the clients registered): 48 signatures per workgroup (the hash wavefront on a SIMD of its own,
# the new default) against 64 (lib_t64), and both against the round's earlier form (lib_old: 64,
# rotated entry buffer). rocprofv3 kernel averages over 40 proposals each, interleaved; phase
# probes of 48 and 64; then the keyed / config / plugin GPU tests on the default build.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
out=gpurun_out/r05am_ab.txt; : > $out
for rep in 1 2 3; do
  for v in cur t64 old; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    KEYED_PROBE_CALLS=40 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05am_st_${v}_$rep -o st --output-format csv -- python3 tools/keyed_lanes_probe.py > gpurun_out/r05am_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05am_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05am_st_${v}_$rep/st_kernel_stats.csv $v $rep >> $out <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "keyed_lanes" in r["Name"]:
        print(sys.argv[2], "rep", sys.argv[3], r["Name"].split("(")[0], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1), "min_us", round(float(r["MinNs"]) / 1e3, 1))
PY
  done
done
unset SBFT_GV_LIB
for v in kprobe kprobe64; do
  SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 300 python tools/keyed_lanes_probe.py > gpurun_out/r05am_p_$v.log 2>&1 || { tail -5 gpurun_out/r05am_p_$v.log; exit 1; }
  echo "== $v" >> $out; grep keyed-probe gpurun_out/r05am_p_$v.log | tail -5 >> $out
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_configs.py tests/test_gpu_plugin.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05am_tests.log 2>&1 || { tail -15 gpurun_out/r05am_tests.log; exit 1; }
tail -1 gpurun_out/r05am_tests.log >> $out
cat $out
