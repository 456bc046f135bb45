#!/bin/bash
# Round 5: the half kernel's table stores from the even lane of each pair only (SBFT_HALF_ST_EVEN=1;
# both lanes stored the same words): phases (probe builds) and kernel stats, one box, interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
out=gpurun_out/r05w_ab.txt; : > $out
for rep in 1 2; do
  for v in probe probeeven; do
    echo "== $v rep $rep" >> $out
    SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05w_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05w_${v}_$rep.log; exit 1; }
    grep "half-probe verify inputs" gpurun_out/r05w_${v}_$rep.log >> $out
  done
done
for rep in 1 2; do
  for v in cur steven; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05w_stats_${v}_$rep -o st --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05w_stats_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05w_stats_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05w_stats_${v}_$rep/st_kernel_stats.csv $v $rep >> $out <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "half_kernel<true>" in r["Name"]:
        print(sys.argv[2], "rep", sys.argv[3], "half<true> calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1), "min_us", round(float(r["MinNs"]) / 1e3, 1))
PY
  done
done
unset SBFT_GV_LIB
cat $out
