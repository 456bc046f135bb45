#!/bin/bash
# Round 5: private arrays kept out of LDS (-mllvm -disable-promote-alloca-to-lds: ~8.7 KB of the half
# kernel's LDS were promoted per-thread arrays, now 40 B of scratch) against the default build:
# half-kernel phases (probe builds, constant-slot stamps), kernel stats and config 2, one box.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
B="--no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined --steps 10 --warmup 3"
out=gpurun_out/r05ad_ab.txt; : > $out
for v in probe probenolds; do
  echo "== $v" >> $out
  SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05ad_$v.log 2>&1 || { tail -5 gpurun_out/r05ad_$v.log; exit 1; }
  grep "half-probe" gpurun_out/r05ad_$v.log | grep -v clk | tail -8 >> $out
done
for rep in 1 2; do
  for v in cur nolds; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ad_st_${v}_$rep -o st --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05ad_st_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05ad_st_${v}_$rep.log; exit 1; }
    timeout -k 10 300 python bench.py $B > gpurun_out/r05ad_b_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05ad_b_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05ad_st_${v}_$rep/st_kernel_stats.csv gpurun_out/r05ad_b_${v}_$rep.log $v $rep >> $out <<'PY'
import csv, json, sys
h = [r for r in csv.DictReader(open(sys.argv[1])) if "half_kernel<true>" in r["Name"]][0]
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[3], "rep", sys.argv[4], "half<true> avg_us", round(float(h["AverageNs"]) / 1e3, 1), "| bench", d["value"], d["ms_per_step"])
PY
  done
done
unset SBFT_GV_LIB
cat $out
