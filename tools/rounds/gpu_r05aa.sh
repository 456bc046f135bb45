#!/bin/bash
# Round 5: what the empty fix-up launch after config 2's verify kernel costs: the current build
# against one whose fix-up kernel has no body (SBFT_FIXUP_NOP; dispatch cost only), kernel-trace
# stats of the bench command, one box (the body-less build skips the init self-test, which
# runs the exact kernel over its vectors).
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
B="--no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined --steps 10 --warmup 3"
out=gpurun_out/r05aa_ab.txt; : > $out
for rep in 1 2; do
  for v in cur fixnop; do
    case $v in cur) unset SBFT_GV_LIB SBFT_GV_SELFTEST;; *) export SBFT_GV_LIB=$V/lib_$v.so SBFT_GV_SELFTEST=0;; esac
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05aa_${v}_$rep -o st --output-format csv -- python3 bench.py $B > gpurun_out/r05aa_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05aa_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05aa_${v}_$rep $v $rep >> $out <<'PY'
import csv, json, sys
d = json.loads([l for l in open(sys.argv[1] + ".log") if l.startswith("{")][-1])
ks = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(sys.argv[1] + "/st_kernel_stats.csv"))}
f = ks.get("sbft::p256_verify_fixup_kernel")
print(sys.argv[2], "rep", sys.argv[3], "value", d["value"], "ms_per_step", d["ms_per_step"], "fixup avg_us", round(float(f["AverageNs"]) / 1e3, 1) if f else None)
PY
  done
done
unset SBFT_GV_LIB SBFT_GV_SELFTEST
cat $out
