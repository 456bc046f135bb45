#!/bin/bash
# Round 5: the always-launched fix-up kernel's grid (empty list) after config 2's verify kernel:
# 2048 blocks (the old cap, SBFT_FIXUP_BLOCKS=2048) against the new 64, kernel-trace stats of the
# bench command and its line, interleaved on one box; then the exceptional-tuple GPU tests.
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined --steps 10 --warmup 3"
out=gpurun_out/r05z_ab.txt; : > $out
for rep in 1 2; do
  for v in new old; do
    case $v in new) unset SBFT_FIXUP_BLOCKS;; old) export SBFT_FIXUP_BLOCKS=2048;; esac
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05z_${v}_$rep -o st --output-format csv -- python3 bench.py $B > gpurun_out/r05z_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05z_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05z_${v}_$rep $v $rep >> $out <<'PY'
import csv, json, sys, glob
d = json.loads([l for l in open(sys.argv[1] + ".log") if l.startswith("{")][-1])
ks = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(sys.argv[1] + "/st_kernel_stats.csv"))}
f = ks.get("sbft::p256_verify_fixup_kernel")
print(sys.argv[2], "rep", sys.argv[3], "value", d["value"], "ms_per_step", d["ms_per_step"], "fixup avg_us", round(float(f["AverageNs"]) / 1e3, 1) if f else None)
PY
  done
done
unset SBFT_FIXUP_BLOCKS
timeout -k 10 600 python -u -m pytest tests/test_gpu_exceptional.py tests/test_gpu_fixup.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z_tests.log 2>&1 || { tail -15 gpurun_out/r05z_tests.log; exit 1; }
tail -1 gpurun_out/r05z_tests.log >> $out
cat $out
