#!/bin/bash
# Round 5: the half kernel's table-conversion phase under a full batch, per build (probe builds,
# interleaved): probe = HEAD, probeA = lgkmcnt(0) after every conversion step, probeB = after the
# first and fourth (what the probetab marks imply), probetab = HEAD with marks in the loop.
mkdir -p gpurun_out
V=$PWD/tools/variants
out=gpurun_out/r05o_phases.txt; : > $out
for rep in 1 2; do
  for v in probe probeA probeB probetab; do
    echo "== $v rep $rep" >> $out
    SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05o_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05o_${v}_$rep.log; exit 1; }
    grep "half-probe verify" gpurun_out/r05o_${v}_$rep.log >> $out
  done
done
cat $out
