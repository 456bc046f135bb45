#!/bin/bash
# Round 5: per-wavefront phases of the half kernel's workgroup 0 (probe builds print waves 0, 1, 2
# and the helper): HEAD (probe) and HEAD with marks inside the conversion loop (probetab).
mkdir -p gpurun_out
V=$PWD/tools/variants
out=gpurun_out/r05p_phases.txt; : > $out
for rep in 1 2; do
  for v in probe probetab; do
    echo "== $v rep $rep" >> $out
    SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05p_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05p_${v}_$rep.log; exit 1; }
    grep "half-probe" gpurun_out/r05p_${v}_$rep.log | grep -v "clk" >> $out
  done
done
cat $out
