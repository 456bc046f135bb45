#!/bin/bash
# Round 5: is the table conversion's slowness under load a first-execution (cold code) effect?
# probedry runs the conversion once without stores before the real one (columns: inputs, chain,
# inverse, dry run, tables, barrier 1, ladder, barrier 2); probe = HEAD.
mkdir -p gpurun_out
V=$PWD/tools/variants
out=gpurun_out/r05v_phases.txt; : > $out
for rep in 1 2; do
  for v in probe probedry; do
    echo "== $v rep $rep" >> $out
    SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05v_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05v_${v}_$rep.log; exit 1; }
    grep "half-probe verify inputs" gpurun_out/r05v_${v}_$rep.log >> $out
  done
done
cat $out
