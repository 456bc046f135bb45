#!/bin/bash
# Round 5: phase probes (SBFT_HALF_PROBE builds) of the half kernel, interleaved on one box:
# probe = HEAD (pair inversion, five-step addition), probeinv1 = one-lane inversion,
# probeplw6 = one-lane inversion and six-step addition.
mkdir -p gpurun_out
V=$PWD/tools/variants
out=gpurun_out/r05j_phases.txt; : > $out
for rep in 1 2; do
  for v in probe probeinv1 probeplw6; do
    echo "== $v rep $rep" >> $out
    SBFT_GV_LIB=$V/lib_$v.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05j_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r05j_${v}_$rep.log; exit 1; }
    grep half-probe gpurun_out/r05j_${v}_$rep.log >> $out
  done
done
cat $out
