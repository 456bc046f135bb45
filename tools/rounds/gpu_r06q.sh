#!/bin/bash
# Round 6: ladder-digit timing probe (tools/isa/digit_bench.hip) at one wavefront per SIMD, field
# arithmetic variants: inline-asm fused DPP selects vs compiler moves, Montgomery look-ahead.
mkdir -p gpurun_out
T=r06q
out=gpurun_out/$T.txt; : > $out
for v in base qp0 la0 la2 la6 la8; do
  echo "== $v" >> $out
  timeout -k 10 60 tools/isa/digit_bench_$v 256 256 >> $out 2>&1 || { cat $out; exit 1; }
done
echo "== base G=512 (two wavefronts per SIMD)" >> $out
timeout -k 10 60 tools/isa/digit_bench_base 256 512 >> $out 2>&1 || { cat $out; exit 1; }
cat $out
