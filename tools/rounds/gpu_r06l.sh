#!/bin/bash
# Round 6: the wide kernel's affine (v u1) G -- none (general join, g0), safegcd (g1), Fermat chain
# (g2): phase probes at 5,000 and 1,250, and the half suites on the Fermat build.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
out=gpurun_out/r06l_probe.txt; : > $out
SBFT_GV_LIB=$V/lib_g2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06l_tests.log 2>&1 || { tail -30 gpurun_out/r06l_tests.log; exit 1; }
tail -1 gpurun_out/r06l_tests.log >> $out
for n in 5000 1250; do
for g in 0 1 2; do
  echo "== n=$n gaff=$g" >> $out
  HALF_PROBE_N=$n HALF_PROBE_WIDE=1 SBFT_GV_LIB=$V/lib_probe_g$g.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r06l_${n}_$g.log 2>&1 || { tail -5 gpurun_out/r06l_${n}_$g.log; exit 1; }
  grep half-probe gpurun_out/r06l_${n}_$g.log | tail -8 >> $out
done
done
cat $out
