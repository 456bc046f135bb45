#!/bin/bash
# Round 6: why the ladders of h1-h3 run ~2.5% more cycles than HEAD's (h0): helper pairing off (h4),
# the helper's comb skipped (h6, h0i: probe-only, wrong verdicts), at 1,250 (wide) and 10,000 (four-lane).
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06u
out=gpurun_out/$T.txt; : > $out
for n in 1250 10000; do
for h in h0 h2 h4 h6 h0i h0 h2 h4; do
  w=1; [ $n = 10000 ] && w=0
  echo "== n=$n $h" >> $out
  nc=0; case $h in h6|h0i) nc=1;; esac
  SBFT_GV_SELFTEST=$((1-nc)) HALF_PROBE_NOCHECK=$nc HALF_PROBE_N=$n HALF_PROBE_WIDE=$w SBFT_GV_LIB=$V/lib_probe_$h.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/${T}_${n}_$h.log 2>&1 || { tail -5 gpurun_out/${T}_${n}_$h.log; exit 1; }
  grep "half-probe-clk" gpurun_out/${T}_${n}_$h.log | tail -4 | grep "verify inputs\|helper" >> $out
done
done
cat $out
