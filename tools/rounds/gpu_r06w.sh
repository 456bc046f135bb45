#!/bin/bash
# Round 6: is the ladders' ~2.5% cycle difference between builds the helper's concurrent code?
# h10 / h11: the helper idle from barrier 1 to barrier 2 (probe-only, wrong verdicts), pairing on / off.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06w
out=gpurun_out/$T.txt; : > $out
for n in 1250; do
for h in h0 h2 h10 h11 h4 h0 h2 h10 h11 h4; do
  nc=0; case $h in h10|h11) nc=1;; esac
  echo "== n=$n $h" >> $out
  SBFT_GV_SELFTEST=$((1-nc)) HALF_PROBE_NOCHECK=$nc HALF_PROBE_N=$n HALF_PROBE_WIDE=1 SBFT_GV_LIB=$V/lib_probe_$h.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/${T}_${n}_$h.log 2>&1 || { tail -5 gpurun_out/${T}_${n}_$h.log; exit 1; }
  grep "half-probe-clk" gpurun_out/${T}_${n}_$h.log | tail -4 | grep "verify inputs" >> $out
done
done
cat $out
