#!/bin/bash
# Round 6: the ladder loop's code alignment (-falign-loops) against the ~2.5% build-to-build cycle
# difference: h2 code (helper pairs) and h4 code (one lane per tuple) at 256 B / 1 KiB / 4 KiB.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06x
out=gpurun_out/$T.txt; : > $out
for n in 1250 10000; do
for h in h0 h2 a256 a1k a4k h4 h4a1k h4a4k h0 a1k a4k h4a1k h4a4k; do
  w=1; [ $n = 10000 ] && w=0
  echo "== n=$n $h" >> $out
  HALF_PROBE_N=$n HALF_PROBE_WIDE=$w SBFT_GV_LIB=$V/lib_probe_$h.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/${T}_${n}_$h.log 2>&1 || { tail -5 gpurun_out/${T}_${n}_$h.log; exit 1; }
  grep "half-probe-clk" gpurun_out/${T}_${n}_$h.log | tail -4 | grep "verify inputs\|helper" >> $out
done
done
cat $out
