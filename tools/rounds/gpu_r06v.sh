#!/bin/bash
# Round 6: ladder cycles against the helper's activity: h4 (helper one lane per tuple, idle lanes
# copy tuple 0), h9 (idle lanes on zeros), h2 (lane pairs), h0 (HEAD), at 1,250 (wide) and 10,000.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06v
out=gpurun_out/$T.txt; : > $out
for n in 1250 10000; do
for h in h0 h4 h9 h2 h0 h4 h9 h2; do
  w=1; [ $n = 10000 ] && w=0
  echo "== n=$n $h" >> $out
  HALF_PROBE_N=$n HALF_PROBE_WIDE=$w SBFT_GV_LIB=$V/lib_probe_$h.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/${T}_${n}_$h.log 2>&1 || { tail -5 gpurun_out/${T}_${n}_$h.log; exit 1; }
  grep "half-probe-clk" gpurun_out/${T}_${n}_$h.log | tail -4 | grep "verify inputs\|helper" >> $out
done
done
cat $out
