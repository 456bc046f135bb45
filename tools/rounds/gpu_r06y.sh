#!/bin/bash
# Round 6: the shipped library's link order against build_variants' (lib_h0, same sources): half
# kernels' HIP-event times at 1,250 / 5,000 / 10,000, interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06y
out=gpurun_out/$T.txt; : > $out
for n in 1250 5000 10000; do
  for g in main h0 main h0; do
    if [ $g = main ]; then L=$PWD/smartbft_amd/libsbft_gpuverify.so; else L=$V/lib_$g.so; fi
    echo -n "$g " >> $out
    SBFT_GV_LIB=$L timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> $out 2> gpurun_out/${T}_${g}_$n.err || { tail -20 gpurun_out/${T}_${g}_$n.err; cat $out; exit 1; }
  done
done
cat $out
