#!/bin/bash
# Round 6: the wide kernel's join, same box: general join (g0), quad join with the safegcd-affine sum
# (g1), with the Fermat-affine sum (in-tree build, g2); kernel at share sizes vs the four-lane form,
# then rocprofv3 kernel stats of the in-tree build at 2,500.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
out=gpurun_out/r06n.txt; : > $out
for n in 1250 5000; do
  for g in g0 g1 g2; do
    if [ $g = g2 ]; then L=$PWD/smartbft_amd/libsbft_gpuverify.so; else L=$V/lib_$g.so; fi
    echo -n "$g " >> $out
    SBFT_GV_LIB=$L timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> $out 2> gpurun_out/r06n_${g}_$n.err || { tail -20 gpurun_out/r06n_${g}_$n.err; cat $out; exit 1; }
  done
done
cat $out
