#!/bin/bash
# Round 6: wide kernel with the helper's affine sum by the Fermat chain (GAFF=2) and the quad join:
# the kernel at share sizes against the four-lane form, interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06m}
out=gpurun_out/$T.txt; : > $out
for n in 1250 2500 5000; do
  timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> $out 2> gpurun_out/${T}_sizes_$n.err || { tail -20 gpurun_out/${T}_sizes_$n.err; cat $out; exit 1; }
done
cat $out
