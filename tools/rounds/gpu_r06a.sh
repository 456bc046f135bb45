#!/bin/bash
# Round 6: the wide half kernel (a quad per ladder). Unit test of the quad ladder, the half-kernel
# suites in every mode, then kernel times of the four-lane and wide forms at share sizes.
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r06a}.txt; : > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG:-r06a}_field.log 2>&1 || { tail -30 gpurun_out/${TAG:-r06a}_field.log; exit 1; }
tail -1 gpurun_out/${TAG:-r06a}_field.log >> $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r06a}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-r06a}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-r06a}_tests.log >> $out
for n in 1250 2500 5000 6144 10000; do
  timeout -k 10 180 python -u tools/half_wide_sizes.py $n 30 >> $out 2> gpurun_out/${TAG:-r06a}_sizes_$n.err || { tail -20 gpurun_out/${TAG:-r06a}_sizes_$n.err; cat $out; exit 1; }
done
cat $out
