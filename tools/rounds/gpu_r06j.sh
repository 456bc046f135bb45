#!/bin/bash
# Round 6: the wide kernel's join as a quad mixed addition (the helper makes (v u1) G affine): the
# half / exceptional / config suites, then the kernel at share sizes against the four-lane form.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06j}
out=gpurun_out/$T.txt; : > $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py tests/test_gpu_configs.py tests/test_gpu_fixup.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for n in 1250 2500 5000; do
  timeout -k 10 180 python -u tools/half_wide_sizes.py $n 30 >> $out 2> gpurun_out/${T}_sizes_$n.err || { tail -20 gpurun_out/${T}_sizes_$n.err; cat $out; exit 1; }
done
cat $out
