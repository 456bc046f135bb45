#!/bin/bash
# Round 6: affine-sum join in both half-kernel forms (quad and pair mixed addition): half /
# exceptional / config / fixup suites, then same-box sizes against the general join (lib_g0).
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06o
out=gpurun_out/$T.txt; : > $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py tests/test_gpu_configs.py tests/test_gpu_fixup.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for n in 1250 5000 10000; do
  for g in g0 new; do
    if [ $g = new ]; then L=$PWD/smartbft_amd/libsbft_gpuverify.so; else L=$V/lib_$g.so; fi
    echo -n "$g " >> $out
    SBFT_GV_LIB=$L timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> $out 2> gpurun_out/${T}_${g}_$n.err || { tail -20 gpurun_out/${T}_${g}_$n.err; cat $out; exit 1; }
  done
done
cat $out
