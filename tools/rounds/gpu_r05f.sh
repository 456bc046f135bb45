#!/bin/bash
# Round 5: the half kernel's rare square test gated on valid, non-fallback tuples: the half-kernel
# GPU tests, then worst-case batches (bench.adversarial) and config-3 latency, cur vs base.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py tests/test_gpu_configs.py tests/test_gpu_fixup.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1 || { tail -20 gpurun_out/r05f_tests.log; exit 1; }
tail -2 gpurun_out/r05f_tests.log
out=gpurun_out/r05f_ab.txt; : > $out
for rep in 1 2; do
  for v in cur base; do
    case $v in cur) unset SBFT_GV_LIB;; *) export SBFT_GV_LIB=$V/lib_$v.so;; esac
    timeout -k 10 300 python tools/adv_probe.py > gpurun_out/r05f_adv_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05f_adv_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep '^{' gpurun_out/r05f_adv_${v}_$rep.log | tail -1)" >> $out
  done
done
unset SBFT_GV_LIB
cat $out
