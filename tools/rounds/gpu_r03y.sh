#!/bin/bash
# mul_sub on one accumulator (mc = -DSBFT_MULSUB_CHAIN=1: no 64-bit add per column in the
# additions' Y3) against the two-accumulator default: parity on mc, then same-box config-2 A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_mc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mc_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2 3; do
  for v in cur mc; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab_mc.log
  done
done
