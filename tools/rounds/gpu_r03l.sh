#!/bin/bash
# Queue launch of the throughput kernel (resident grid, waves pull 64-tuple chunks): the verify
# and exceptional GPU tests on this build, then same-box A/B:
#   queue  = this build (default: queue launch above one resident round)
#   static = this build with SBFT_VERIFY_QUEUE=0 (spread / per-thread grids)
#   prev   = the previous commit's p256_verify.hip (no verify_lane loop) with the same objects
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V=$PWD/tools/variants
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in queue static prev; do
    unset SBFT_GV_LIB SBFT_VERIFY_QUEUE
    [ $v = static ] && export SBFT_VERIFY_QUEUE=0
    [ $v = prev ] && export SBFT_GV_LIB=$V/lib_prev.so
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
  done
done
echo done
