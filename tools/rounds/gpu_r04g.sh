#!/bin/bash
# Throughput-kernel occupancy A/B: the current 4-waves/SIMD build against
# 5 waves (-DSBFT_VERIFY_WAVES=5: 96 VGPRs, 1,184 B of scratch per lane) and 3 waves (168 VGPRs).
# Sizes: BASELINE's 1,000,000 and 1,310,720 (a whole number of resident rounds at 4 AND 5 waves,
# so wave quantisation does not favour either). Parity of the 5-wave build first.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_w5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_w5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04g_w5_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --no-pipelined --steps 20 --warmup 5"
for rep in 1 2; do
  for n in 1000000 1310720; do
    for v in cur w5 w3; do
      if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
      timeout -k 10 200 python bench.py $Q --n $n > gpurun_out/r04g_${v}_${n}_$rep.log 2>&1 || { tail -3 gpurun_out/r04g_${v}_${n}_$rep.log; exit 1; }
      echo "$v n=$n rep=$rep $(grep -o '"value": [0-9.]*' gpurun_out/r04g_${v}_${n}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/r04g_${v}_${n}_$rep.log)" | tee -a gpurun_out/r04g_ab.log
    done
  done
done
echo done
