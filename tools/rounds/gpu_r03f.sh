#!/bin/bash
# Full suite (final check by zero tests, SHA clamp fast path), then same-box A/Bs:
#   table probe (the ladder reads one fixed Q-table entry: the cost of the table loads);
#   SHA-256 with and without the DMA clamp (config-5 hash kernel, 1M messages).
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -4 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
fi
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur tprobe; do
    if [ $v = cur ]; then unset SBFT_GV_LIB SBFT_GV_SELFTEST; else export SBFT_GV_LIB=$PWD/tools/variants/lib_$v.so SBFT_GV_SELFTEST=0; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
  done
done
for rep in 1 2; do
  for v in cur shanoclamp; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$PWD/tools/variants/lib_$v.so; fi
    timeout -k 10 300 python -c "
import json, torch, bench
from smartbft_amd import GpuVerifier
gv = GpuVerifier()
r = bench.sha_config5(gv, torch.device('cuda:0'), 1048576, e2e_msgs=16384)
print('$v $rep', r['value'], r['avg_kernel_ms'], r['roofline'].get('frac_of_valu_ceiling'), r['hash_verify']['value'], r['hash_verify']['mismatches'])
" > gpurun_out/sha_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/sha_${v}_$rep.log; exit 1; }
    tail -1 gpurun_out/sha_${v}_$rep.log | tee -a gpurun_out/ab.log
  done
done
