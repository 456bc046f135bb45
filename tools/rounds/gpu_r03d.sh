#!/bin/bash
# In-place exceptional additions: full GPU suite, then same-box A/B of the throughput kernel and
# the adversarial batches against the previous kernel (tools/variants/lib_old.so).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -5 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export SBFT_GV_LIB=$PWD/tools/variants/lib_old.so; else unset SBFT_GV_LIB; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
  done
done
unset SBFT_GV_LIB
for v in new old; do
  if [ $v = old ]; then export SBFT_GV_LIB=$PWD/tools/variants/lib_old.so; else unset SBFT_GV_LIB; fi
  timeout -k 10 300 python -c "
import json, torch, bench
from smartbft_amd import GpuVerifier
gv = GpuVerifier()
print('$v', json.dumps(bench.adversarial(gv, torch.device('cuda:0'))))
" > gpurun_out/adv_$v.log 2>&1 || { tail -5 gpurun_out/adv_$v.log; exit 1; }
  tail -1 gpurun_out/adv_$v.log | tee -a gpurun_out/ab.log
done
