#!/bin/bash
# Round checkpoint (tests, smoke, bench, rocprofv3 stats + PMC passes of the verify kernel), then
# the throughput kernel with u2 in radix 2^5 (w5 = -DSBFT_TQWIN=5: 16-entry Q table, 51 additions
# instead of 64): its parity tests and an interleaved same-box A/B against this build.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
mv $V/lib_w5.so /tmp/lib_w5.so 2>/dev/null   # keep the round's variant loop off it
SKIP_PROF= bash tools/gpu_round.sh || exit $?
SBFT_GV_LIB=/tmp/lib_w5.so timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/w5_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur w5; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=/tmp/lib_w5.so; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
  done
done
echo done
