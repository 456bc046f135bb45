#!/bin/bash
# Correctness first, then A/B the verify-kernel variants under tools/variants/.
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=3 > gpurun_out/tests.log 2>&1
rc=$?; tail -15 gpurun_out/tests.log; [ $rc -gt 1 ] && exit $rc
for lib in tools/variants/*.so; do
  [ -e "$lib" ] || continue
  echo "== $lib"
  SBFT_GV_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path > gpurun_out/var_$(basename $lib).log 2>&1 || { echo "fail $?"; tail -5 gpurun_out/var_$(basename $lib).log; exit 1; }
  python -c "import json,sys; j=json.loads(open('gpurun_out/var_$(basename $lib).log').read().strip().splitlines()[-1]); print(j['value'], j['roofline']['avg_kernel_ms'], j['parity'])"
done
