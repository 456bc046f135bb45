#!/bin/bash
# u1*G comb windows of 22 bits (g22 = -DSBFT_GCOMB_W=22: 12 additions instead of 17, a 2.0 GB
# table built on first use) against the 16-bit default: parity tests on g22, then same-box A/B
# of config 2 (bench) and config 3/4 latency.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_g22.so timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g22_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g22_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur g22; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
    timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_${v}_$rep.log; exit 1; }
    python - $v gpurun_out/lat_${v}_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
echo done
