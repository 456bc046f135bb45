#!/bin/bash
# Halved-representative doubling (dh = -DSBFT_DBL_FORM=3, p29_dbl_h: 765 mads against 810)
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_dh.so timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dh_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dh_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur dh; do
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

cd /tmp 2>/dev/null; cd - >/dev/null
SBFT_GV_LIB=$V/lib_dh.so timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc_valu_dh -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined > gpurun_out/pmc_valu_dh.log 2>&1 || { tail -5 gpurun_out/pmc_valu_dh.log; exit 1; }
echo pmc done
