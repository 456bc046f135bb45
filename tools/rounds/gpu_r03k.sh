#!/bin/bash
# Products with addends (X3 = al^2 - 4 b2, Y3 = al t0 - 8 g^2, the additions' X3 = r^2 - HHH - 2V
# folded inside the Montgomery pass): full GPU suite on this build, then same-box A/Bs against
#   nofuse (-DSBFT_DBL_FORM=1 -DSBFT_ADD_FUSED=0 -DSBFT_PAIR_FUSED=0: the previous kernels) and
#   noaddf (-DSBFT_ADD_FUSED=0: fused doubling only),
# config-3/4 latency for cur and nofuse, and the SQ_INSTS_VALU pass of cur.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_nofuse.so timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py -x -q --timeout 300 --timeout-method thread > gpurun_out/nofuse_tests.log 2>&1
rc=$?; tail -2 gpurun_out/nofuse_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur nofuse noaddf; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
  done
done
for rep in 1 2; do
  for v in cur nofuse; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_${v}_$rep.log; exit 1; }
    python - $v gpurun_out/lat_${v}_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
unset SBFT_GV_LIB
P="--steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_valu -o run --output-format csv -- python3 bench.py $P > gpurun_out/pmc_valu.log 2>&1 || { tail -3 gpurun_out/pmc_valu.log; exit 1; }
echo done
