#!/bin/bash
# Full GPU suite on this build (shared-reduction Y3 in the additions; VerifyProposal launches
# after the length walk and checks the format during the verify), then same-box A/Bs:
#   cur vs qg (-DSBFT_QTAB_GLOBAL=1: Q table in a per-lane contiguous workspace region instead of
#   lane-interleaved scratch) vs nomulsub (-DSBFT_MULSUB=0: two products + subtraction);
#   config-3/4 latency; FETCH_SIZE / WRITE_SIZE passes of cur and qg.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_qg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_exceptional.py -x -q --timeout 300 --timeout-method thread > gpurun_out/qg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/qg_tests.log; [ $rc -ne 0 ] && exit $rc
Q="--no-sha --no-latency --no-host-path --no-cpu-baseline --steps 20 --warmup 5"
for rep in 1 2; do
  for v in cur qg nomulsub; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python bench.py $Q > gpurun_out/ab_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/ab_${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log) $(grep -o '"pipelined": {"value": [0-9.]*' gpurun_out/ab_${v}_$rep.log)" | tee -a gpurun_out/ab.log
  done
done
unset SBFT_GV_LIB
for rep in 1 2; do
  timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_$rep.log 2>&1 || { tail -5 gpurun_out/lat_$rep.log; exit 1; }
  python - gpurun_out/lat_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(*[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
done
SBFT_VP_TRACE=1 timeout -k 10 300 python tools/latency_probe.py --calls 30 > gpurun_out/lat_trace.log 2>&1 || { tail -5 gpurun_out/lat_trace.log; exit 1; }
P="--steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-sha --no-host-path --no-pipelined"
for v in cur qg; do
  if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${v}_$c -o run --output-format csv -- python3 bench.py $P > gpurun_out/pmc_${v}_$c.log 2>&1 || { tail -3 gpurun_out/pmc_${v}_$c.log; exit 1; }
  done
done
echo done
