#!/bin/bash
# VerifyProposal verdicts written by the kernels straight to mapped host memory (no D2H copy):
# GPU plugin/config/split tests, then config-3 latency A/B against prevhost (the previous host
# code, same kernels), and the same probe with HSA_ENABLE_SDMA=0 (copies as blit kernels on the
# compute queue: measures the copy-engine hand-off in front of the verify launch).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
V=$PWD/tools/variants
for rep in 1 2; do
  for v in cur prevhost nosdma; do
    unset SBFT_GV_LIB HSA_ENABLE_SDMA
    [ $v = prevhost ] && export SBFT_GV_LIB=$V/lib_prevhost.so
    [ $v = nosdma ] && export HSA_ENABLE_SDMA=0
    timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_${v}_$rep.log; exit 1; }
    python - $v gpurun_out/lat_${v}_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
unset HSA_ENABLE_SDMA SBFT_GV_LIB
SBFT_VP_TRACE=1 timeout -k 10 300 python tools/latency_probe.py --calls 30 > gpurun_out/lat_trace.log 2>&1 || { tail -5 gpurun_out/lat_trace.log; exit 1; }
echo done
