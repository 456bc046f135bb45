#!/bin/bash
# Registered-client VerifyProposal with the key lookups trailing the walk on a parse-pool thread:
# plugin/config GPU tests first, then the full suite, then config-3/4 latency x2 with a trace.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/plugin.log 2>&1
rc=$?; tail -3 gpurun_out/plugin.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_$rep.log 2>&1 || { tail -5 gpurun_out/lat_$rep.log; exit 1; }
  python - gpurun_out/lat_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(*[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
done
SBFT_VP_TRACE=1 timeout -k 10 300 python tools/latency_probe.py --calls 30 > gpurun_out/lat_trace.log 2>&1 || { tail -5 gpurun_out/lat_trace.log; exit 1; }
echo done
