#!/bin/bash
# Full suite, then config-3/4 latency with the proposal parse on 1, 3 and 4 threads (same box),
# and one SBFT_VP_TRACE sample of the phases (copy staging / parse / wait / launch+sync).
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -4 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for t in 1 3 4; do
    SBFT_PARSE_THREADS=$t timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_t${t}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_t${t}_$rep.log; exit 1; }
    python - "$t" "$rep" gpurun_out/lat_t${t}_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print("threads", sys.argv[1], "rep", sys.argv[2], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
SBFT_VP_TRACE=1 SBFT_PARSE_TRACE=1 timeout -k 10 300 python tools/latency_probe.py --calls 30 > gpurun_out/lat_trace.log 2>&1 || { tail -5 gpurun_out/lat_trace.log; exit 1; }
tail -3 gpurun_out/lat_trace.log
