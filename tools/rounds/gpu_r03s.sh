#!/bin/bash
# Registered-client VerifyProposal: how far ahead the key-map slots are prefetched during the
# lookups after the walk (SBFT_KEY_AHEAD = 8, the default, vs 16, 32, 64), config-3/4 latency.
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for a in 8 16 32 64; do
    SBFT_KEY_AHEAD=$a timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_${a}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_${a}_$rep.log; exit 1; }
    python - $a gpurun_out/lat_${a}_$rep.log <<'PY' | tee -a gpurun_out/lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("ahead", sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
SBFT_VP_TRACE=1 SBFT_KEY_AHEAD=32 timeout -k 10 300 python tools/latency_probe.py --calls 30 > gpurun_out/lat_trace.log 2>&1 || { tail -5 gpurun_out/lat_trace.log; exit 1; }
echo done
