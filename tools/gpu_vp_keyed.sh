#!/bin/bash
# VerifyProposal with registered clients on the overlapped keyed launch: parity tests, then
# config-3 latency (both variants) twice.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "proposal or config3" > gpurun_out/keyed_tests.log 2>&1 || { tail -15 gpurun_out/keyed_tests.log; exit 1; }
tail -1 gpurun_out/keyed_tests.log
for i in 1 2; do
  timeout -k 10 200 python tools/latency_probe.py --calls 100 > gpurun_out/lat_k$i.txt 2>&1 || { tail -5 gpurun_out/lat_k$i.txt; exit 1; }
  python - "$i" <<'PY'
import json, sys
d = json.loads(open('gpurun_out/lat_k%s.txt' % sys.argv[1]).read().strip().splitlines()[-1])
print({k: (v.get('p50_ms') if isinstance(v, dict) else v) for k, v in d.items()})
PY
done | tee gpurun_out/keyed_lat.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/vp_trace -o run --output-format csv -- python3 tools/latency_probe.py --calls 20 > gpurun_out/vp_trace.log 2>&1 || { tail -5 gpurun_out/vp_trace.log; exit 1; }
python3 tools/vp_timeline.py gpurun_out/vp_trace > gpurun_out/vp_timeline.txt && tail -12 gpurun_out/vp_timeline.txt
