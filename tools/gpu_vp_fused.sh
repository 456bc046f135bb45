#!/bin/bash
# VerifyProposal with the hash fused into the small-batch verify launch: parity tests, the
# config-3 latency A/B (SBFT_VP_SYNC=1 vs 0: stream sync after the payload copy, alternated), and the fused kernel timeline.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_configs.py tests/test_gpu_verify.py -m gpu -x -q --timeout 120 --timeout-method thread -k "framed or proposal or exceptional or config3 or consenter or sha256" > gpurun_out/fused_tests.log 2>&1 || { tail -15 gpurun_out/fused_tests.log; exit 1; }
tail -1 gpurun_out/fused_tests.log
for i in 1 2; do
  for f in 1 0; do
    SBFT_VP_SYNC=$f timeout -k 10 200 python tools/latency_probe.py --calls 100 > gpurun_out/lat_f$f.txt 2>&1 || { tail -5 gpurun_out/lat_f$f.txt; exit 1; }
    python - "$f" <<'PY'
import json, sys
d = json.loads(open('gpurun_out/lat_f%s.txt' % sys.argv[1]).read().strip().splitlines()[-1])
print('sync=%s' % sys.argv[1], {k: (v.get('p50_ms') if isinstance(v, dict) else v) for k, v in d.items()})
PY
  done
done | tee gpurun_out/fused_ab.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/vp_trace -o run --output-format csv -- python3 tools/latency_probe.py --calls 20 > gpurun_out/vp_trace.log 2>&1 || { tail -5 gpurun_out/vp_trace.log; exit 1; }
python3 tools/vp_timeline.py gpurun_out/vp_trace > gpurun_out/vp_timeline.txt && tail -16 gpurun_out/vp_timeline.txt
