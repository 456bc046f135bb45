mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plugin.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vp_tests.log 2>&1 || { tail -5 gpurun_out/vp_tests.log; exit 1; }
tail -1 gpurun_out/vp_tests.log
timeout -k 10 200 python tools/vp_breakdown.py > gpurun_out/vp_breakdown.txt 2>&1 || exit 1
SBFT_VP_TRACE=1 timeout -k 10 200 python tools/latency_probe.py --calls 100 > gpurun_out/lat_probe.txt 2> gpurun_out/lat_trace.txt || exit 1
cat gpurun_out/vp_breakdown.txt; python - <<'PY'
import json
d=json.loads(open('gpurun_out/lat_probe.txt').read().strip().splitlines()[-1])
print({k: (v.get('p50_ms') if isinstance(v, dict) else v) for k, v in d.items()})
PY
tail -5 gpurun_out/lat_trace.txt
