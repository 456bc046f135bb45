#!/bin/bash
# Fix-up kernel launched only when the verify kernel raised the mapped flag (VerifyProposal):
# the exceptional/plugin/config tests first (quad mode exercises the flag), then the full suite,
# then config-3/4 latency x2 and a kernel trace of the latency probe.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_exceptional.py -x -v --timeout 120 --timeout-method thread > gpurun_out/exc.log 2>&1
rc=$?; tail -8 gpurun_out/exc.log; [ $rc -ne 0 ] && exit $rc
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
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lat_prof -o run --output-format csv -- python3 tools/latency_probe.py --calls 50 > gpurun_out/lat_prof.log 2>&1 || { tail -3 gpurun_out/lat_prof.log; exit 1; }
echo done
