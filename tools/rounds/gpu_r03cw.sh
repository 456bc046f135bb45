#!/bin/bash
# u1*G on its own wavefront in the framed pair kernel (cw = -DSBFT_PAIR_COMB_WAVE=1): the whole
# GPU suite on cw, then config-3/4 latency A/B against the default, interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_cw.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cw_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/cw_tests.log | head -20; exit $rc; }
for rep in 1 2 3; do
  for v in cur cw; do
    if [ $v = cur ]; then unset SBFT_GV_LIB; else export SBFT_GV_LIB=$V/lib_$v.so; fi
    timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/lat_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/lat_${v}_$rep.log; exit 1; }
    python - $v gpurun_out/lat_${v}_$rep.log <<'PY' | tee -a gpurun_out/lat_cw.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
