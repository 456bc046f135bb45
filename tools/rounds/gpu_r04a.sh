#!/bin/bash
# Round 4: the half-size-scalar latency kernel (p256_verify_half_kernel). Its GPU tests, then
# config-3/4 latency A/B against the pair kernel (SBFT_GV_HALF_MAX=-1), interleaved, then a
# kernel trace of the latency probe. Stops at the first failing step.
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${PYTEST_K:-"half or config3 or framed or golden or fault or bounds"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04a_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04a_tests.log | head -30; exit $rc; }
for rep in 1 2; do
  for v in pair half; do
    if [ $v = pair ]; then export SBFT_GV_HALF_MAX=-1; else unset SBFT_GV_HALF_MAX; fi
    timeout -k 10 300 python tools/latency_probe.py --calls 200 > gpurun_out/r04a_lat_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/r04a_lat_${v}_$rep.log; exit 1; }
    python - $v gpurun_out/r04a_lat_${v}_$rep.log <<'PY' | tee -a gpurun_out/r04a_lat.log
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], *[(k, d[k]["p50_ms"], d[k]["p99_ms"]) for k in d if isinstance(d[k], dict) and "p50_ms" in d[k]])
PY
  done
done
unset SBFT_GV_HALF_MAX
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04a_prof -o lat -- python3 $GRAFT_REPO_ROOT/tools/latency_probe.py --calls 50 > $GRAFT_REPO_ROOT/gpurun_out/r04a_prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; find gpurun_out/r04a_prof -name "*kernel_stats.csv" | head -3; exit $rc
