#!/bin/bash
# GPU-box check: parity tests, then (only if they ended without a crash) a quick timing run.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=5 > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/quick_bench.py ${QB_N:-262144} > gpurun_out/qb.log 2>&1
rc2=$?
cat gpurun_out/qb.log
exit $rc2
