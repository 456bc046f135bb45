#!/bin/bash
# Coalescer pre-wake A/B (SBFT_CS_PREWAKE=0/1) for the stock config-4 fan-out, interleaved
# runs; then the init cost of the power-on self-test.
mkdir -p gpurun_out
out=gpurun_out/r02i_prewake_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plugin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/plugin_tests.log 2>&1 || { tail -5 gpurun_out/plugin_tests.log; exit 1; }
tail -1 gpurun_out/plugin_tests.log >> $out
for rep in 1 2; do
  for pw in 0 1; do
    for cfg in "66 50" "33 20" "22 15"; do
      set -- $cfg
      echo "prewake=$pw max=$1 wait=$2" >> $out
      SBFT_CS_PREWAKE=$pw timeout -k 10 120 tools/latency_harness quorum-gpu 66 200 $1 $2 >> $out 2>&1 || exit $?
    done
  done
  timeout -k 10 60 tools/latency_harness quorum-cpu 66 200 16 >> $out 2>&1 || exit $?
done
timeout -k 10 120 python tools/init_probe.py >> $out 2>&1 || exit $?
cat $out
