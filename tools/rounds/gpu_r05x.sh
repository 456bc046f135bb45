#!/bin/bash
# Round 5: s^-1 from the host for small zero-copy keyed batches (SBFT_KEYED_HOST_SINV_MAX, default
# 96) against the kernel's own inversion (=0): keyed / proposal / plugin / fault / runtime GPU
# tests on the new default, then config-4 latencies interleaved on one box.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_plugin.py tests/test_gpu_configs.py tests/test_gpu_faults.py tests/test_gpu_runtime.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05x_tests.log 2>&1 || { tail -15 gpurun_out/r05x_tests.log; exit 1; }
tail -2 gpurun_out/r05x_tests.log
SBFT_KEYED_HOST_SINV_MAX=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05x_tests_dev.log 2>&1 || { tail -15 gpurun_out/r05x_tests_dev.log; exit 1; }
echo "device-inversion keyed tests:"; tail -1 gpurun_out/r05x_tests_dev.log
out=gpurun_out/r05x_ab.txt; : > $out
for rep in 1 2 3; do
  for v in host dev; do
    case $v in host) unset SBFT_KEYED_HOST_SINV_MAX;; dev) export SBFT_KEYED_HOST_SINV_MAX=0;; esac
    timeout -k 10 240 python tools/latency_probe.py --calls 200 > gpurun_out/r05x_${v}_$rep.log 2>&1 || { tail -3 gpurun_out/r05x_${v}_$rep.log; exit 1; }
    python3 - gpurun_out/r05x_${v}_$rep.log $v $rep >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
q = d["commit_quorum_n100"]; h = d["commit_quorum_n100_hook"]; c = d["commit_quorum_n100_concurrent_singles"]["coalesced"]
pp = d["commit_quorum_n100_pipelined"]["gpu"]
print(sys.argv[2], "rep", sys.argv[3], "batch67 p50", q["c_harness"]["p50_ms"], "| hook p50/p99", h["p50_ms"], h["p99_ms"],
      "| singles coalesced p50/p99", c["p50_ms"], c["p99_ms"], "| pipelined", pp["decisions_per_s"], "| vp10k", d["verify_proposal_10k"]["p50_ms"])
PY
  done
done
unset SBFT_KEYED_HOST_SINV_MAX
cat $out
