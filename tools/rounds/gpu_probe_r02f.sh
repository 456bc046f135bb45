#!/bin/bash
# batcher/coalescer tests + quorum latency sweep
mkdir -p gpurun_out
true

rm -f gpurun_out/quorum_sweep2.log
for w in 20 50 150; do timeout -k 10 120 tools/latency_harness quorum-gpu 66 300 66 $w >> gpurun_out/quorum_sweep2.log 2>&1 || exit $?; done
timeout -k 10 120 tools/latency_harness quorum-cpu 66 300 16 >> gpurun_out/quorum_sweep2.log 2>&1
grep -v amdgpu.ids gpurun_out/quorum_sweep2.log
timeout -k 10 120 tools/latency_harness quorum-gpu 66 300 0 0 >> gpurun_out/quorum_sweep2.log 2>&1; timeout -k 10 120 tools/latency_harness proposal-cpu 10000 20 16 >> gpurun_out/quorum_sweep2.log 2>&1; grep -v amdgpu.ids gpurun_out/quorum_sweep2.log | tail -2
