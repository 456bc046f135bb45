#!/bin/bash
# Round 5: phase times of the registered-client keyed kernel (p256_verify_keyed_lanes_kernel<true>)
# on a 10k config-3 proposal (tools/keyed_lanes_probe.py, lib_kprobe = -DSBFT_KEYED_PROBE).
mkdir -p gpurun_out
SBFT_GV_LIB=$PWD/tools/variants/lib_kprobe.so timeout -k 10 300 python tools/keyed_lanes_probe.py > gpurun_out/r05ai_probe.log 2>&1 || { tail -5 gpurun_out/r05ai_probe.log; exit 1; }
grep keyed-probe gpurun_out/r05ai_probe.log | tail -24
