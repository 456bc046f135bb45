#!/bin/bash
# Round 5: half-kernel phases with the in-kernel clock (SBFT_HALF_PROBE build: s_memrealtime and
# s_memtime at every phase mark of workgroup 0).
mkdir -p gpurun_out
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_probe.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05k_probe.log 2>&1 || { tail -5 gpurun_out/r05k_probe.log; exit 1; }
grep half-probe gpurun_out/r05k_probe.log
