#!/bin/bash
# Round 5: where the half kernel's table conversion spends its time under a full batch (probe build
# with marks after the first and the fourth of the seven conversion steps; columns: inputs, chain,
# inverse, conversion 1, conversion 4, tables, barrier 1, ladder) and the in-kernel clock.
mkdir -p gpurun_out
V=$PWD/tools/variants
SBFT_GV_LIB=$V/lib_probetab.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r05l_probe.log 2>&1 || { tail -5 gpurun_out/r05l_probe.log; exit 1; }
grep half-probe gpurun_out/r05l_probe.log
