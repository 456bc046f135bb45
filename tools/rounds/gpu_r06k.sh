#!/bin/bash
# Round 6: phase times (SBFT_HALF_PROBE build) of the wide half kernel (quad ladder v3) against the
# four-lane one at 5,000 and 1,250 requests: where the pre-ladder and join time goes now.
mkdir -p gpurun_out
V=$PWD/tools/variants
out=gpurun_out/r06k_probe.txt; : > $out
for spec in "5000 1" "5000 0" "1250 1" "1250 0"; do
  set -- $spec
  echo "== n=$1 wide=$2" >> $out
  HALF_PROBE_N=$1 HALF_PROBE_WIDE=$2 SBFT_GV_LIB=$V/lib_probe.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/r06k_$1_$2.log 2>&1 || { tail -5 gpurun_out/r06k_$1_$2.log; exit 1; }
  grep half-probe gpurun_out/r06k_$1_$2.log | tail -8 >> $out
done
cat $out
