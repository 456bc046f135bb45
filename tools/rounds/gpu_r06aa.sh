#!/bin/bash
# Round 6: the payload-copy helper in the caller's L3 domain (SBFT_HELPER_L3=1, an earlier form of
# SBFT_HELPER_AFFINITY=l3) against none: VerifyProposal phases (copy start / return from the call's start),
# interleaved; the CPU topology beside it.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06aa
out=gpurun_out/$T.txt; : > $out
lscpu | grep -i "model name\|L3\|NUMA node(s)\|^CPU(s)" >> $out
cat /sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list >> $out 2>&1
for rep in 1 2 3; do
for mode in "0 1" "0 0" "1 1" "1 0"; do
  set -- $mode
  echo "== registered=$1 helper_l3=$2" >> $out
  SBFT_HELPER_L3=$2 timeout -k 10 300 tools/latency_harness proposal-phases 10000 200 $1 >> $out 2> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; cat $out; exit 1; }
done
done
cat $out
