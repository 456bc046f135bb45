#!/bin/bash
# Round 6: the payload-copy helper pinned to the NUMA node of the GPU (numa), to the caller's L3 domain (l3) or not (0):
# (0): VerifyProposal phases (copy start / return from the call's start), generic and registered,
# interleaved; the CPU topology beside it.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06ab
out=gpurun_out/$T.txt; : > $out
lscpu | grep -i "model name\|L3\|NUMA node(s)\|^CPU(s)" >> $out
cat /sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list >> $out 2>&1
for rep in 1 2 3; do
for mode in "0 numa" "0 0" "0 l3" "1 numa" "1 0"; do
  set -- $mode
  echo "== registered=$1 affinity=$2" >> $out
  SBFT_HELPER_AFFINITY=$2 timeout -k 10 300 tools/latency_harness proposal-phases 10000 200 $1 >> $out 2> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; cat $out; exit 1; }
done
done
cat $out
