#!/bin/bash
# Coalesced config-4 fan-out tail: is the multi-ms p99 the job's CPU quota throttling the
# spinning followers? cgroup cpu.max / cpu.stat deltas per run, pre-wake on/off interleaved.
mkdir -p gpurun_out
out=gpurun_out/r03w_cs_tail.txt
{ echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')";
  echo "cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; } > $out
for rep in 1 2 3; do
  for pw in 1 0; do
    echo "prewake=$pw rep=$rep" >> $out
    SBFT_CS_PREWAKE=$pw timeout -k 10 120 tools/latency_harness quorum-gpu 66 400 66 50 2>/dev/null | grep '^{' >> $out || exit $?
  done
done
timeout -k 10 120 tools/latency_harness quorum-cpu 66 400 16 2>/dev/null | grep '^{' >> $out
cat $out
