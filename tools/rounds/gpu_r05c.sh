#!/bin/bash
# Round 5, VERDICT r04 #3: config 4 CPU per decision. Interleaved A/B on one box:
#   old = round-4 waits (engine zero-copy wait spins to the end, collector spins, workers spin 50 us)
#   new = bounded spins then blocking waits (defaults)
mkdir -p gpurun_out
export TMPDIR=/tmp
H=tools/latency_harness
OLD="SBFT_ZC_SPIN_US=100000000 SBFT_HOOK_COLLECT_SPIN_US=100000000 SBFT_HOOK_WORKER_SPIN_US=50 SBFT_PIPE_DELIVERERS=0"
out=gpurun_out/r05c_config4.txt; : > $out
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then E="$OLD"; else E=""; fi
    r=$(env $E timeout -k 10 120 $H quorum-pipe 2 200 gpu) || exit $?
    echo "$rep $v pipe-gpu $r" >> $out
    r=$(env $E timeout -k 10 120 $H quorum-hook 67 66 400 2) || exit $?
    echo "$rep $v hook $r" >> $out
  done
  r=$(timeout -k 10 120 $H quorum-pipe 2 200 cpu) || exit $?
  echo "$rep new pipe-cpu $r" >> $out
  r=$(env SBFT_HOOK_COLLECT_SPIN_US=100000000 SBFT_PIPE_DELIVERERS=0 timeout -k 10 120 $H quorum-pipe 2 200 cpu) || exit $?
  echo "$rep old pipe-cpu $r" >> $out
  echo "rep $rep done"
done
cat $out
