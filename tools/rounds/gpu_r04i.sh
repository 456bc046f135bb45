#!/bin/bash
# Config-4 A/B, second pass: batch workers armed (SBFT_HOOK_ARM=1) or not, 5 interleaved reps of
# the hook and 3 of the pipelined mode, against quorum-vote-cpu (the hook's own scenario on the
# CPU: same releases, bad vote every 10th decision) at 16 threads and at one thread per vote.
mkdir -p gpurun_out
export TMPDIR=/tmp
H=tools/latency_harness
out=gpurun_out/r04i_hook_arm.txt
: > $out
for rep in 1 2 3 4 5; do
  for arm in 0 1; do
    echo "== hook arm=$arm rep=$rep" >> $out
    SBFT_HOOK_ARM=$arm timeout -k 10 120 $H quorum-hook 67 66 400 2 >> $out 2>&1 || exit 1
  done
  echo "== vote-cpu16 rep=$rep" >> $out
  timeout -k 10 120 $H quorum-vote-cpu 67 66 400 16 >> $out 2>&1 || exit 1
  echo "== vote-cpu67 rep=$rep" >> $out
  timeout -k 10 120 $H quorum-vote-cpu 67 66 400 67 >> $out 2>&1 || exit 1
done
for rep in 1 2 3; do
  for arm in 0 1; do
    echo "== pipe gpu arm=$arm rep=$rep" >> $out
    SBFT_HOOK_ARM=$arm timeout -k 10 120 $H quorum-pipe 2 300 gpu >> $out 2>&1 || exit 1
  done
done
echo "== pipe cpu" >> $out
timeout -k 10 120 $H quorum-pipe 2 300 cpu >> $out 2>&1 || exit 1
cat $out
