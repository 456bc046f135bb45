#!/bin/bash
# Config-4 processCommits hook: batch workers armed for the whole collection (SBFT_HOOK_ARM=1)
# against sleeping until a batch is posted (0), interleaved on one box, with the OpenSSL quorum
# at 16 threads and at one thread per vote, and the pipelined-decisions mode both ways.
mkdir -p gpurun_out
export TMPDIR=/tmp
H=tools/latency_harness
out=gpurun_out/r04h_hook_arm.txt
: > $out
for rep in 1 2 3; do
  for arm in 0 1; do
    echo "== hook arm=$arm rep=$rep" >> $out
    SBFT_HOOK_ARM=$arm timeout -k 10 120 $H quorum-hook 67 66 400 2 >> $out 2>&1 || exit 1
  done
  echo "== cpu16 rep=$rep" >> $out
  timeout -k 10 120 $H quorum-cpu 66 400 16 >> $out 2>&1 || exit 1
  echo "== cpu66 rep=$rep" >> $out
  timeout -k 10 120 $H quorum-cpu 66 400 66 >> $out 2>&1 || exit 1
done
for arm in 0 1; do
  echo "== pipe gpu arm=$arm" >> $out
  SBFT_HOOK_ARM=$arm timeout -k 10 120 $H quorum-pipe 2 300 gpu >> $out 2>&1 || exit 1
done
echo "== pipe cpu" >> $out
timeout -k 10 120 $H quorum-pipe 2 300 cpu >> $out 2>&1 || exit 1
cat $out
