#!/bin/bash
# Config-4 stock fan-out (66 concurrent VerifyConsenterSig calls per decision) with the
# zero-copy keyed path on four lanes (own stream + mapped buffer each): coalescer window sweep.
# Args of latency_harness quorum-gpu: CALLERS DECISIONS COALESCE_MAX COALESCE_WAIT_US.
mkdir -p gpurun_out
out=gpurun_out/r02h_quorum_sweep_slack.txt
: > $out
for cfg in "66 50" "66 30" "66 20" "33 15" "22 15" "22 10" "16 10" "11 8"; do
  set -- $cfg
  echo "max=$1 wait=$2" >> $out
  timeout -k 10 120 tools/latency_harness quorum-gpu 66 200 $1 $2 >> $out 2>&1 || exit $?
done
timeout -k 10 60 tools/latency_harness quorum-cpu 66 200 16 >> $out 2>&1 || exit $?
timeout -k 10 60 tools/latency_harness quorum-batch 67 200 >> $out 2>&1 || exit $?
cat $out
