#!/bin/bash
# Round 6, final tree: a split VerifyProposal's cost on one GPU with the quad-table wide kernel
# (tools/split_probe.py: 2,500 requests over 2 slots against 1,250 on one slot; K slots stand in for
# K GPUs), and config 3 (10k) on one slot for reference.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06ae
out=gpurun_out/$T.txt; : > $out
for spec in "2500 2" "2500 2" "10000 2"; do
  set -- $spec
  timeout -k 10 300 python -u tools/split_probe.py $1 $2 100 >> $out 2> gpurun_out/${T}_probe_$1_$2.err || { tail -10 gpurun_out/${T}_probe_$1_$2.err; cat $out; exit 1; }
done
cat $out
