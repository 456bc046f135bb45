#!/bin/bash
# Round 6: the split VerifyProposal's shares in the mapped-memory form (enqueue_framed_share):
# the split, config, framed and plugin suites, then the split path's host cost on one GPU.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06g
out=gpurun_out/$T.txt; : > $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_verify.py tests/test_gpu_plugin.py tests/test_gpu_faults.py tests/test_gpu_exceptional.py tests/test_gpu_keyed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for spec in "2500 2" "5000 4" "10000 8" "10000 2"; do
  set -- $spec
  timeout -k 10 300 python -u tools/split_probe.py $1 $2 100 >> $out 2> gpurun_out/${T}_probe_$1_$2.err || { tail -10 gpurun_out/${T}_probe_$1_$2.err; cat $out; exit 1; }
done
cat $out
