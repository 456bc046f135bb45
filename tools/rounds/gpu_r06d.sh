#!/bin/bash
# Round 6: v3 quad forms (fused DPP selects): unit + half suites, kernel times at share sizes,
# the torch-free config-2 harness, and the split / config suites (default min_split now splits 10k).
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06d
out=gpurun_out/$T.txt; : > $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for n in 1250 2500 5000 10000; do
  timeout -k 10 180 python -u tools/half_wide_sizes.py $n 30 >> $out 2> gpurun_out/${T}_sizes_$n.err || { tail -20 gpurun_out/${T}_sizes_$n.err; cat $out; exit 1; }
done
timeout -k 10 300 tools/config2_harness 1000000 20 3 >> $out 2> gpurun_out/${T}_c2.err || { tail -20 gpurun_out/${T}_c2.err; cat $out; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_split.log 2>&1 || { tail -30 gpurun_out/${T}_split.log; cat $out; exit 1; }
tail -1 gpurun_out/${T}_split.log >> $out
cat $out  # (more below)
timeout -k 10 300 tools/latency_harness quorum-hook 67 66 200 2 > gpurun_out/${T}_hook.json 2> gpurun_out/${T}_hook.err || { tail -5 gpurun_out/${T}_hook.err; exit 1; }
timeout -k 10 300 tools/latency_harness proposal-phases 10000 200 0 > gpurun_out/${T}_vp0.json 2> gpurun_out/${T}_vp0.err || { tail -5 gpurun_out/${T}_vp0.err; exit 1; }
timeout -k 10 300 tools/latency_harness proposal-phases 10000 200 1 > gpurun_out/${T}_vp1.json 2> gpurun_out/${T}_vp1.err || { tail -5 gpurun_out/${T}_vp1.err; exit 1; }
for b in gpu cpu-batched cpu; do
  timeout -k 10 300 tools/latency_harness quorum-pipe 2 200 $b > gpurun_out/${T}_pipe_$b.json 2> gpurun_out/${T}_pipe_$b.err || { tail -5 gpurun_out/${T}_pipe_$b.err; exit 1; }
done
cat gpurun_out/${T}_hook.json gpurun_out/${T}_vp0.json gpurun_out/${T}_vp1.json gpurun_out/${T}_pipe_*.json
