#!/bin/bash
# Round 6: rocprofv3 kernel-trace stats of the four-lane and wide half kernels at share sizes
# (tools/half_wide_sizes.py, both kernels interleaved in one process per size), and of the
# default bench command (the headline's p256_verify_kernel and the latency legs' kernels).
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06f
out=gpurun_out/$T.txt; : > $out
for n in 1250 2500 5000; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_$n -o st --output-format csv -- python3 tools/half_wide_sizes.py $n 20 >> $out 2> gpurun_out/${T}_$n.err || { tail -5 gpurun_out/${T}_$n.err; exit 1; }
done
timeout -s KILL 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_bench -o st --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
find gpurun_out/${T}_* -name "*kernel_stats.csv" | sort >> $out
cat $out
