#!/bin/bash
# Round 6, final tree: the whole GPU suite, smoke, the default bench line, and rocprofv3
# kernel-trace stats of the bench command and of the half kernels at share sizes.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
timeout -s KILL 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o st --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_bench_prof.log 2> gpurun_out/${T}_bench_prof.err || { tail -5 gpurun_out/${T}_bench_prof.err; exit 1; }
for n in 1250 5000; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_half_$n -o st --output-format csv -- python3 tools/half_wide_sizes.py $n 20 >> gpurun_out/${T}_half.txt 2> gpurun_out/${T}_half_$n.err || { tail -5 gpurun_out/${T}_half_$n.err; exit 1; }
done
find gpurun_out/${T}_* -name "*kernel_stats.csv" | sort
tail -c 1500 gpurun_out/${T}_bench.log
