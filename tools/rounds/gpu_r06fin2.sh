#!/bin/bash
# Round 6, final tree (quad table build, helper pairs): the whole GPU suite, smoke, the default bench line,
# kernel-trace stats of the bench command and of the half kernels at share sizes.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06fin2
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
V=$PWD/tools/variants
for n in 1250 5000; do
  for g in new q0 new q0; do
    if [ $g = new ]; then L=$PWD/smartbft_amd/libsbft_gpuverify.so; else L=$V/lib_$g.so; fi
    echo -n "$g " >> gpurun_out/${T}_sizes.txt
    SBFT_GV_LIB=$L timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> gpurun_out/${T}_sizes.txt 2> gpurun_out/${T}_${g}_$n.err || { tail -20 gpurun_out/${T}_${g}_$n.err; exit 1; }
  done
done
timeout -k 10 600 python -u tools/parity_sweep.py --n 500000 --seed 2607 --threads 16 --hash 100000 --framed 20000 > gpurun_out/${T}_sweep.log 2>&1 || { tail -20 gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sizes.txt
tail -c 1200 gpurun_out/${T}_sweep.log
