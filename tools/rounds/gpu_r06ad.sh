#!/bin/bash
# Round 6: the quad table build on the rebuilt shipped library (helper option off) against the
# pair build (lib_q0) and with the helper on lane pairs (lib_hp1): HIP-event sizes, interleaved;
# half suites on lib_hp1.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06ad
out=gpurun_out/$T.txt; : > $out
SBFT_GV_LIB=$V/lib_hp1.so timeout -k 10 900 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for n in 1250 5000; do
  for g in new q0 hp1 new q0 hp1; do
    if [ $g = new ]; then L=$PWD/smartbft_amd/libsbft_gpuverify.so; else L=$V/lib_$g.so; fi
    echo -n "$g " >> $out
    SBFT_GV_LIB=$L timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> $out 2> gpurun_out/${T}_${g}_$n.err || { tail -20 gpurun_out/${T}_${g}_$n.err; cat $out; exit 1; }
  done
done
cat $out
