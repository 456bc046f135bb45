#!/bin/bash
# Round 6: the wide form's Q tables built on the quad (build_q_table_quad_w, 39 product steps
# instead of 54): half / exceptional / config / fixup / verify / field suites on the new build,
# phase probes (q1 new, q0 the pair build) and HIP-event sizes (new vs lib_q0), interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06ac
out=gpurun_out/$T.txt; : > $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_verify.py tests/test_gpu_configs.py tests/test_gpu_fixup.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for n in 1250 5000; do
for h in q0 q1 q0 q1; do
  echo "== probe n=$n $h" >> $out
  HALF_PROBE_N=$n HALF_PROBE_WIDE=1 SBFT_GV_LIB=$V/lib_probe_$h.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/${T}_${n}_$h.log 2>&1 || { tail -5 gpurun_out/${T}_${n}_$h.log; exit 1; }
  grep "half-probe-clk" gpurun_out/${T}_${n}_$h.log | tail -4 | grep "verify inputs\|helper" >> $out
done
done
for n in 1250 5000 10000; do
  for g in new q0 new q0; do
    if [ $g = new ]; then L=$PWD/smartbft_amd/libsbft_gpuverify.so; else L=$V/lib_$g.so; fi
    echo -n "$g " >> $out
    SBFT_GV_LIB=$L timeout -k 10 180 python -u tools/half_wide_sizes.py $n 40 >> $out 2> gpurun_out/${T}_${g}_$n.err || { tail -20 gpurun_out/${T}_${g}_$n.err; cat $out; exit 1; }
  done
done
cat $out
