#!/bin/bash
# Round 6: the helper's curve check in radix 2^29 before barrier 1 (h2), + even-lane-only hash (h3),
# against h1 (8 x 32 check after barrier 1) and HEAD (h0): half suites on the new default build,
# then phase probes (cycles) at 1,250 and 5,000 (wide) and 10,000 (four-lane), interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
T=r06t
out=gpurun_out/$T.txt; : > $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_exceptional.py tests/test_gpu_configs.py tests/test_gpu_fixup.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log >> $out
for n in 1250 5000 10000; do
for h in h0 h1 h2 h3 h0 h2; do
  w=1; [ $n = 10000 ] && w=0
  echo "== n=$n $h" >> $out
  HALF_PROBE_N=$n HALF_PROBE_WIDE=$w SBFT_GV_LIB=$V/lib_probe_$h.so timeout -k 10 120 python tools/half_probe.py > gpurun_out/${T}_${n}_$h.log 2>&1 || { tail -5 gpurun_out/${T}_${n}_$h.log; exit 1; }
  grep "half-probe" gpurun_out/${T}_${n}_$h.log | tail -8 | grep "verify inputs\|helper" >> $out
done
done
cat $out
