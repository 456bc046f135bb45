#!/bin/bash
# Stop at the first failing size; every run is its own process with its own time limit.
mkdir -p gpurun_out
for n in 1024 16384 65280 65536 66000 131072 417664; do
  SBFT_GV_LIB=$PWD/tools/variants/lib_debug.so timeout -k 10 120 python tools/diag_sizes.py $n > gpurun_out/diag_$n.log 2>&1
  rc=$?
  grep -v "^W2026\|^E2026\|amdgpu.ids" gpurun_out/diag_$n.log | tail -8
  if [ $rc -ne 0 ]; then echo "size $n failed rc=$rc: stopping"; exit $rc; fi
done
