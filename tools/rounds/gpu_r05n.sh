#!/bin/bash
# Round 5: why the half kernel's table conversion is slow under a full batch in some builds:
# wait / LDS counters of lib_probe (slow conversion) and lib_probetab (fast conversion).
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/tools/variants
R=--kernel-include-regex=p256_verify_half_kernel
P1="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
for v in probe probetab; do
  n=1
  for P in "$P1" "$P2"; do
    SBFT_GV_LIB=$V/lib_$v.so timeout -s KILL 120 rocprofv3 $R --pmc $P -d gpurun_out/r05n_${v}_$n -o pmc --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05n_${v}_$n.log 2>&1 || { tail -5 gpurun_out/r05n_${v}_$n.log; exit 1; }
    n=$((n+1))
  done
done
find gpurun_out -path "*r05n_*" -name "pmc_counter_collection.csv" | sort
