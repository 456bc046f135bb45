#!/bin/bash
# Round 5: instruction-cache counters of the half kernel (is its code streaming from L2?).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r05m_avail.txt 2>&1
grep -o "SQC_[A-Z_0-9]*" gpurun_out/r05m_avail.txt | sort -u | head -60
R=--kernel-include-regex=p256_verify_half_kernel
timeout -s KILL 120 rocprofv3 $R --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    -d gpurun_out/r05m_pmc_ic -o pmc --output-format csv -- python3 tools/half_probe.py > gpurun_out/r05m_pmc_ic.log 2>&1 || { tail -5 gpurun_out/r05m_pmc_ic.log; exit 1; }
find gpurun_out/r05m_pmc_ic -name "*.csv"
