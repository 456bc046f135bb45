#!/bin/bash
# Where the config-3 latency kernel's wave-cycles go: SQ stall buckets (one pass), then the
# instruction-cache counters (a pass of their own), over 4 VerifyProposal calls of 10k requests.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=--kernel-include-regex=p256_verify_half_kernel
timeout -s KILL 120 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    -d gpurun_out/r04y_sq -o pmc --output-format csv -- python3 tools/half_probe.py > gpurun_out/r04y_sq.log 2>&1 || { tail -5 gpurun_out/r04y_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 $R --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
    -d gpurun_out/r04y_ic -o pmc --output-format csv -- python3 tools/half_probe.py > gpurun_out/r04y_ic.log 2>&1 || { tail -5 gpurun_out/r04y_ic.log; exit 1; }
find gpurun_out/r04y_sq gpurun_out/r04y_ic -name "*counter_collection.csv" | sort
