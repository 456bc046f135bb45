#!/bin/bash
# Round 4: the half kernel's prescribed-u2 edge tests, init times (1 and 8 slots, concurrent
# self-tests), and the latency of the three verify kernels by batch size (half_max tuning).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04f_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04f_tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/init_probe.py > gpurun_out/r04f_init.log 2>&1 || { tail -5 gpurun_out/r04f_init.log; exit 1; }
tail -1 gpurun_out/r04f_init.log
timeout -k 10 600 python tools/pair_probe.py 1000 4096 8192 10000 12288 16384 24576 32768 49152 > gpurun_out/r04f_sizes.log 2>&1 || { tail -5 gpurun_out/r04f_sizes.log; exit 1; }
grep "'n'" gpurun_out/r04f_sizes.log
