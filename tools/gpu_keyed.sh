#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/keyed_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/keyed_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/keyed_probe.py > gpurun_out/keyed_probe.log 2>&1; rc=$?; tail -3 gpurun_out/keyed_probe.log; exit $rc
