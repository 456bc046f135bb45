#!/bin/bash
# SHA-256 variants A/B + the SHA tests on the default kernel + a traced streamed run
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sha or config5 or framed or fused" > gpurun_out/sha_tests.log 2>&1 || { tail -30 gpurun_out/sha_tests.log; exit 1; }
tail -2 gpurun_out/sha_tests.log
for v in 1 2 0; do SBFT_SHA_VARIANT=$v timeout -k 10 300 python tools/sha_ab.py >> gpurun_out/sha_ab.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/sha_ab.log
SBFT_STREAM_TRACE=1 timeout -k 10 300 python -c "
import sys; sys.argv=['x','8192']; exec(open('tools/stream_probe.py').read())" > gpurun_out/stream_trace.log 2>&1
grep -v amdgpu.ids gpurun_out/stream_trace.log | head -40; tail -2 gpurun_out/stream_trace.log
