#!/bin/bash
# SHA-256 variants A/B, VALU issue rates, SHA tests, streamed pipeline probe
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/valu_rates > gpurun_out/valu_rates.log 2>&1 || exit $?
cat gpurun_out/valu_rates.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sha or config5 or framed or fused" > gpurun_out/sha_tests.log 2>&1 || { tail -30 gpurun_out/sha_tests.log; exit 1; }
tail -1 gpurun_out/sha_tests.log
for v in 2 3 4 1; do SBFT_SHA_VARIANT=$v timeout -k 10 300 python tools/sha_ab.py >> gpurun_out/sha_ab.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/sha_ab.log
timeout -k 10 300 python tools/stream_probe.py > gpurun_out/stream_probe.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stream_probe.log
