#!/bin/bash
# SHA-256 kernel variants: parity tests + A/B timing at config-5 size
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/sha_ceiling > gpurun_out/sha_ceiling.log 2>&1 && cat gpurun_out/sha_ceiling.log || exit 1
for v in 5 6 7 2; do
  SBFT_SHA_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sha or config5 or fused or framed" > gpurun_out/sha_tests_$v.log 2>&1 || { echo "variant $v"; tail -30 gpurun_out/sha_tests_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/sha_tests_$v.log)"
  SBFT_SHA_VARIANT=$v timeout -k 10 300 python tools/sha_ab.py >> gpurun_out/sha_ab2.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/sha_ab2.log
