#!/bin/bash
# Round 4: the self-test with step tracing, then the r04a steps (tests, latency A/B, trace).
mkdir -p gpurun_out
export TMPDIR=/tmp
SBFT_POST_TRACE=1 AMD_LOG_LEVEL=1 timeout -k 10 120 python -c "
from smartbft_amd import GpuVerifier
g = GpuVerifier(device_mask=1); print('init ok'); g.close()
g = GpuVerifier(); print('init ok (all devices)'); g.close()" > gpurun_out/r04c_init.log 2>&1
rc=$?; grep -v "^W2026\|amdgpu.ids" gpurun_out/r04c_init.log | tail -15; [ $rc -ne 0 ] && exit $rc
bash tools/rounds/gpu_r04a.sh
