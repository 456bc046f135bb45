#!/bin/bash
# Round 5: the fixup-kernel fix on the GPU. First the torch-free child alone (init runs the
# power-on self-test, now with the exact fixup net; then every kernel on the golden vectors) --
# if the fix were wrong this is the one process that faults -- then the whole GPU suite, smoke.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tests/gpu_child_runtime.py > gpurun_out/r05b_child.log 2>&1
rc=$?; echo "== child rc=$rc"; grep -v amdgpu.ids gpurun_out/r05b_child.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -15 gpurun_out/r05b_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1
rc=$?; echo "== smoke rc=$rc"; tail -3 gpurun_out/r05b_smoke.log; exit $rc
