#!/bin/bash
# Round 4: the whole GPU suite on the new default (half kernel for batches <= 12,288), smoke,
# the half kernel's phase probe, config-4 hook (1 vs 2 batches in flight) and pipelined
# decisions (GPU vs OpenSSL), then the default bench line. Stops at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name" | tee -a gpurun_out/r04d.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/r04d_$name.log" 2>&1
    local rc=$?
    grep -v "^W2026\|^E2026\|amdgpu.ids" "gpurun_out/r04d_$name.log" | tail -4 | tee -a gpurun_out/r04d.log
    echo "rc=$rc" | tee -a gpurun_out/r04d.log
    return $rc
}
step tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
SBFT_GV_LIB=$PWD/tools/variants/lib_probe.so step probe 120 python tools/half_probe.py || exit $?
for r in 1 2; do
  step hook1_$r 120 tools/latency_harness quorum-hook 67 66 400 1 || exit $?
  step hook2_$r 120 tools/latency_harness quorum-hook 67 66 400 2 || exit $?
  step qcpu_$r 120 tools/latency_harness quorum-cpu 66 400 66 || exit $?
done
step pipe_gpu 180 tools/latency_harness quorum-pipe 2 300 gpu || exit $?
step pipe_cpu 180 tools/latency_harness quorum-pipe 2 300 cpu || exit $?
step pipe_gpu4 180 tools/latency_harness quorum-pipe 4 300 gpu || exit $?
step pipe_cpu4 180 tools/latency_harness quorum-pipe 4 300 cpu || exit $?
step bench 600 python bench.py || exit $?
echo "== done" | tee -a gpurun_out/r04d.log
