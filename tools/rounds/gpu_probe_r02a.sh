mkdir -p gpurun_out
timeout -k 10 300 python tools/stream_probe.py > gpurun_out/stream_probe.log 2>&1 || exit $?
for w in 50 150 300 600; do timeout -k 10 120 tools/latency_harness quorum-gpu 66 200 66 $w >> gpurun_out/quorum_sweep.log 2>&1 || exit $?; done
timeout -k 10 120 tools/latency_harness quorum-gpu 66 200 0 0 >> gpurun_out/quorum_sweep.log 2>&1
cat gpurun_out/stream_probe.log gpurun_out/quorum_sweep.log | grep -v amdgpu.ids
