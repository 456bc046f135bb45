#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/vp_trace -o run --output-format csv -- python3 tools/latency_probe.py --calls 20 > gpurun_out/vp_trace.log 2>&1 || { tail -5 gpurun_out/vp_trace.log; exit 1; }
python3 tools/vp_timeline.py gpurun_out/vp_trace | tee gpurun_out/vp_timeline.txt | tail -40
