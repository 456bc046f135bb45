#!/bin/bash
# Round 6, last library build (split-path trace added): the whole GPU suite and smoke.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06ah
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
