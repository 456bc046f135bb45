#!/bin/bash
# Round 6 (re-entry): the whole GPU suite and smoke on HEAD (affine join), then the default bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 3000 gpurun_out/${T}_bench.log
