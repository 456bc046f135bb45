#!/bin/bash
# Round 5: the whole GPU suite and smoke on the final tree (after the keyed lanes kernel's Z^2/Z^3 change).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ar_tests.log 2>&1 || { tail -15 gpurun_out/r05ar_tests.log; exit 1; }
tail -1 gpurun_out/r05ar_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ar_smoke.log 2>&1 || { tail -5 gpurun_out/r05ar_smoke.log; exit 1; }
tail -1 gpurun_out/r05ar_smoke.log
