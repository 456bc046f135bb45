#!/bin/bash
# Full GPU suite, then the default bench line (all configs) and the rocprofv3 kernel summary.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -4 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 3000 gpurun_out/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-sha --no-latency --no-host-path --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*kernel_stats.csv" | head -3
