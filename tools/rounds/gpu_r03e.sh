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
cd $GRAFT_REPO_ROOT
# coalescer follow-up window A/B (SBFT_CS_FOLLOW_US: 50 = the round-2 behaviour, a full window
# for every batch) and the processCommits hook, same box, interleaved
for rep in 1 2; do
  for f in 50 12 0; do
    SBFT_CS_FOLLOW_US=$f timeout -k 10 120 tools/latency_harness quorum-gpu 66 400 66 50 > gpurun_out/cs_${f}_${rep}.txt 2>&1 || { cat gpurun_out/cs_${f}_${rep}.txt; exit 1; }
    echo "follow=$f $(cat gpurun_out/cs_${f}_${rep}.txt)" | tee -a gpurun_out/cs_ab.txt
  done
  timeout -k 10 120 tools/latency_harness quorum-hook 67 66 400 | tee -a gpurun_out/cs_ab.txt || exit 1
  timeout -k 10 120 tools/latency_harness quorum-cpu 66 400 16 | tee -a gpurun_out/cs_ab.txt || exit 1
done
