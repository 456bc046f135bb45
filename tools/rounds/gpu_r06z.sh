#!/bin/bash
# Round 6: where VerifyProposal's payload copy spends its time inside the call (copy start / return
# from the call's start, SBFT_VP_TRACE), beside the parse and with the copy first (SBFT_VP_COPY_FIRST=1,
# diagnostics), generic and registered; the h2d_pinned diagnostic's standalone pageable copy beside it.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06z
out=gpurun_out/$T.txt; : > $out
for rep in 1 2; do
for mode in "0 0" "0 1" "1 0"; do
  set -- $mode
  echo "== registered=$1 copy_first=$2" >> $out
  SBFT_VP_COPY_FIRST=$2 timeout -k 10 300 tools/latency_harness proposal-phases 10000 200 $1 >> $out 2> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; cat $out; exit 1; }
done
done
timeout -k 10 120 tools/h2d_pinned >> $out 2>&1 || true
cat $out
