#!/bin/bash
# Round 6: where a split VerifyProposal's ~50 us over one share goes: SBFT_VP_TRACE share pick-up /
# end times (tools/split_trace_summary.py) for 2,500 requests over 2 slots and 1,250 on one slot.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r06ag
out=gpurun_out/$T.txt; : > $out
SBFT_VP_TRACE=1 timeout -k 10 300 python -u tools/split_probe.py 2500 2 100 >> $out 2> gpurun_out/${T}_trace.err || { tail -10 gpurun_out/${T}_trace.err; cat $out; exit 1; }
python tools/split_trace_summary.py gpurun_out/${T}_trace.err >> $out
cat $out
